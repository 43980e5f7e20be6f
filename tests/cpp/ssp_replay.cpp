// ssp_replay.cpp — BASELINE config 5 / SURVEY §8f-1: an LR-pattern push/pull
// trace replayed through the consistency models over S range shards, once with
// the CPU oracle storage (oracle/liboracle.so, the MapStorage restatement) and
// once with HipStorage<double> (HBM shards, HIP kernels), comparing EVERY Get
// reply and the final shard contents bit for bit.
//
// The trace restates the worker loop of app/logistic_regression.cpp:309-503:
//   per iteration: _kvs cache reset (:332); per sample b: keys = [0] + sorted
//   feature ids (:377-382); Get the keys not cached yet (:411-420); predict,
//   gradient, update every pulled value (:443-463); Add(keys, vals) (:490);
//   Clock after the batch (:503).  Val = double (:154).
// The worker side restates KVClientTable (worker/kv_client_table.hpp:47-146):
// range slicing, one message per server, Get replies merged into a std::map and
// returned in key order.  Messages are processed by a deterministic
// single-threaded scheduler: round-robin over workers, every message handled by
// its server's model at once (FIFO per server); an SSP-released request
// (ssp_model.cpp:18-22 pushes the REQUEST to the reply queue) is routed by its
// recver back to the server and served there.  Because both runs
// use the same models and scheduler, any difference comes from the storages.
//
// usage: ssp_replay [--model ssp|bsp|asp] [--workers W] [--shards S] [--iters I]
//                   [--batch B] [--staleness T] [--skew K] [--cpu-only] [--known-answers]
//                   [--partition range|hash] [--trace FILE]
// --trace FILE (not with --threads) writes the second run's model traffic: every
// message handed to a server's model, the replies that handling pushed, and
// every shard's final contents, so oracle/consistency_ref.py -- a restatement of
// the reference models independent of include/ps/consistency.hpp -- can replay
// the same arrivals and check each reply (tests/test_replay.py).
// --partition hash slices with the reference Engine's DEFAULT partitioner, the
// jump consistent hash (base/consistent_hashing_partition_manager.hpp; the LR
// app's own configuration, driver/engine.hpp:143-150): every shard then owns
// the whole feature range [0, n_features).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ps/callback_runner.hpp"
#include "ps/consistency.hpp"
#include "ps/hip_storage.hpp"
#include "ps/consistent_hashing_partition_manager.hpp"
#include "ps/range_partition_manager.hpp"
#include "ps/server_thread.hpp"
#include "ps/storage_factory.hpp"

using namespace csci5570;

extern "C" {  // oracle/liboracle.so — the checker (test infrastructure)
void* oracle_create(int kind, int dtype);
void oracle_destroy(void* h);
void oracle_add(void* h, const uint32_t* keys, const void* vals, uint64_t n);
void oracle_get(void* h, const uint32_t* keys, uint64_t n, void* out);
}

namespace {

template <typename Val>
struct OracleDtype;
template <>
struct OracleDtype<int> {
  static constexpr int value = 0;
};
template <>
struct OracleDtype<double> {
  static constexpr int value = 2;
};

// The oracle's MapStorage restatement behind the reference plugin interface.
template <typename Val>
class OracleStorage : public AbstractStorage {
 public:
  OracleStorage() : h_(oracle_create(0, OracleDtype<Val>::value)) {}
  ~OracleStorage() override { oracle_destroy(h_); }
  void SubAdd(const third_party::SArray<Key>& keys, const third_party::SArray<char>& vals) override {
    auto v = third_party::SArray<Val>(vals);
    PS_CHECK(keys.size() == v.size());
    oracle_add(h_, keys.data(), v.data(), keys.size());
  }
  third_party::SArray<char> SubGet(const third_party::SArray<Key>& keys) override {
    third_party::SArray<Val> out(keys.size());
    oracle_get(h_, keys.data(), keys.size(), out.data());
    return third_party::SArray<char>(out);
  }
  void FinishIter() override {}

 private:
  void* h_;
};

struct Rng {  // splitmix64
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

struct Sample {
  std::vector<uint32_t> idx;  // sorted, unique, >= 1 (Eigen SparseVector inner order)
  std::vector<double> val;
  int label;
};

struct Config {
  std::string model = "ssp";
  int workers = 4, shards = 8, iters = 6, batch = 30, staleness = 3, pool = 48, skew = 2;
  uint32_t n_features = 1000000;
  uint64_t seed = 2026;
  bool cpu_only = false;
  bool bsp_ungrouped = false;
  bool threads = false;  // one ServerThread per shard (concurrent HipStorage use)
  bool frames = false;   // payloads delivered in page-locked frames (HipStorage runs only)
  std::string partition = "range";  // range | hash
  std::string trace;                // model traffic of the second run (--trace)
};

// Trace records (little-endian): 'I' (a message handed to server s's model) and
// 'O' (a message that handling pushed to the reply queue) carry
//   u8 kind, i32 server, i8 flag, i32 sender, i32 recver, i32 model_id,
//   u32 ndata, ndata x (u64 bytes, bytes);
// 'F' (server s's final contents, every key of its range in order) carries
//   u8 kind, i32 server, u64 n, n x f64.
class TraceWriter {
 public:
  explicit TraceWriter(const std::string& path) : f_(std::fopen(path.c_str(), "wb")) {
    if (!f_) throw std::runtime_error("cannot open trace file " + path);
  }
  ~TraceWriter() { std::fclose(f_); }
  void message(char kind, int server, const Message& m) {
    put(kind);
    put((int32_t)server);
    put((int8_t)m.meta.flag);
    put((int32_t)m.meta.sender);
    put((int32_t)m.meta.recver);
    put((int32_t)m.meta.model_id);
    put((uint32_t)m.data.size());
    for (const auto& d : m.data) {
      put((uint64_t)d.size());
      if (d.size()) std::fwrite(d.data(), 1, d.size(), f_);
    }
  }
  void final_vals(int server, const std::vector<double>& v) {
    put('F');
    put((int32_t)server);
    put((uint64_t)v.size());
    if (!v.empty()) std::fwrite(v.data(), sizeof(double), v.size(), f_);
  }

 private:
  template <typename T>
  void put(T x) {
    std::fwrite(&x, sizeof(T), 1, f_);
  }
  std::FILE* f_;
};

struct ReplyRecord {
  int server, worker;
  std::vector<uint32_t> keys;
  std::vector<double> vals;
};

struct Run {
  std::vector<ReplyRecord> log;
  std::vector<std::vector<double>> final_vals;  // per server, every key of its range
  uint64_t msgs = 0, adds = 0, gets = 0, clocks = 0, echoes = 0;
  double seconds = 0;
};

class Replay {
 public:
  Replay(const Config& c, bool hip, TraceWriter* trace = nullptr) : c_(c), hip_(hip), trace_(trace) {
    const uint64_t step = c.n_features / c.shards;
    const bool hashed = c.partition == "hash";
    for (int s = 0; s < c.shards; ++s) {
      const uint64_t lo = s * step, hi = s + 1 == c.shards ? c.n_features : (s + 1) * step;
      ranges_.push_back(hashed ? std::make_pair((uint64_t)0, (uint64_t)c.n_features) : std::make_pair(lo, hi));
      ids_.push_back((uint32_t)s);
    }
    if (hashed)
      map_.reset(new ConsistentHashShardMap(ids_));
    else
      map_.reset(new RangeShardMap(ids_, ranges_));
    int ndev = pskv_device_count();
    if (c.threads) {
      // Engine::CreateTable (driver/engine.hpp:93-131) through the restated
      // factory: one ServerThread, storage and model per range
      for (int s = 0; s < c.shards; ++s) threads_.emplace_back(new ServerThread((uint32_t)s));
      const ModelType mt = c.model == "ssp" ? ModelType::SSP : c.model == "bsp" ? ModelType::BSP : ModelType::ASP;
      storages_ = CreateTable<double>(
          threads_, ranges_, 0, mt, hip ? StorageType::Hip : StorageType::Map, c.staleness, &replies_,
          PSKV_ASSIGN, [](StorageType) { return std::unique_ptr<AbstractStorage>(new OracleStorage<double>()); });
      for (auto& t : threads_) {
        if (auto* bsp = dynamic_cast<BSPModel*>(t->GetModel(0))) bsp->SetGroupedFlush(!c.bsp_ungrouped);
        t->SetOnProcessed([this] {
          std::lock_guard<std::mutex> lk(qm_);
          if (--inflight_ == 0) quiet_.notify_all();
        });
      }
    }
    for (int s = 0; s < c.shards && !c.threads; ++s) {
      std::unique_ptr<AbstractStorage> st;
      if (hip)
        st.reset(new HipStorage<double>(s % (ndev > 0 ? ndev : 1), (uint32_t)ranges_[s].first,
                                        ranges_[s].second));
      else
        st.reset(new OracleStorage<double>());
      storages_.push_back(st.get());
      std::unique_ptr<AbstractModel> md;
      if (c.model == "ssp") {
        md.reset(new SSPModel(0, std::move(st), c.staleness, &replies_));
      } else if (c.model == "bsp") {
        auto* m = new BSPModel(0, std::move(st), &replies_);
        m->SetGroupedFlush(!c.bsp_ungrouped);
        md.reset(m);
      } else {
        md.reset(new ASPModel(0, std::move(st), &replies_));
      }
      models_.push_back(std::move(md));
    }
    server_q_.resize(c.shards);
    for (auto& t : threads_) t->Start();
    // samples: feature popularity is skewed (idx ~ n * u^3) so workers collide on keys
    for (int w = 0; w < c.workers; ++w) {
      Rng r(c.seed * 1000003ull + (uint64_t)w);
      std::vector<Sample> pool;
      for (int p = 0; p < c.pool; ++p) {
        Sample smp;
        const int nf = 4 + (int)(r.next() % 21);
        std::map<uint32_t, double> f;
        while ((int)f.size() < nf) {
          const double u = r.uni();
          const uint32_t i = 1 + (uint32_t)((c.n_features - 1) * u * u * u);
          f[i] = 0.05 + r.uni();
        }
        for (auto& kv : f) {
          smp.idx.push_back(kv.first);
          smp.val.push_back(kv.second);
        }
        smp.label = (int)(r.next() & 1);
        pool.push_back(smp);
      }
      pools_.push_back(pool);
      Worker wk;
      wk.tid = 100 + w;
      wk.rng = Rng(c.seed + 77 * (uint64_t)w);
      workers_.push_back(wk);
    }
  }

  Run run() {
    const auto t0 = std::chrono::steady_clock::now();
    // kResetWorkerInModel to every server (Engine::InitTable, driver/engine.cpp:169-213)
    std::vector<uint32_t> tids;
    for (auto& w : workers_) tids.push_back((uint32_t)w.tid);
    for (int s = 0; s < c_.shards; ++s) {
      Message m;
      m.meta.flag = Flag::kResetWorkerInModel;
      m.meta.sender = 9999;
      m.meta.recver = s;
      m.meta.model_id = 0;
      m.AddData(third_party::SArray<uint32_t>(tids));
      deliver(m);
    }
    pump();
    for (;;) {
      bool all_done = true, progressed = false;
      // worker w takes 1 + w*skew operations per round: fast workers run ahead
      // of the straggler until staleness (SSP) or the barrier (BSP) holds them
      for (size_t wi = 0; wi < workers_.size(); ++wi) {
        Worker& w = workers_[wi];
        for (int op = 0; op <= (int)wi * c_.skew; ++op) {
          if (w.done) break;
          all_done = false;
          if (w.outstanding > 0) break;
          step(w);
          progressed = true;
          pump();
        }
      }
      if (all_done) break;
      if (!progressed) throw std::runtime_error("replay deadlock: every worker waits on a reply");
    }
    for (auto& t : threads_) t->Stop();  // kExit; the storages stay alive in their models
    // final contents of every shard, read through the plugin interface
    for (int s = 0; s < c_.shards; ++s) {
      std::vector<uint32_t> ks;
      for (uint64_t k = ranges_[s].first; k < ranges_[s].second; ++k) ks.push_back((uint32_t)k);
      third_party::SArray<Key> keys(ks);
      auto v = third_party::SArray<double>(storages_[s]->SubGet(keys));
      out_.final_vals.emplace_back(v.begin(), v.end());
      if (trace_) trace_->final_vals(s, out_.final_vals.back());
      storages_[s]->FinishIter();
    }
    out_.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return out_;
  }

 private:
  struct Worker {
    int tid = 0, iter = 0, b = 0;
    bool done = false, in_batch = false, have_vals = false;
    int outstanding = 0;
    std::vector<unsigned> order;
    std::map<Key, double> kvs;     // _kvs (logistic_regression.cpp:332)
    std::map<Key, double> reply;   // KVClientTable::Get's std::map (kv_client_table.hpp:112)
    std::vector<Key> keys_;        // the keys of the outstanding Get
    Rng rng{0};
  };

  void deliver(const Message& in) {
    ++out_.msgs;
    Message m = in;
    if (c_.frames && hip_) {
      // the mailbox after SURVEY §8f-3: every data frame received into a
      // page-locked frame (comm/mailbox.cpp:246-257)
      for (auto& d : m.data) d = RecvIntoFrame(d.data(), d.size());
    }
    if (c_.threads) {
      {
        std::lock_guard<std::mutex> lk(qm_);
        ++inflight_;
      }
      threads_[m.meta.recver]->GetWorkQueue()->Push(m);
    } else {
      server_q_[m.meta.recver].push(m);
    }
  }

  // Threaded mode: wait until every server thread is idle, then route the
  // replies of that window ordered by server (each server's replies keep
  // their FIFO order), so the run is deterministic.
  void pump_threads() {
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(qm_);
        quiet_.wait(lk, [&] { return inflight_ == 0; });
      }
      std::vector<Message> window;
      Message r;
      while (replies_.Pop(&r)) window.push_back(r);
      if (window.empty()) return;
      std::stable_sort(window.begin(), window.end(), [](const Message& a, const Message& b) {
        const int sa = a.data.size() == 1 ? a.meta.recver : a.meta.sender;
        const int sb = b.data.size() == 1 ? b.meta.recver : b.meta.sender;
        return sa < sb;
      });
      // route the window itself: echoes delivered now are served concurrently
      // and their replies land in the NEXT window
      for (auto& m : window) route_one(m);
    }
  }

  // Process every queued server message and route every reply, until quiet.
  void pump() {
    if (c_.threads) return pump_threads();
    for (;;) {
      bool any = false;
      for (int s = 0; s < c_.shards; ++s) {
        while (!server_q_[s].empty()) {
          Message m = server_q_[s].front();
          server_q_[s].pop();
          any = true;
          AbstractModel* md = models_[s].get();
          if (trace_) trace_->message('I', s, m);
          switch (m.meta.flag) {  // server/server_thread.cpp:29-46
            case Flag::kClock: md->Clock(m); break;
            case Flag::kAdd: md->Add(m); break;
            case Flag::kGet: md->Get(m); break;
            case Flag::kResetWorkerInModel: md->ResetWorker(m); break;
            default: break;
          }
          route(s);
        }
      }
      if (!any) break;
    }
  }

  void route(int server) {
    Message r;
    while (replies_.Pop(&r)) {
      if (trace_) trace_->message('O', server, r);
      route_one(r);
    }
  }

  void route_one(const Message& r) {
    if (r.meta.flag == Flag::kGet && r.data.size() == 1) {  // SSP-released request: back to its server
      ++out_.echoes;
      deliver(r);
      return;
    }
    if (r.meta.flag != Flag::kGet) return;  // reset acknowledgements
    Worker& w = workers_[r.meta.recver - 100];
    auto k = third_party::SArray<Key>(r.data[0]);
    auto v = third_party::SArray<double>(r.data[1]);
    ReplyRecord rec{r.meta.sender, r.meta.recver, std::vector<uint32_t>(k.begin(), k.end()),
                    std::vector<double>(v.begin(), v.end())};
    out_.log.push_back(rec);
    for (size_t i = 0; i < k.size(); ++i) w.reply.insert(std::make_pair(k[i], v[i]));
    if (--w.outstanding == 0) finish_get(w);
  }

  void send_get(Worker& w, const std::vector<Key>& keys) {  // kv_client_table.hpp:107-139
    ++out_.gets;
    std::vector<std::pair<int, AbstractPartitionManager::Keys>> sl;
    map_->Slice(third_party::SArray<Key>(keys), &sl);
    w.reply.clear();
    w.keys_ = keys;
    w.outstanding = (int)sl.size();
    for (auto& s : sl) {
      Message m;
      m.meta.sender = w.tid;
      m.meta.recver = s.first;
      m.meta.model_id = 0;
      m.meta.flag = Flag::kGet;
      m.AddData(s.second);
      deliver(m);
    }
  }

  void finish_get(Worker& w) {  // values in map order (kv_client_table.hpp:144-145), cached in _kvs
    size_t i = 0;
    for (auto& kv : w.reply) {
      PS_CHECK(i < w.keys_.size());
      w.kvs[w.keys_[i++]] = kv.second;
    }
    w.have_vals = true;
  }

  void send_add(Worker& w, const std::vector<Key>& keys, const std::vector<double>& vals) {
    ++out_.adds;  // kv_client_table.hpp:78-105 (double -> Val is exact for Val = double)
    // the KV form of Slice (values as double, abstract_partition_manager.hpp:21-22)
    std::vector<std::pair<int, AbstractPartitionManager::KVPairs>> sl;
    map_->Slice(std::make_pair(third_party::SArray<Key>(keys), third_party::SArray<double>(vals)), &sl);
    for (auto& s : sl) {
      Message m;
      m.meta.sender = w.tid;
      m.meta.recver = s.first;
      m.meta.model_id = 0;
      m.meta.flag = Flag::kAdd;
      m.AddData(s.second.first);
      m.AddData(s.second.second);
      deliver(m);
    }
  }

  void send_clock(Worker& w) {  // kv_client_table.hpp:47-60
    ++out_.clocks;
    for (int s = 0; s < c_.shards; ++s) {
      Message m;
      m.meta.sender = w.tid;
      m.meta.recver = s;
      m.meta.model_id = 0;
      m.meta.flag = Flag::kClock;
      deliver(m);
    }
  }

  // One operation of the worker loop (logistic_regression.cpp:309-503).
  void step(Worker& w) {
    const auto& pool = pools_[w.tid - 100];
    if (!w.in_batch) {
      if (w.iter == c_.iters) {
        w.done = true;
        return;
      }
      w.kvs.clear();
      w.order.resize(pool.size());
      for (unsigned i = 0; i < w.order.size(); ++i) w.order[i] = i;
      for (size_t i = w.order.size(); i > 1; --i) std::swap(w.order[i - 1], w.order[w.rng.next() % i]);
      w.b = 0;
      w.in_batch = true;
      w.have_vals = false;
    }
    if (w.b == c_.batch) {
      send_clock(w);
      w.in_batch = false;
      ++w.iter;
      return;
    }
    const Sample& smp = pool[w.order[w.b % pool.size()]];
    std::vector<Key> keys{0};
    keys.insert(keys.end(), smp.idx.begin(), smp.idx.end());
    if (!w.have_vals) {
      std::vector<Key> missing;
      for (Key k : keys)
        if (!w.kvs.count(k)) missing.push_back(k);
      w.have_vals = true;
      if (!missing.empty()) {
        send_get(w, missing);  // blocks the worker until every slice is answered
        return;
      }
    }
    std::vector<double> vals;
    for (Key k : keys) vals.push_back(w.kvs[k]);
    double yhat = vals.at(0);
    for (size_t i = 1; i < keys.size(); ++i) yhat += vals[i] * smp.val[i - 1];
    const double predict = 1.0 / (1.0 + std::exp(-yhat));
    const double error = (smp.label > 0 ? 1 : 0) - predict;
    double gradient = vals.at(0);
    for (double x : smp.val) gradient += x * error;
    const double lr = 0.01;
    for (double& v : vals) v += lr * gradient;
    send_add(w, keys, vals);
    w.have_vals = false;
    ++w.b;
  }

  Config c_;
  bool hip_;
  TraceWriter* trace_;
  std::vector<std::pair<uint64_t, uint64_t>> ranges_;
  std::vector<uint32_t> ids_;
  std::unique_ptr<AbstractPartitionManager> map_;
  std::vector<AbstractStorage*> storages_;
  std::vector<std::unique_ptr<AbstractModel>> models_;
  std::vector<std::unique_ptr<ServerThread>> threads_;
  std::mutex qm_;
  std::condition_variable quiet_;
  int64_t inflight_ = 0;
  std::vector<std::queue<Message>> server_q_;
  ReplyQueue replies_;
  std::vector<std::vector<Sample>> pools_;
  std::vector<Worker> workers_;
  Run out_;
};

bool same(const Run& a, const Run& b, std::string* why) {
  if (a.log.size() != b.log.size()) {
    *why = "reply count " + std::to_string(a.log.size()) + " vs " + std::to_string(b.log.size());
    return false;
  }
  for (size_t i = 0; i < a.log.size(); ++i) {
    const auto &x = a.log[i], &y = b.log[i];
    if (x.server != y.server || x.worker != y.worker || x.keys != y.keys ||
        x.vals.size() != y.vals.size() ||
        std::memcmp(x.vals.data(), y.vals.data(), x.vals.size() * sizeof(double)) != 0) {
      *why = "reply " + std::to_string(i) + " differs";
      return false;
    }
  }
  for (size_t s = 0; s < a.final_vals.size(); ++s)
    if (a.final_vals[s].size() != b.final_vals[s].size() ||
        std::memcmp(a.final_vals[s].data(), b.final_vals[s].data(),
                    a.final_vals[s].size() * sizeof(double)) != 0) {
      *why = "final contents of server " + std::to_string(s) + " differ";
      return false;
    }
  return true;
}

// The reference model tests (server/consistency/*_model_test.cpp) over a storage,
// and its server/util tests (ProgressTracker, PendingBuffer).  Each case prints
// "case <name>: ok" — the names of tests/golden/reference_known_answers.json's
// model_cases / util_cases, which tests/test_replay.py checks are all present.
template <typename MakeStorage>
int known_answers(MakeStorage make, const char* label) {
  int fails = 0, case_fails = 0;
  auto expect = [&](bool c, const char* what) {
    if (!c) {
      ++fails;
      ++case_fails;
      std::printf("  FAIL [%s] %s\n", label, what);
    }
  };
  auto done = [&](const char* name) {
    std::printf("[%s] case %s: %s\n", label, name, case_fails ? "FAIL" : "ok");
    case_fails = 0;
  };
  auto msg = [](Flag f, int sender, std::vector<int> keys, std::vector<int> vals) {
    Message m;
    m.meta.flag = f;
    m.meta.model_id = 0;
    m.meta.sender = sender;
    m.meta.recver = 0;
    if (!keys.empty()) m.AddData(third_party::SArray<int>(keys));
    if (!vals.empty()) m.AddData(third_party::SArray<int>(vals));
    return m;
  };
  auto reset = [&](AbstractModel* md, ReplyQueue& q) {
    Message r;
    r.AddData(third_party::SArray<uint32_t>({2, 3}));
    md->ResetWorker(r);
    Message ack;
    expect(q.Pop(&ack) && ack.meta.flag == Flag::kResetWorkerInModel, "reset reply");
  };
  {  // ssp_model_test.cpp:29-117 CheckGetAndAdd
    ReplyQueue q;
    SSPModel md(0, make(), 1, &q);
    reset(&md, q);
    Message m3 = msg(Flag::kAdd, 2, {0}, {1}), m4 = msg(Flag::kAdd, 3, {1}, {2});
    Message m5 = msg(Flag::kGet, 2, {0}, {}), m6 = msg(Flag::kGet, 3, {1}, {});
    md.Add(m3);
    md.Add(m4);
    md.Get(m5);
    md.Get(m6);
    expect(q.Size() == 2, "ssp: two replies");
    Message r;
    q.Pop(&r);
    expect(third_party::SArray<int>(r.data[1])[0] == 1 && r.meta.sender == 0 && r.meta.recver == 2,
           "ssp: key 0 -> 1 to worker 2");
    q.Pop(&r);
    expect(third_party::SArray<int>(r.data[1])[0] == 2 && r.meta.recver == 3, "ssp: key 1 -> 2 to worker 3");
    done("SSP CheckGetAndAdd");
  }
  {  // ssp_model_test.cpp:161-251 CheckStaleness
    ReplyQueue q;
    SSPModel md(0, make(), 2, &q);
    reset(&md, q);
    Message m1 = msg(Flag::kGet, 2, {0}, {});
    md.Get(m1);
    Message junk;
    q.Pop(&junk);
    Message c = msg(Flag::kClock, 2, {}, {});
    md.Clock(c);
    Message a = msg(Flag::kAdd, 2, {0}, {1});
    md.Add(a);
    md.Clock(c);
    md.Clock(c);
    Message g = msg(Flag::kGet, 2, {0}, {});
    md.Get(g);
    expect(md.GetPendingSize(1) == 1, "ssp staleness: buffered at 1");
    Message c3 = msg(Flag::kClock, 3, {}, {});
    md.Clock(c3);
    Message g2 = msg(Flag::kGet, 2, {0}, {});
    md.Get(g2);
    expect(md.GetPendingSize(1) == 0, "ssp staleness: released");
    done("SSP CheckStaleness");
  }
  {  // bsp_model_test.cpp:29-130 CheckGetAndAdd
    ReplyQueue q;
    BSPModel md(0, make(), &q);
    reset(&md, q);
    Message m0 = msg(Flag::kGet, 2, {1}, {});
    md.Get(m0);
    Message r;
    expect(q.Pop(&r), "bsp: first get served");
    Message m1 = msg(Flag::kAdd, 2, {1}, {100}), m2 = msg(Flag::kClock, 2, {}, {});
    md.Add(m1);
    md.Clock(m2);
    expect(md.GetAddPendingSize() == 1, "bsp: add deferred");
    Message cm1 = msg(Flag::kGet, 3, {1}, {});
    md.Get(cm1);
    expect(q.Pop(&r) && third_party::SArray<int>(r.data[1])[0] == 0, "bsp: 0 before the clock");
    Message m3 = msg(Flag::kClock, 3, {}, {});
    md.Clock(m3);
    expect(md.GetAddPendingSize() == 0, "bsp: adds applied");
    Message cm2 = msg(Flag::kGet, 3, {1}, {});
    md.Get(cm2);
    expect(q.Pop(&r) && third_party::SArray<int>(r.data[1])[0] == 100, "bsp: 100 after the clock");
    done("BSP CheckGetAndAdd");
  }
  {  // restatement choice (tests/golden restatement_cases): a Get
     // still ahead after a min-clock advance is buffered again and answered at
     // the next advance (bsp_model.cpp:27-30 would drop it)
    ReplyQueue q;
    BSPModel md(0, make(), &q);
    reset(&md, q);
    Message c2 = msg(Flag::kClock, 2, {}, {}), c3 = msg(Flag::kClock, 3, {}, {});
    md.Clock(c2);
    md.Clock(c2);
    Message a = msg(Flag::kAdd, 2, {1}, {7}), g = msg(Flag::kGet, 2, {1}, {});
    md.Add(a);
    md.Get(g);
    expect(md.GetGetPendingSize() == 1 && q.Size() == 0, "bsp ahead: get buffered");
    md.Clock(c3);
    expect(md.GetAddPendingSize() == 0, "bsp ahead: add flushed at the advance");
    expect(md.GetGetPendingSize() == 1 && q.Size() == 0, "bsp ahead: still ahead, buffered again");
    md.Clock(c3);
    expect(md.GetGetPendingSize() == 0, "bsp ahead: released at the next advance");
    Message r;
    expect(q.Pop(&r) && r.meta.recver == 2 && third_party::SArray<int>(r.data[0])[0] == 1 &&
               third_party::SArray<int>(r.data[1])[0] == 7,
           "bsp ahead: answered with the flushed value");
    done("BSP Get two clocks ahead is re-buffered");
  }
  {  // asp_model_test.cpp:33-179 CheckGetAndAdd: Gets served at once, in order
     // with the Adds; Clock a no-op
    ReplyQueue q;
    ASPModel md(0, make(), &q);
    reset(&md, q);
    auto reply = [&](int recver, int key, int val, const char* what) {
      Message r;
      const bool got = q.Pop(&r);
      expect(got && r.meta.flag == Flag::kGet && r.meta.sender == 0 && r.meta.recver == recver &&
                 r.data.size() == 2 && third_party::SArray<int>(r.data[0]).size() == 1 &&
                 third_party::SArray<int>(r.data[0])[0] == key && third_party::SArray<int>(r.data[1])[0] == val,
             what);
    };
    Message g0 = msg(Flag::kGet, 2, {0}, {}), g1 = msg(Flag::kGet, 3, {1}, {});
    md.Get(g0);
    md.Get(g1);
    reply(2, 0, 0, "asp: key 0 -> 0 to worker 2");
    reply(3, 1, 0, "asp: key 1 -> 0 to worker 3");
    Message g2 = msg(Flag::kGet, 3, {1}, {}), a2 = msg(Flag::kAdd, 2, {1}, {1});
    md.Get(g2);
    md.Add(a2);
    expect(q.Size() == 1, "asp: the Get is not blocked");
    reply(3, 1, 0, "asp: the Get before the Add reads 0");
    Message g3 = msg(Flag::kGet, 2, {1}, {});
    md.Clock(g3);
    md.Get(g3);
    expect(q.Size() == 1, "asp: clock then get");
    reply(2, 1, 1, "asp: key 1 -> 1 after the Add");
    Message a3 = msg(Flag::kAdd, 3, {0}, {1});
    md.Add(a3);
    md.Clock(a3);
    Message g4 = msg(Flag::kGet, 3, {0}, {});
    md.Get(g4);
    expect(q.Size() == 1, "asp: add, clock, get");
    reply(3, 0, 1, "asp: key 0 -> 1");
    done("ASP CheckGetAndAdd");
  }
  {  // progress_tracker_test.cpp:19-25 Basic
    ProgressTracker t;
    t.Init({2, 7});
    expect(t.GetNumThreads() == 2 && t.GetProgress(2) == 0 && t.GetProgress(7) == 0, "tracker basic");
    done("ProgressTracker Basic");
  }
  {  // progress_tracker_test.cpp:27-34 CheckThreadValid
    ProgressTracker t;
    t.Init({2, 7});
    expect(t.CheckThreadValid(2) && !t.CheckThreadValid(3) && !t.CheckThreadValid(6) && t.CheckThreadValid(7),
           "tracker valid threads");
    done("ProgressTracker CheckThreadValid");
  }
  {  // progress_tracker_test.cpp:36-47 Advance
    ProgressTracker t;
    t.Init({2, 7});
    expect(t.GetMinClock() == 0, "tracker min 0");
    expect(t.AdvanceAndGetChangedMinClock(2) == -1, "advance 2 -> [1,0]");
    expect(t.AdvanceAndGetChangedMinClock(7) == 1, "advance 7 -> [1,1]");
    expect(t.AdvanceAndGetChangedMinClock(7) == -1, "advance 7 -> [1,2]");
    expect(t.AdvanceAndGetChangedMinClock(7) == -1, "advance 7 -> [1,3]");
    expect(t.AdvanceAndGetChangedMinClock(2) == 2, "advance 2 -> [2,3]");
    expect(t.GetProgress(2) == 2 && t.GetProgress(7) == 3, "tracker progress");
    done("ProgressTracker Advance");
  }
  {  // progress_tracker_test.cpp:49-55 UniqueMin
    ProgressTracker t;
    t.Init({2, 7});
    expect(!t.IsUniqueMin(2), "not unique min at [0,0]");
    t.AdvanceAndGetChangedMinClock(2);
    expect(t.IsUniqueMin(7), "unique min at [1,0]");
    done("ProgressTracker UniqueMin");
  }
  {  // pending_buffer_test.cpp:21-61 PushAndPop
    PendingBuffer b;
    Message m1 = msg(Flag::kAdd, 2, {0}, {1}), m2 = msg(Flag::kAdd, 2, {0}, {1});
    b.Push(0, m1);
    b.Push(0, m1);
    b.Push(1, m2);
    expect(b.Size(0) == 2 && b.Size(1) == 1, "buffer sizes");
    const auto p0 = b.Pop(0);
    const auto p1 = b.Pop(1);
    expect(p0.size() == 2 && p1.size() == 1, "buffer pops");
    expect(b.Size(0) == 0 && b.Size(1) == 0, "buffer empty after the pops");
    done("PendingBuffer PushAndPop");
  }
  {  // server_thread_test.cpp:35-120: one FIFO thread dispatches by flag
    struct FakeModel : AbstractModel {
      void Clock(Message&) override { ++clocks; }
      void Add(Message&) override { ++adds; }
      void Get(Message&) override { ++gets; }
      int GetProgress(int) override { return -1; }
      void ResetWorker(Message&) override {}
      int clocks = 0, adds = 0, gets = 0;
    };
    {
      ServerThread st(0);
      st.RegisterModel(0, std::unique_ptr<AbstractModel>(new FakeModel()));
      expect(st.GetModel(0) != nullptr, "server thread: registered model");
      done("ServerThread RegisterModel");
    }
    const Flag flags[3] = {Flag::kClock, Flag::kAdd, Flag::kGet};
    const int pushes[3] = {2, 1, 3};  // Clock x2, Add x1, Get x3 (:46-119)
    const char* names[3] = {"ServerThread Clock", "ServerThread Add", "ServerThread Get"};
    for (int c = 0; c < 3; ++c) {
      ServerThread st(0);
      st.RegisterModel(0, std::unique_ptr<AbstractModel>(new FakeModel()));
      auto* p = static_cast<FakeModel*>(st.GetModel(0));
      st.Start();
      Message m;
      m.meta.flag = flags[c];
      m.meta.model_id = 0;
      for (int i = 0; i < pushes[c]; ++i) st.GetWorkQueue()->Push(m);
      Message ex;
      ex.meta.flag = Flag::kExit;
      st.GetWorkQueue()->Push(ex);
      st.Stop();
      const int got = c == 0 ? p->clocks : c == 1 ? p->adds : p->gets;
      expect(got == pushes[c] && p->clocks + p->adds + p->gets == pushes[c], names[c]);
      done(names[c]);
    }
  }
  {  // callback_runner_test.cpp:19-108: replies handed to the receive handle,
     // the finish handle after the last expected one, two app threads apart
    auto reply_msg = [](std::vector<uint32_t> k, std::vector<float> v) {
      Message m;
      m.AddData(third_party::SArray<uint32_t>(k));
      m.AddData(third_party::SArray<float>(v));
      return m;
    };
    {
      CallbackRunner runner;
      std::map<uint32_t, float> reply;
      bool finished = false;
      runner.RegisterRecvHandle(0, 0, [&reply](Message& m) {
        third_party::SArray<uint32_t> k(m.data[0]);
        third_party::SArray<float> v(m.data[1]);
        for (size_t i = 0; i < k.size(); ++i) reply.insert(std::make_pair(k[i], v[i]));
      });
      runner.RegisterRecvFinishHandle(0, 0, [&finished] { finished = true; });
      runner.NewRequest(0, 0, 2);
      Message r1 = reply_msg({3}, {0.1f}), r2 = reply_msg({4, 5, 6}, {0.4f, 0.2f, 0.3f});
      runner.AddResponse(0, 0, r1);
      runner.AddResponse(0, 0, r2);
      runner.WaitRequest(0, 0);
      const std::map<uint32_t, float> want{{3, 0.1f}, {4, 0.4f}, {5, 0.2f}, {6, 0.3f}};
      expect(reply == want && finished, "callback runner: replies and finish");
      done("CallbackRunner AddResponse");
    }
    {
      CallbackRunner runner;
      std::map<uint32_t, float> reply;
      float sum = 0;
      runner.RegisterRecvHandle(0, 0, [&reply](Message& m) {
        third_party::SArray<uint32_t> k(m.data[0]);
        third_party::SArray<float> v(m.data[1]);
        for (size_t i = 0; i < k.size(); ++i) reply.insert(std::make_pair(k[i], v[i]));
      });
      runner.RegisterRecvFinishHandle(0, 0, [] {});
      runner.NewRequest(0, 0, 2);
      runner.RegisterRecvHandle(1, 0, [&sum](Message& m) {
        third_party::SArray<float> v(m.data[1]);
        for (size_t i = 0; i < v.size(); ++i) sum += v[i];
      });
      runner.RegisterRecvFinishHandle(1, 0, [] {});
      runner.NewRequest(1, 0, 2);
      Message r1 = reply_msg({3}, {0.1f}), r2 = reply_msg({4, 5, 6}, {0.4f, 0.2f, 0.3f});
      runner.AddResponse(0, 0, r1);
      runner.AddResponse(0, 0, r2);
      runner.AddResponse(1, 0, r1);
      runner.AddResponse(1, 0, r2);
      runner.WaitRequest(0, 0);
      const std::map<uint32_t, float> want{{3, 0.1f}, {4, 0.4f}, {5, 0.2f}, {6, 0.3f}};
      expect(reply == want, "callback runner: worker 0 replies");
      runner.WaitRequest(1, 0);
      // the reference asserts EXPECT_EQ(sum, 1.0): 0.1f + 0.4f + 0.2f + 0.3f in
      // this order is 1.0f exactly
      expect(sum == 1.0f, "callback runner: worker 1 sum");
      done("CallbackRunner AddResponseTwoWorkers");
    }
  }
  std::printf("[%s] model known answers: %s\n", label, fails ? "FAIL" : "ok");
  return fails;
}

}  // namespace

int main(int argc, char** argv) {
  std::setvbuf(stdout, nullptr, _IOLBF, 0);  // each line out as printed (logs survive an abort)
  Config c;
  bool ka = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto nxt = [&]() { return std::string(argv[++i]); };
    if (a == "--model") c.model = nxt();
    else if (a == "--workers") c.workers = std::stoi(nxt());
    else if (a == "--shards") c.shards = std::stoi(nxt());
    else if (a == "--iters") c.iters = std::stoi(nxt());
    else if (a == "--batch") c.batch = std::stoi(nxt());
    else if (a == "--staleness") c.staleness = std::stoi(nxt());
    else if (a == "--skew") c.skew = std::stoi(nxt());
    else if (a == "--features") c.n_features = (uint32_t)std::stoul(nxt());
    else if (a == "--cpu-only") c.cpu_only = true;
    else if (a == "--bsp-ungrouped") c.bsp_ungrouped = true;
    else if (a == "--threads") c.threads = true;
    else if (a == "--frames") c.frames = true;
    else if (a == "--known-answers") ka = true;
    else if (a == "--partition") c.partition = nxt();
    else if (a == "--trace") c.trace = nxt();
  }
  int fails = 0;
  if (ka) {
    fails += known_answers([] { return std::unique_ptr<AbstractStorage>(new OracleStorage<int>()); }, "oracle");
    if (!c.cpu_only)
      fails += known_answers(
          [] { return std::unique_ptr<AbstractStorage>(new HipStorage<int>(0, 0, 1024)); }, "hip");
  }
  if (!c.trace.empty() && c.threads) {
    std::fprintf(stderr, "--trace needs the single-threaded scheduler (no --threads)\n");
    return 2;
  }
  Run ref = Replay(c, false).run();
  std::unique_ptr<TraceWriter> tw(c.trace.empty() ? nullptr : new TraceWriter(c.trace));
  Run other = Replay(c, !c.cpu_only, tw.get()).run();
  tw.reset();
  std::string why;
  const bool ok = same(ref, other, &why);
  std::printf("replay model=%s partition=%s%s workers=%d shards=%d iters=%d batch=%d staleness=%d: msgs=%llu "
              "adds=%llu gets=%llu clocks=%llu ssp_releases=%llu replies=%zu\n",
              c.model.c_str(), c.partition.c_str(), c.frames ? " frames" : "", c.workers, c.shards, c.iters, c.batch, c.staleness,
              (unsigned long long)ref.msgs, (unsigned long long)ref.adds, (unsigned long long)ref.gets,
              (unsigned long long)ref.clocks, (unsigned long long)ref.echoes, ref.log.size());
  std::printf("cpu %.3f s, %s %.3f s\n", ref.seconds, c.cpu_only ? "cpu" : "hip", other.seconds);
  std::printf("%s%s\n", ok ? "REPLAY OK (bit-exact)" : "REPLAY MISMATCH: ", ok ? "" : why.c_str());
  // every shard is gone (the Replay objects and models above own them); hand
  // the cached page-locked frames back while the HIP runtime is still up
  if (!c.cpu_only) (void)pskv_host_pool_trim();
  return ok && fails == 0 ? 0 : 1;
}
