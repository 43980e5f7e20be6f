// kv_client_table_test.cpp — the worker-side surface (ps/kv_client_table.hpp)
// against the reference's own tests, and the whole drop-in path end to end.
//
//   Init / Add / Get        worker/kv_client_table_test.cpp:113-229 restated:
//                           FakePartitionManager (split at key 4, zero-copy
//                           segments), FakeCallbackRunner, keys {3,4,5,6};
//                           Get returns {0.1, 0.4, 0.2, 0.3} from the two replies
//   TypedSliceEqualsReference  RangeShardMap: the typed value cut (no double round
//                           trip) produces the same messages as the reference's
//                           double path (forced with a copying partition manager)
//   MergeUnsorted           unsorted keys with duplicates: std::map order, one
//                           value per key (kv_client_table.hpp:112-145)
//   System <model>          W worker threads, each with a KVClientTable over a
//                           RangeShardMap of S servers; a sender thread routes
//                           messages to S ServerThreads (FIFO, one model + one
//                           storage each, built by CreateTable); a receiver thread
//                           hands Get replies to the CallbackRunner and routes
//                           SSP-released requests back to their server.  Workers
//                           own disjoint keys (k % W), so ASP and SSP Gets must
//                           read the worker's own last Add; for all models the
//                           final shard contents must equal the last write of
//                           every key (BSP flushes on the last Clock).
//
// usage: kv_client_table_test [--host-only] [--storage hip|cpu]
//   --host-only runs everything on the CPU storage (no GPU needed);
//   --storage hip (default) drives HipStorage<float> shards on the GPU.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "ps/consistent_hashing_partition_manager.hpp"
#include "ps/kv_client_table.hpp"
#include "ps/range_partition_manager.hpp"
#include "ps/server_thread.hpp"
#include "ps/storage_factory.hpp"

using namespace csci5570;

static std::atomic<int> g_fail{0}, g_pass{0};
#define EXPECT(cond)                                                            \
  do {                                                                          \
    if (cond) {                                                                 \
      ++g_pass;                                                                 \
    } else {                                                                    \
      ++g_fail;                                                                 \
      std::printf("  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);             \
    }                                                                           \
  } while (0)

namespace {

const uint32_t kTestAppThreadId = 15;
const uint32_t kTestModelId = 23;

// kv_client_table_test.cpp:22-50: two servers, split at `split`, zero-copy segments
class FakePartitionManager : public AbstractPartitionManager {
 public:
  FakePartitionManager(const std::vector<uint32_t>& ids, uint32_t split)
      : AbstractPartitionManager(ids), split_(split) {}
  void Slice(const Keys& keys, std::vector<std::pair<int, Keys>>* sliced) const override {
    const size_t n = keys.size();
    const size_t pos = std::lower_bound(keys.begin(), keys.end(), split_) - keys.begin();
    sliced->resize(2);
    sliced->at(0) = std::make_pair(0, keys.segment(0, pos));
    sliced->at(1) = std::make_pair(1, keys.segment(pos, n));
  }
  void Slice(const KVPairs& kvs, std::vector<std::pair<int, KVPairs>>* sliced) const override {
    const size_t n = kvs.first.size();
    const size_t pos = std::lower_bound(kvs.first.begin(), kvs.first.end(), split_) - kvs.first.begin();
    sliced->resize(2);
    sliced->at(0) = std::make_pair((int)server_thread_ids_[0],
                                   std::make_pair(kvs.first.segment(0, pos), kvs.second.segment(0, pos)));
    sliced->at(1) = std::make_pair((int)server_thread_ids_[1],
                                   std::make_pair(kvs.first.segment(pos, n), kvs.second.segment(pos, n)));
  }

 private:
  uint32_t split_;
};

// A partition manager whose key slices are COPIES: KVClientTable must take the
// reference's double path with it.
class CopyingPartitionManager : public AbstractPartitionManager {
 public:
  explicit CopyingPartitionManager(const RangeShardMap& m) : AbstractPartitionManager(m.GetServerThreadIds()), m_(m) {}
  void Slice(const Keys& keys, std::vector<std::pair<int, Keys>>* sliced) const override {
    m_.Slice(keys, sliced);
    for (auto& s : *sliced) s.second = Copy(s.second);
  }
  void Slice(const KVPairs& kvs, std::vector<std::pair<int, KVPairs>>* sliced) const override {
    m_.Slice(kvs, sliced);
    for (auto& s : *sliced) s.second.first = Copy(s.second.first);
  }

 private:
  static Keys Copy(const Keys& k) { return Keys(std::vector<Key>(k.begin(), k.end())); }
  const RangeShardMap& m_;
};

// kv_client_table_test.cpp:52-111
class FakeCallbackRunner : public AbstractCallbackRunner {
 public:
  void RegisterRecvHandle(uint32_t a, uint32_t m, const std::function<void(Message&)>& h) override {
    EXPECT(a == kTestAppThreadId && m == kTestModelId);
    recv_ = h;
  }
  void RegisterRecvFinishHandle(uint32_t a, uint32_t m, const std::function<void()>& h) override {
    EXPECT(a == kTestAppThreadId && m == kTestModelId);
    finish_ = h;
  }
  void NewRequest(uint32_t a, uint32_t m, uint32_t expected) override {
    EXPECT(a == kTestAppThreadId && m == kTestModelId);
    std::lock_guard<std::mutex> lk(mu_);
    tracker_ = std::make_pair(expected, 0u);
  }
  void WaitRequest(uint32_t, uint32_t) override {
    std::unique_lock<std::mutex> lk(mu_);
    cond_.wait(lk, [this] { return tracker_.first == tracker_.second; });
  }
  void AddResponse(uint32_t, uint32_t, Message& m) override {
    bool last;
    {
      std::lock_guard<std::mutex> lk(mu_);
      last = tracker_.first == tracker_.second + 1;
    }
    recv_(m);
    if (last) finish_();
    std::lock_guard<std::mutex> lk(mu_);
    tracker_.second += 1;
    if (last) cond_.notify_all();
  }
  bool registered() {
    std::lock_guard<std::mutex> lk(mu_);
    return tracker_.first != 0;
  }

 private:
  std::function<void(Message&)> recv_;
  std::function<void()> finish_;
  std::mutex mu_;
  std::condition_variable cond_;
  std::pair<uint32_t, uint32_t> tracker_{0, 0};
};

void ReferenceCases() {
  std::printf("[ RUN ] Init / Add / Get (worker/kv_client_table_test.cpp)\n");
  {
    ThreadsafeQueue<Message> queue;
    FakePartitionManager manager({0, 1}, 4);
    FakeCallbackRunner cb;
    KVClientTable<float> table(kTestAppThreadId, kTestModelId, &queue, &manager, &cb);
  }
  {
    ThreadsafeQueue<Message> queue;
    FakePartitionManager manager({0, 1}, 4);
    FakeCallbackRunner cb;
    KVClientTable<float> table(kTestAppThreadId, kTestModelId, &queue, &manager, &cb);
    std::vector<Key> keys = {3, 4, 5, 6};
    std::vector<float> vals = {0.1f, 0.1f, 0.1f, 0.1f};
    table.Add(keys, vals);  // {3,4,5,6} -> {3}, {4,5,6}
    Message m1, m2;
    queue.WaitAndPop(&m1);
    queue.WaitAndPop(&m2);
    EXPECT(m1.meta.sender == (int)kTestAppThreadId && m1.meta.recver == 0);
    EXPECT(m1.meta.model_id == (int)kTestModelId && m1.meta.flag == Flag::kAdd);
    EXPECT(m1.data.size() == 2);
    third_party::SArray<Key> k1(m1.data[0]);
    third_party::SArray<float> v1(m1.data[1]);
    EXPECT(k1.size() == 1 && k1[0] == 3 && v1.size() == 1 && v1[0] == 0.1f);
    EXPECT(m2.meta.recver == 1 && m2.meta.flag == Flag::kAdd && m2.data.size() == 2);
    third_party::SArray<Key> k2(m2.data[0]);
    third_party::SArray<float> v2(m2.data[1]);
    EXPECT(k2.size() == 3 && k2[0] == 4 && k2[1] == 5 && k2[2] == 6);
    EXPECT(v2.size() == 3 && v2[0] == 0.1f && v2[1] == 0.1f && v2[2] == 0.1f);
  }
  {
    ThreadsafeQueue<Message> queue;
    FakePartitionManager manager({0, 1}, 4);
    FakeCallbackRunner cb;
    std::thread th([&] {
      KVClientTable<float> table(kTestAppThreadId, kTestModelId, &queue, &manager, &cb);
      std::vector<Key> keys = {3, 4, 5, 6};
      std::vector<float> vals;
      table.Get(keys, &vals);
      std::vector<float> expected{0.1f, 0.4f, 0.2f, 0.3f};
      EXPECT(vals == expected);
    });
    Message m1, m2;
    queue.WaitAndPop(&m1);
    queue.WaitAndPop(&m2);
    EXPECT(m1.meta.recver == 0 && m1.meta.flag == Flag::kGet && m1.data.size() == 1);
    EXPECT(third_party::SArray<Key>(m1.data[0]).size() == 1);
    EXPECT(m2.meta.recver == 1 && m2.meta.flag == Flag::kGet && m2.data.size() == 1);
    EXPECT(third_party::SArray<Key>(m2.data[0]).size() == 3);
    while (!cb.registered()) std::this_thread::yield();  // requests were pushed after NewRequest
    Message r1, r2;
    r1.AddData(third_party::SArray<Key>({3}));
    r1.AddData(third_party::SArray<float>({0.1f}));
    r2.AddData(third_party::SArray<Key>({4, 5, 6}));
    r2.AddData(third_party::SArray<float>({0.4f, 0.2f, 0.3f}));
    cb.AddResponse(kTestAppThreadId, kTestModelId, r1);
    cb.AddResponse(kTestAppThreadId, kTestModelId, r2);
    th.join();
  }
}

void TypedSliceEqualsReference() {
  std::printf("[ RUN ] TypedSliceEqualsReference\n");
  RangeShardMap map({10, 11, 12}, {{0, 100}, {100, 200}, {200, 300}});
  CopyingPartitionManager copying(map);
  // sorted, out-of-range, and unsorted tails (fall-through to the last server)
  const std::vector<Key> keys = {1, 2, 99, 100, 150, 250, 299, 300, 7000, 5, 120};
  std::vector<double> vals;
  for (size_t i = 0; i < keys.size(); ++i) vals.push_back(0.1 * (double)i - 3.0);
  ThreadsafeQueue<Message> qa, qb;
  CallbackRunner cb;
  KVClientTable<double> fast(1, 2, &qa, &map, &cb);
  KVClientTable<double> ref(1, 2, &qb, &copying, &cb);
  fast.Add(keys, vals);
  ref.Add(keys, vals);
  EXPECT(qa.Size() == qb.Size() && qa.Size() == 3);
  while (qa.Size()) {
    Message a, b;
    qa.WaitAndPop(&a);
    qb.WaitAndPop(&b);
    EXPECT(a.meta.recver == b.meta.recver && a.meta.flag == b.meta.flag && a.meta.sender == b.meta.sender);
    third_party::SArray<Key> ka(a.data[0]), kb(b.data[0]);
    third_party::SArray<double> va(a.data[1]), vb(b.data[1]);
    EXPECT(ka.size() == kb.size() && va.size() == vb.size() && ka.size() == va.size());
    EXPECT(std::memcmp(ka.data(), kb.data(), ka.size() * 4) == 0);
    EXPECT(std::memcmp(va.data(), vb.data(), va.size() * 8) == 0);
  }
  // the values are copies: changing the caller's array after Add changes nothing
  third_party::SArray<Key> sk(keys);
  third_party::SArray<double> sv(vals);
  fast.Add(sk, sv);
  sv[0] = 1e9;
  Message m;
  qa.WaitAndPop(&m);
  EXPECT(third_party::SArray<double>(m.data[1])[0] == vals[0]);
  while (qa.Size()) qa.WaitAndPop(&m);
}

void MergeUnsorted() {
  std::printf("[ RUN ] MergeUnsorted\n");
  RangeShardMap map({0, 1}, {{0, 8}, {8, 16}});
  ThreadsafeQueue<Message> q;
  CallbackRunner cb;
  std::vector<float> got;
  std::atomic<bool> done{false};
  std::thread th([&] {
    KVClientTable<float> t(5, 6, &q, &map, &cb);
    t.Get(std::vector<Key>{9, 3, 3, 12, 1}, &got);  // forward walk: all to srv1 (3 and 1 fall through)
    done = true;
  });
  while (!done.load()) {  // play the server: reply with value = key / 2
    if (!q.Size()) {
      std::this_thread::yield();
      continue;
    }
    Message req;
    q.WaitAndPop(&req);
    third_party::SArray<Key> k(req.data[0]);
    third_party::SArray<float> v(k.size());
    for (size_t i = 0; i < k.size(); ++i) v[i] = (float)k[i] * 0.5f;
    Message rep;
    rep.AddData(k);
    rep.AddData(v);
    cb.AddResponse(5, 6, rep);
  }
  th.join();
  const std::vector<float> want = {0.5f, 1.5f, 4.5f, 6.0f};  // keys 1, 3, 9, 12
  EXPECT(got == want);
}

// The reference's MapStorage semantics for the CPU leg of the system test
// (std::map, last write wins, 0 if absent; server/map_storage.hpp:17-45).
template <typename Val>
class LocalMapStorage : public AbstractStorage {
 public:
  void SubAdd(const third_party::SArray<Key>& k, const third_party::SArray<char>& vals) override {
    third_party::SArray<Val> v(vals);
    PS_CHECK(k.size() == v.size());
    for (size_t i = 0; i < k.size(); ++i) m_[k[i]] = v[i];
  }
  third_party::SArray<char> SubGet(const third_party::SArray<Key>& k) override {
    third_party::SArray<Val> out(k.size());
    for (size_t i = 0; i < k.size(); ++i) {
      auto it = m_.find(k[i]);
      out[i] = it == m_.end() ? Val(0) : it->second;
    }
    return third_party::SArray<char>(out);
  }
  void FinishIter() override {}

 private:
  std::map<Key, Val> m_;
};

float ValueOf(int w, int it, Key k) { return (float)((it * 131 + (int)(k % 977)) * 4 + w) * 0.25f; }

bool InSet(Key k, int it) { return ((k * 2654435761u) >> 7 ^ (uint32_t)it * 40503u) % 3 != 0; }

void System(ModelType model_type, const char* model_name, StorageType storage_type, bool hashed = false) {
  std::printf("[ RUN ] System %s (%s storage, %s partitioning)\n", model_name,
              storage_type == StorageType::Hip ? "hip" : "cpu", hashed ? "consistent-hash" : "range");
  const int W = 4, S = 3, I = 12;
  const Key K = 3000;  // range keys [0, K); each worker also owns one key >= K
  const uint32_t model_id = 0;
  std::vector<uint32_t> sids = {0, 1, 2};
  RangeShardMap range_map(sids, {{0, 1000}, {1000, 2000}, {2000, 3000}});
  // the reference Engine's default partitioner: every server owns [0, K) and
  // the keys >= K land in the overflow table of whichever server they hash to
  ConsistentHashShardMap hash_map(sids);
  const AbstractPartitionManager& map = hashed ? static_cast<const AbstractPartitionManager&>(hash_map)
                                               : static_cast<const AbstractPartitionManager&>(range_map);
  std::vector<std::unique_ptr<ServerThread>> servers;
  for (auto id : sids) servers.emplace_back(new ServerThread(id));
  ReplyQueue replies;
  auto cpu = [](StorageType) { return std::unique_ptr<AbstractStorage>(new LocalMapStorage<float>()); };
  auto storages = hashed ? CreateTable<float>(servers, hash_map, K, model_id, model_type, storage_type,
                                              /*staleness=*/1, &replies, PSKV_ASSIGN, cpu)
                         : CreateTable<float>(servers, range_map, model_id, model_type, storage_type,
                                              /*staleness=*/1, &replies, PSKV_ASSIGN, cpu);
  // ResetWorker: every model tracks the W worker threads (server/abstract_model.hpp)
  std::vector<uint32_t> tids;
  for (int w = 0; w < W; ++w) tids.push_back(100 + w);
  for (auto& s : servers) {
    Message r;
    r.meta.flag = Flag::kResetWorkerInModel;
    r.meta.sender = 999;
    r.meta.recver = (int)s->GetId();
    r.AddData(third_party::SArray<uint32_t>(tids));
    s->GetModel(model_id)->ResetWorker(r);
  }
  Message drop;
  while (replies.Pop(&drop)) {
  }
  for (auto& s : servers) s->Start();

  // sender: worker messages -> the server's FIFO (comm/sender.cpp role)
  ThreadsafeQueue<Message> sender_queue;
  std::thread sender([&] {
    for (;;) {
      Message m;
      sender_queue.WaitAndPop(&m);
      if (m.meta.flag == Flag::kExit) break;
      servers.at((size_t)m.meta.recver)->GetWorkQueue()->Push(m);
    }
  });
  // receiver: Get replies -> CallbackRunner; SSP-released requests -> back to
  // their server (ssp_model.cpp:18-22 pushes the request itself)
  CallbackRunner callbacks;
  std::atomic<bool> stop{false};
  std::atomic<int> released{0};
  std::thread receiver([&] {
    while (!stop.load()) {
      Message m;
      if (!replies.Pop(&m)) {
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        continue;
      }
      if (m.meta.flag == Flag::kGet && m.data.size() == 1) {
        released += 1;
        servers.at((size_t)m.meta.recver)->GetWorkQueue()->Push(m);
      } else if (m.meta.flag == Flag::kGet) {
        callbacks.AddResponse((uint32_t)m.meta.recver, (uint32_t)m.meta.model_id, m);
      }
    }
  });

  std::vector<std::thread> workers;
  std::atomic<int> mismatches{0};
  for (int w = 0; w < W; ++w) {
    workers.emplace_back([&, w] {
      KVClientTable<float> table(100 + w, model_id, &sender_queue, &map, &callbacks);
      for (int it = 0; it < I; ++it) {
        std::vector<Key> keys;
        std::vector<float> vals;
        for (Key k = (Key)w; k < K; k += W)
          if (InSet(k, it)) keys.push_back(k);
        keys.push_back(K + 1000 + (Key)w);  // beyond every range: the last server's overflow table
        for (Key k : keys) vals.push_back(ValueOf(w, it, k));
        table.Add(keys, vals);
        std::vector<float> got;
        table.Get(keys, &got);
        if (model_type != ModelType::BSP && got != vals) mismatches += 1;
        if (got.size() != keys.size()) mismatches += 1;
        table.Clock();
      }
    });
  }
  for (auto& t : workers) t.join();
  // drain the sender first: every worker message (the last Clocks, which
  // trigger BSP's final flush) is in its server's FIFO before kExit is
  Message ex;
  ex.meta.flag = Flag::kExit;
  sender_queue.Push(ex);
  sender.join();
  for (auto& s : servers) s->Stop();  // FIFO: every queued message is handled first
  stop = true;
  receiver.join();
  EXPECT(mismatches.load() == 0);
  if (model_type == ModelType::SSP) std::printf("  SSP released %d buffered requests\n", released.load());

  // final contents: the last write of every key
  std::map<Key, float> want;
  for (int w = 0; w < W; ++w)
    for (int it = 0; it < I; ++it) {
      for (Key k = (Key)w; k < K; k += W)
        if (InSet(k, it)) want[k] = ValueOf(w, it, k);
      want[K + 1000 + (Key)w] = ValueOf(w, it, K + 1000 + (Key)w);
    }
  std::vector<std::pair<int, RangeShardMap::Keys>> sl;
  std::vector<Key> all;
  for (Key k = 0; k < K; ++k) all.push_back(k);
  for (int w = 0; w < W; ++w) all.push_back(K + 1000 + (Key)w);
  third_party::SArray<Key> ak(all);
  map.Slice(ak, &sl);
  size_t bad = 0;
  for (auto& s : sl) {
    Message g;
    g.meta.flag = Flag::kGet;
    g.AddData(s.second);
    Message r = storages[(size_t)s.first]->Get(g);
    third_party::SArray<float> v(r.data[1]);
    for (size_t i = 0; i < s.second.size(); ++i) {
      auto it = want.find(s.second[i]);
      const float e = it == want.end() ? 0.0f : it->second;
      if (std::memcmp(&e, &v[i], 4) != 0) ++bad;
    }
  }
  EXPECT(bad == 0);
}

}  // namespace

int main(int argc, char** argv) {
  bool host_only = false;
  StorageType st = StorageType::Hip;
  for (int i = 1; i < argc; ++i) {
    if (std::strcmp(argv[i], "--host-only") == 0) host_only = true;
    if (std::strcmp(argv[i], "--storage") == 0 && i + 1 < argc)
      st = std::strcmp(argv[++i], "cpu") == 0 ? StorageType::Map : StorageType::Hip;
  }
  if (host_only) st = StorageType::Map;
  ReferenceCases();
  TypedSliceEqualsReference();
  MergeUnsorted();
  System(ModelType::ASP, "ASP", st);
  System(ModelType::SSP, "SSP", st);
  System(ModelType::BSP, "BSP", st);
  System(ModelType::ASP, "ASP", st, /*hashed=*/true);
  System(ModelType::SSP, "SSP", st, /*hashed=*/true);
  System(ModelType::BSP, "BSP", st, /*hashed=*/true);
  std::printf("%d passed, %d failed\n", g_pass.load(), g_fail.load());
  // every shard is gone; hand the cached page-locked frames back while the HIP
  // runtime is still up (not from a static destructor at exit)
  if (st == StorageType::Hip) (void)pskv_host_pool_trim();
  return g_fail.load() ? 1 : 0;
}
