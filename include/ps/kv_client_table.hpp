// ps/kv_client_table.hpp — the worker-side producer of the storage path,
// restated from worker/kv_client_table.hpp:19-155 with its API unchanged:
//
//   KVClientTable<Val>(app_thread_id, model_id, sender_queue, partition_manager,
//                      callback_runner)
//   Clock()                                  one kClock message per server (:47-60)
//   Add(keys, vals)   vector / SArray forms  slice, one kAdd message per server (:63-105)
//   Get(keys, &vals)  vector / SArray forms  slice, one kGet per server, wait for
//                                            every reply; values returned in
//                                            SORTED UNIQUE KEY ORDER (:107-146)
//
// What the HBM shard path changes ("double round-trip removal"):
// the reference widens every value to double, slices the (keys, doubles) pair
// and narrows each slice back to Val element by element (:82-97).  For
// Val ∈ {int, float, double} that round trip is exact, so when the partition
// manager's key slices are segments of the caller's key array (RangeShardMap's
// are; so are the reference's test fakes) the values are cut at the same
// offsets and copied once, typed (one memcpy per server).  Any other partition
// manager (e.g. a consistent-hash one that gathers keys) takes the reference's
// path.  The messages are identical either way (tests/cpp/kv_client_table_test.cpp).
//
// Get merges the replies as the reference's std::map does (:112-120): one value
// per distinct key, in key order.  When the replies' keys, put in order of their
// first key, are already strictly increasing (sorted unique requests — the LR
// worker's case, logistic_regression.cpp:377-382) they are concatenated without
// the map; the result is the same.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "ps/abstract_partition_manager.hpp"
#include "ps/callback_runner.hpp"
#include "ps/message.hpp"
#include "ps/threadsafe_queue.hpp"

namespace csci5570 {

template <typename Val>
class KVClientTable {
 public:
  using Keys = third_party::SArray<Key>;
  using KVPairs = std::pair<third_party::SArray<Key>, third_party::SArray<double>>;

  KVClientTable(uint32_t app_thread_id, uint32_t model_id, ThreadsafeQueue<Message>* const sender_queue,
                const AbstractPartitionManager* const partition_manager,
                AbstractCallbackRunner* const callback_runner)
      : app_thread_id_(app_thread_id),
        model_id_(model_id),
        sender_queue_(sender_queue),
        partition_manager_(partition_manager),
        callback_runner_(callback_runner) {}

  void Clock() {
    PS_CHECK(partition_manager_ != nullptr);
    for (auto server_id : partition_manager_->GetServerThreadIds()) {
      Message msg = NewMsg((int)server_id, Flag::kClock);
      sender_queue_->Push(msg);
    }
  }

  void Add(const std::vector<Key>& keys, const std::vector<Val>& vals) {
    Add(Keys(keys), third_party::SArray<Val>(vals));
  }

  void Get(const std::vector<Key>& keys, std::vector<Val>* vals) {
    third_party::SArray<Val> result;
    Get(Keys(keys), &result);
    vals->assign(result.begin(), result.end());
  }

  void Add(const Keys& keys, const third_party::SArray<Val>& vals) {
    PS_CHECK(keys.size() == vals.size());
    std::vector<std::pair<int, Keys>> sliced;
    partition_manager_->Slice(keys, &sliced);
    std::vector<size_t> offs;
    if (SegmentsOf(keys, sliced, &offs)) {
      for (size_t i = 0; i < sliced.size(); ++i) {
        const size_t n = sliced[i].second.size();
        third_party::SArray<Val> v(n);
        if (n) std::memcpy(static_cast<void*>(v.data()), vals.data() + offs[i], n * sizeof(Val));
        Send(sliced[i].first, sliced[i].second, v);
      }
      return;
    }
    // the reference's path (kv_client_table.hpp:80-104)
    third_party::SArray<double> dv(vals.size());
    for (size_t i = 0; i < vals.size(); ++i) dv[i] = static_cast<double>(vals[i]);
    std::vector<std::pair<int, KVPairs>> kv_sliced;
    partition_manager_->Slice(std::make_pair(keys, dv), &kv_sliced);
    for (auto& s : kv_sliced) {
      third_party::SArray<Val> v(s.second.second.size());
      for (size_t i = 0; i < v.size(); ++i) v[i] = static_cast<Val>(s.second.second[i]);
      Send(s.first, s.second.first, v);
    }
  }

  void Get(const Keys& keys, third_party::SArray<Val>* vals) {
    std::vector<std::pair<int, Keys>> sliced;
    partition_manager_->Slice(keys, &sliced);
    std::mutex mu;
    std::vector<std::pair<Keys, third_party::SArray<Val>>> replies;
    callback_runner_->RegisterRecvHandle(app_thread_id_, model_id_, [&](Message& msg) {
      PS_CHECK(msg.data.size() == 2);
      std::lock_guard<std::mutex> lk(mu);
      replies.emplace_back(Keys(msg.data[0]), third_party::SArray<Val>(msg.data[1]));
    });
    callback_runner_->RegisterRecvFinishHandle(app_thread_id_, model_id_, [] {});
    callback_runner_->NewRequest(app_thread_id_, model_id_, (uint32_t)sliced.size());
    for (auto& s : sliced) {
      Message msg = NewMsg(s.first, Flag::kGet);
      msg.AddData(s.second);
      sender_queue_->Push(msg);
    }
    callback_runner_->WaitRequest(app_thread_id_, model_id_);
    Merge(replies, vals);
  }

 private:
  Message NewMsg(int recver, Flag flag) const {
    Message msg;
    msg.meta.sender = (int)app_thread_id_;
    msg.meta.recver = recver;
    msg.meta.model_id = (int)model_id_;
    msg.meta.flag = flag;
    return msg;
  }

  void Send(int server, const Keys& k, const third_party::SArray<Val>& v) {
    Message msg = NewMsg(server, Flag::kAdd);
    msg.AddData(k);
    msg.AddData(v);
    sender_queue_->Push(msg);
  }

  // True when every key slice is a segment of `keys` (a view into its buffer);
  // offs[i] = where slice i starts.
  static bool SegmentsOf(const Keys& keys, const std::vector<std::pair<int, Keys>>& sliced,
                         std::vector<size_t>* offs) {
    offs->clear();
    const Key* b = keys.data();
    const Key* e = b + keys.size();
    for (auto& s : sliced) {
      const Key* p = s.second.data();
      const size_t n = s.second.size();
      if (n == 0) {
        offs->push_back(0);
        continue;
      }
      if (b == nullptr || p < b || p + n > e) return false;
      offs->push_back((size_t)(p - b));
    }
    return true;
  }

  // std::map<Key, Val> semantics: insert keeps the value of the first reply
  // (in arrival order) that carries a key; values emitted in key order.
  static void Merge(const std::vector<std::pair<Keys, third_party::SArray<Val>>>& replies,
                    third_party::SArray<Val>* vals) {
    std::vector<size_t> order;
    size_t total = 0;
    for (size_t i = 0; i < replies.size(); ++i) {
      PS_CHECK(replies[i].first.size() == replies[i].second.size());
      if (!replies[i].first.empty()) order.push_back(i);
      total += replies[i].first.size();
    }
    std::sort(order.begin(), order.end(),
              [&](size_t a, size_t b) { return replies[a].first[0] < replies[b].first[0]; });
    bool increasing = true;
    bool have_prev = false;
    Key prev = 0;
    for (size_t i : order) {
      const Keys& k = replies[i].first;
      for (size_t j = 0; j < k.size() && increasing; ++j) {
        if (have_prev && k[j] <= prev) increasing = false;
        prev = k[j];
        have_prev = true;
      }
    }
    if (increasing) {  // disjoint sorted runs: the map's order is their concatenation
      third_party::SArray<Val> out(total);
      size_t o = 0;
      for (size_t i : order) {
        const auto& v = replies[i].second;
        std::memcpy(static_cast<void*>(out.data() + o), v.data(), v.size() * sizeof(Val));
        o += v.size();
      }
      *vals = out;
      return;
    }
    std::map<Key, Val> reply;  // kv_client_table.hpp:112-120
    for (auto& r : replies)
      for (size_t i = 0; i < r.first.size(); ++i) reply.insert(std::make_pair(r.first[i], r.second[i]));
    third_party::SArray<Val> out(reply.size());
    size_t o = 0;
    for (auto& kv : reply) out[o++] = kv.second;
    *vals = out;
  }

  uint32_t app_thread_id_;
  uint32_t model_id_;
  ThreadsafeQueue<Message>* const sender_queue_;                // not owned
  const AbstractPartitionManager* const partition_manager_;     // not owned
  AbstractCallbackRunner* const callback_runner_;               // not owned
};

}  // namespace csci5570
