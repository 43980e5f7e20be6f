// ps/consistency.hpp — the CALLERS of the storage path, restated so the
// HBM-backed storage can be driven exactly as the reference drives it:
//
//   ProgressTracker  server/util/progress_tracker.cpp:7-47
//   PendingBuffer    server/util/pending_buffer.cpp:5-28
//   AbstractModel    server/abstract_model.hpp:9-17
//   SSPModel         server/consistency/ssp_model.cpp:6-62
//   BSPModel         server/consistency/bsp_model.cpp:7-87
//   ASPModel         server/consistency/asp_model.cpp:6-40
//
// Behaviour kept on purpose, quirks included:
//   * SSP buffers a Get while  progress(sender) > min_clock + staleness, keyed by
//     progress - staleness, and on a min-clock advance pushes the buffered
//     REQUEST (not a reply) to the reply queue (ssp_model.cpp:18-22); routed by
//     recver it comes back to the server and is served then.
//   * BSP defers every Add until the min clock advances and applies them in
//     arrival order, then re-runs buffered Gets (bsp_model.cpp:14-31).
//   * ProgressTracker::AdvanceAndGetChangedMinClock returns the new min only if
//     the caller was the unique slowest worker (progress_tracker.cpp:14-18).
// Unknown worker ids throw std::out_of_range like progresses_.at() does.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <queue>
#include <unordered_map>
#include <vector>

#include "ps/abstract_storage.hpp"

namespace csci5570 {

// The FIFO models push replies into (the reference uses ThreadsafeQueue,
// base/threadsafe_queue.hpp): several server threads may push concurrently.
class ReplyQueue {
 public:
  void Push(const Message& m) {
    std::lock_guard<std::mutex> lk(m_);
    q_.push(m);
  }
  bool Pop(Message* m) {
    std::lock_guard<std::mutex> lk(m_);
    if (q_.empty()) return false;
    *m = q_.front();
    q_.pop();
    return true;
  }
  size_t Size() {
    std::lock_guard<std::mutex> lk(m_);
    return q_.size();
  }

 private:
  std::mutex m_;
  std::queue<Message> q_;
};

class ProgressTracker {
 public:
  void Init(const std::vector<uint32_t>& tids) {
    min_clock_ = 0;
    for (auto t : tids) progresses_.insert(std::make_pair((int)t, 0));
  }
  int AdvanceAndGetChangedMinClock(int tid) {
    const bool unique_min = IsUniqueMin(tid);
    progresses_.at(tid)++;
    return unique_min ? ++min_clock_ : -1;
  }
  int GetProgress(int tid) const { return progresses_.at(tid); }
  int GetMinClock() const { return min_clock_; }
  int GetNumThreads() const { return (int)progresses_.size(); }
  bool IsUniqueMin(int tid) const {
    if (progresses_.at(tid) != min_clock_) return false;
    int n = 0;
    for (auto& p : progresses_)
      if (p.second == min_clock_ && ++n > 1) break;
    return n == 1;
  }
  bool CheckThreadValid(int tid) const { return progresses_.count(tid) != 0; }

 private:
  std::map<int, int> progresses_;
  int min_clock_ = 0;
};

class PendingBuffer {
 public:
  // Requests buffered at `clock`, in insertion order.
  std::vector<Message> Pop(int clock) {
    std::vector<Message> out;
    auto it = buf_.find(clock);
    if (it != buf_.end()) {
      out.swap(it->second);
      buf_.erase(it);
    }
    return out;
  }
  void Push(int clock, const Message& m) { buf_[clock].push_back(m); }
  int Size(int clock) const {
    auto it = buf_.find(clock);
    return it == buf_.end() ? 0 : (int)it->second.size();
  }

 private:
  std::map<int, std::vector<Message>> buf_;
};

class AbstractModel {
 public:
  virtual void Clock(Message& msg) = 0;
  virtual void Add(Message& msg) = 0;
  virtual void Get(Message& msg) = 0;
  virtual int GetProgress(int tid) = 0;
  virtual void ResetWorker(Message& msg) = 0;
  virtual ~AbstractModel() {}
};

namespace detail {
inline Message reset_reply(const Message& msg, uint32_t model_id) {
  Message r;
  r.meta.model_id = (int)model_id;
  r.meta.sender = msg.meta.recver;
  r.meta.recver = msg.meta.sender;
  r.meta.flag = Flag::kResetWorkerInModel;
  return r;
}
inline std::vector<uint32_t> tids_of(const Message& msg) {
  third_party::SArray<uint32_t> t(msg.data[0]);
  return std::vector<uint32_t>(t.begin(), t.end());
}
}  // namespace detail

class SSPModel : public AbstractModel {
 public:
  SSPModel(uint32_t model_id, std::unique_ptr<AbstractStorage>&& storage, int staleness,
           ReplyQueue* reply_queue)
      : model_id_(model_id), staleness_(staleness), reply_queue_(reply_queue),
        storage_(std::move(storage)) {}
  void Clock(Message& msg) override {
    const int new_min = tracker_.AdvanceAndGetChangedMinClock(msg.meta.sender);
    if (new_min != -1)
      for (auto& m : buffer_.Pop(new_min)) reply_queue_->Push(m);  // the request itself
  }
  void Add(Message& msg) override { storage_->Add(msg); }
  void Get(Message& msg) override {
    const int clock = tracker_.GetProgress(msg.meta.sender);
    if (clock > tracker_.GetMinClock() + staleness_)
      buffer_.Push(clock - staleness_, msg);
    else
      reply_queue_->Push(storage_->Get(msg));
  }
  int GetProgress(int tid) override { return tracker_.GetProgress(tid); }
  void ResetWorker(Message& msg) override {
    tracker_.Init(detail::tids_of(msg));
    Message r = detail::reset_reply(msg, model_id_);
    r.meta.model_id = -1;  // the SSP reply does not set model_id (ssp_model.cpp:52-56)
    reply_queue_->Push(r);
  }
  int GetPendingSize(int progress) { return buffer_.Size(progress); }
  AbstractStorage* storage() { return storage_.get(); }

 private:
  uint32_t model_id_;
  int staleness_;
  ReplyQueue* reply_queue_;
  std::unique_ptr<AbstractStorage> storage_;
  ProgressTracker tracker_;
  PendingBuffer buffer_;
};

class BSPModel : public AbstractModel {
 public:
  BSPModel(uint32_t model_id, std::unique_ptr<AbstractStorage>&& storage, ReplyQueue* reply_queue)
      : model_id_(model_id), reply_queue_(reply_queue), storage_(std::move(storage)) {}
  void Clock(Message& msg) override {
    if (tracker_.AdvanceAndGetChangedMinClock(msg.meta.sender) != -1) {
      // deferred Adds in arrival order (bsp_model.cpp:20-25), as ONE grouped
      // call: HipStorage turns it into one staged copy and one launch
      if (grouped_flush_) {
        if (!add_buffer_.empty()) storage_->AddGrouped(add_buffer_);
      } else {
        for (auto& m : add_buffer_) storage_->Add(m);
      }
      add_buffer_.clear();
      std::vector<Message> gets;
      gets.swap(get_buffer_);
      for (auto& m : gets) Get(m);
    }
  }
  void Add(Message& msg) override { add_buffer_.push_back(msg); }
  void Get(Message& msg) override {
    if (tracker_.GetProgress(msg.meta.sender) > tracker_.GetMinClock())
      get_buffer_.push_back(msg);
    else
      reply_queue_->Push(storage_->Get(msg));
  }
  int GetProgress(int tid) override { return tracker_.GetProgress(tid); }
  void ResetWorker(Message& msg) override {
    tracker_.Init(detail::tids_of(msg));
    reply_queue_->Push(detail::reset_reply(msg, model_id_));
  }
  void SetGroupedFlush(bool on) { grouped_flush_ = on; }  // off = the reference's per-message loop
  int GetGetPendingSize() const { return (int)get_buffer_.size(); }
  int GetAddPendingSize() const { return (int)add_buffer_.size(); }
  AbstractStorage* storage() { return storage_.get(); }

 private:
  uint32_t model_id_;
  ReplyQueue* reply_queue_;
  std::unique_ptr<AbstractStorage> storage_;
  ProgressTracker tracker_;
  std::vector<Message> add_buffer_, get_buffer_;
  bool grouped_flush_ = true;
};

class ASPModel : public AbstractModel {
 public:
  ASPModel(uint32_t model_id, std::unique_ptr<AbstractStorage>&& storage, ReplyQueue* reply_queue)
      : model_id_(model_id), reply_queue_(reply_queue), storage_(std::move(storage)) {}
  void Clock(Message&) override {}
  void Add(Message& msg) override { storage_->Add(msg); }
  void Get(Message& msg) override { reply_queue_->Push(storage_->Get(msg)); }
  int GetProgress(int tid) override { return tracker_.GetProgress(tid); }
  void ResetWorker(Message& msg) override {
    tracker_.Init(detail::tids_of(msg));
    reply_queue_->Push(detail::reset_reply(msg, model_id_));
  }

 private:
  uint32_t model_id_;
  ReplyQueue* reply_queue_;
  std::unique_ptr<AbstractStorage> storage_;
  ProgressTracker tracker_;
};

}  // namespace csci5570
