// ps/threadsafe_queue.hpp — the FIFO between actors, restated from
// base/threadsafe_queue.hpp:14-45 (Push / WaitAndPop / Size).  Server threads
// read their work from one; KVClientTable pushes to the sender's.
#pragma once

#include <condition_variable>
#include <mutex>
#include <queue>

namespace csci5570 {

template <typename T>
class ThreadsafeQueue {
 public:
  ThreadsafeQueue() = default;
  ThreadsafeQueue(const ThreadsafeQueue&) = delete;
  ThreadsafeQueue& operator=(const ThreadsafeQueue&) = delete;

  void Push(T v) {
    std::lock_guard<std::mutex> lk(m_);
    q_.push(std::move(v));
    cv_.notify_all();
  }
  void WaitAndPop(T* v) {
    std::unique_lock<std::mutex> lk(m_);
    cv_.wait(lk, [&] { return !q_.empty(); });
    *v = std::move(q_.front());
    q_.pop();
  }
  int Size() {
    std::lock_guard<std::mutex> lk(m_);
    return (int)q_.size();
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  std::queue<T> q_;
};

}  // namespace csci5570
