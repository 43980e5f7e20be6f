// ps/callback_runner.hpp — where a worker's Get waits for its server replies,
// restated from worker/abstract_callback_runner.hpp:9-37 (the interface) and
// worker/callback_runner.cpp:9-72 (the implementation): per (app thread, model)
// a receive handle, a finish handle and a tracker {expected, received};
// WaitRequest blocks until every expected reply went through AddResponse.
//
// Differences from the reference implementation, none observable by a caller:
// the trackers are read under the lock (the reference reads its std::maps
// unlocked in AddResponse, callback_runner.cpp:48-50, racing NewRequest of
// other threads) and are held by value (the reference leaks a `new` pair per
// request, :33-34).
#pragma once

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <utility>

#include "ps/message.hpp"

namespace csci5570 {

class AbstractCallbackRunner {
 public:
  virtual ~AbstractCallbackRunner() = default;
  virtual void RegisterRecvHandle(uint32_t app_thread_id, uint32_t model_id,
                                  const std::function<void(Message&)>& recv_handle) = 0;
  virtual void RegisterRecvFinishHandle(uint32_t app_thread_id, uint32_t model_id,
                                        const std::function<void()>& recv_finish_handle) = 0;
  virtual void NewRequest(uint32_t app_thread_id, uint32_t model_id, uint32_t expected_responses) = 0;
  virtual void WaitRequest(uint32_t app_thread_id, uint32_t model_id) = 0;
  virtual void AddResponse(uint32_t app_thread_id, uint32_t model_id, Message& msg) = 0;
};

class CallbackRunner : public AbstractCallbackRunner {
 public:
  void RegisterRecvHandle(uint32_t app_thread_id, uint32_t model_id,
                          const std::function<void(Message&)>& recv_handle) override {
    std::lock_guard<std::mutex> lk(mu_);
    recv_[Id(app_thread_id, model_id)] = recv_handle;
  }
  void RegisterRecvFinishHandle(uint32_t app_thread_id, uint32_t model_id,
                                const std::function<void()>& recv_finish_handle) override {
    std::lock_guard<std::mutex> lk(mu_);
    finish_[Id(app_thread_id, model_id)] = recv_finish_handle;
  }
  void NewRequest(uint32_t app_thread_id, uint32_t model_id, uint32_t expected_responses) override {
    std::lock_guard<std::mutex> lk(mu_);
    trackers_[Id(app_thread_id, model_id)] = std::make_pair(expected_responses, 0u);
  }
  void WaitRequest(uint32_t app_thread_id, uint32_t model_id) override {
    std::unique_lock<std::mutex> lk(mu_);
    const auto id = Id(app_thread_id, model_id);
    cond_.wait(lk, [&] {
      const auto& t = trackers_[id];
      return t.first == t.second;
    });
  }
  // Runs the receive handle on the calling (receiving) thread; the finish
  // handle after the last expected reply, then wakes the waiter
  // (callback_runner.cpp:46-68).
  void AddResponse(uint32_t app_thread_id, uint32_t model_id, Message& msg) override {
    const auto id = Id(app_thread_id, model_id);
    std::function<void(Message&)> recv;
    std::function<void()> finish;
    bool last = false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      recv = recv_[id];
      finish = finish_[id];
      const auto& t = trackers_[id];
      last = t.first == t.second + 1;
    }
    PS_CHECK(recv != nullptr);
    recv(msg);
    if (last && finish) finish();
    {
      std::lock_guard<std::mutex> lk(mu_);
      trackers_[id].second += 1;
    }
    if (last) cond_.notify_all();
  }

 private:
  static std::pair<uint32_t, uint32_t> Id(uint32_t a, uint32_t m) { return std::make_pair(a, m); }
  std::mutex mu_;
  std::condition_variable cond_;
  std::map<std::pair<uint32_t, uint32_t>, std::function<void(Message&)>> recv_;
  std::map<std::pair<uint32_t, uint32_t>, std::function<void()>> finish_;
  std::map<std::pair<uint32_t, uint32_t>, std::pair<uint32_t, uint32_t>> trackers_;
};

}  // namespace csci5570
