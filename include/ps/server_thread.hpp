// ps/server_thread.hpp — the server actor that calls the storage, restated:
//   (ThreadsafeQueue: ps/threadsafe_queue.hpp)
//   ServerThread     server/server_thread.{hpp,cpp}: one std::thread per server
//                    id, FIFO WaitAndPop, dispatch by flag to the model of the
//                    message's model_id (server_thread.cpp:20-50); kExit stops it.
// With HipStorage, distinct server threads drive distinct shards concurrently
// — the threading contract of pskv.h.  `on_processed` (an addition for the
// replay harness) runs after every handled message.
#pragma once

#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <queue>
#include <thread>

#include "ps/consistency.hpp"
#include "ps/threadsafe_queue.hpp"

namespace csci5570 {

class ServerThread {
 public:
  explicit ServerThread(uint32_t id) : id_(id) {}
  ~ServerThread() { Stop(); }
  uint32_t GetId() const { return id_; }
  void RegisterModel(uint32_t model_id, std::unique_ptr<AbstractModel>&& model) {
    models_.insert(std::make_pair(model_id, std::move(model)));
  }
  AbstractModel* GetModel(uint32_t model_id) {
    auto it = models_.find(model_id);
    return it == models_.end() ? nullptr : it->second.get();
  }
  ThreadsafeQueue<Message>* GetWorkQueue() { return &queue_; }
  void SetOnProcessed(std::function<void()> f) { on_processed_ = std::move(f); }
  void Start() { thread_ = std::thread([this] { Main(); }); }
  void Stop() {
    if (!thread_.joinable()) return;
    Message m;
    m.meta.flag = Flag::kExit;
    queue_.Push(m);
    thread_.join();
  }

 private:
  void Main() {  // server/server_thread.cpp:20-50
    for (;;) {
      Message msg;
      queue_.WaitAndPop(&msg);
      if (msg.meta.flag == Flag::kExit) break;
      AbstractModel* model = GetModel((uint32_t)msg.meta.model_id);
      if (model != nullptr) {
        switch (msg.meta.flag) {
          case Flag::kClock: model->Clock(msg); break;
          case Flag::kAdd: model->Add(msg); break;
          case Flag::kGet: model->Get(msg); break;
          case Flag::kResetWorkerInModel: model->ResetWorker(msg); break;
          default: break;
        }
      }
      if (on_processed_) on_processed_();
    }
  }
  uint32_t id_;
  std::map<uint32_t, std::unique_ptr<AbstractModel>> models_;
  ThreadsafeQueue<Message> queue_;
  std::thread thread_;
  std::function<void()> on_processed_;
};

}  // namespace csci5570
