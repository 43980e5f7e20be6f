// ps/abstract_storage.hpp — the storage plugin surface of the reference
// (server/abstract_storage.hpp:12-42), restated for the standalone build, with
// ONE deliberate, source-compatible change: a virtual destructor.  The
// reference deletes storages through std::unique_ptr<AbstractStorage>
// (server/consistency/ssp_model.hpp:42, bsp_model.hpp:42, asp_model.hpp:32)
// but declares no virtual destructor, so a subclass holding HBM would leak.
#pragma once

#include <vector>

#include "ps/message.hpp"


namespace csci5570 {

class AbstractStorage {
 public:
  virtual ~AbstractStorage() = default;

  void Add(Message& msg) {
    PS_CHECK(msg.data.size() == 2);
    auto typed_keys = third_party::SArray<Key>(msg.data[0]);
    SubAdd(typed_keys, msg.data[1]);
  }

  Message Get(Message& msg) {
    PS_CHECK(msg.data.size() == 1);
    auto typed_keys = third_party::SArray<Key>(msg.data[0]);
    Message reply;
    reply.meta.recver = msg.meta.sender;
    reply.meta.sender = msg.meta.recver;
    reply.meta.flag = msg.meta.flag;
    reply.meta.model_id = msg.meta.model_id;
    third_party::SArray<Key> reply_keys(typed_keys);  // aliases the request keys
    third_party::SArray<char> reply_vals = SubGet(reply_keys);
    reply.AddData<Key>(reply_keys);
    reply.AddData<char>(reply_vals);
    return reply;
  }

  // Apply several Add messages in order (semantically msgs.size() Add calls).
  // Source-compatible extension: the default loops; HipStorage overrides it
  // with one grouped device call (BSP's flush of add_buffer_,
  // server/consistency/bsp_model.cpp:20-25, is the natural caller).
  virtual void AddGrouped(std::vector<Message>& msgs) {
    for (auto& m : msgs) Add(m);
  }

  virtual void SubAdd(const third_party::SArray<Key>& typed_keys,
                      const third_party::SArray<char>& vals) = 0;
  virtual third_party::SArray<char> SubGet(const third_party::SArray<Key>& typed_keys) = 0;
  virtual void FinishIter() = 0;
};

}  // namespace csci5570
