// ps/hip_storage.hpp — HipStorage<Val>: the HBM-backed drop-in for the
// reference's MapStorage<Val> (server/map_storage.hpp) and VectorStorage<Val>
// (server/vector_storage.hpp), implemented over the pskv C ABI (pskv.h).
//
// Inside the reference tree define PSKV_IN_REFERENCE_TREE before including
// this header so it derives from the reference's own server/abstract_storage.hpp
// (after adding the virtual destructor); standalone it
// uses the restated boundary in include/ps/.
//
// Contract kept from the reference:
//   * SubAdd: CHECK_EQ(keys, vals) then last-write-wins assign (map_storage.hpp:19-24)
//   * SubGet: a new owning SArray<char> of keys.size() values, 0 for missing keys
//     (map_storage.hpp:29-45); the reply keys alias the request (abstract_storage.hpp:27)
//   * errors abort, as glog CHECK does (abstract_storage.hpp:15,20)
//   * called from one server thread; the device is selected inside every call
//     because Engine::CreateTable constructs storages on another thread
//     (driver/engine.hpp:100-109)
// Page-locked frames (ps/host_frames.hpp): every call passes
// PSKV_HOST_FRAME, so request payloads the mailbox received into frames are
// read in place (an Add returns once queued; the frames stay alive through
// the message's SArrays and the pool holds them until the work has run), and
// Get replies are frames the kernel writes directly.  Payloads outside frames
// take the ordinary host paths.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pskv.h"
#include "ps/host_frames.hpp"

#ifdef PSKV_IN_REFERENCE_TREE
#include "server/abstract_storage.hpp"
#else
#include "ps/abstract_storage.hpp"
#endif

namespace csci5570 {

template <typename Val>
struct PskvDtype;
template <>
struct PskvDtype<int> {
  static constexpr int value = PSKV_I32;
};
template <>
struct PskvDtype<float> {
  static constexpr int value = PSKV_F32;
};
template <>
struct PskvDtype<double> {
  static constexpr int value = PSKV_F64;
};

inline void pskv_check(int rc, const char* what) {
  if (rc != PSKV_OK) {
    std::fprintf(stderr, "Check failed: %s returned %d: %s\n", what, rc, pskv_last_error());
    std::abort();
  }
}

template <typename Val>
class HipStorage : public AbstractStorage {
 public:
  // No arguments = the reference's construction: whole key space, assign.
  explicit HipStorage(int device = 0, uint32_t key_begin = 0, uint64_t key_end = 1ull << 32,
                      int mode = PSKV_ASSIGN, uint64_t overflow_slots = 0) {
    pskv_check(pskv_shard_create_ex(device, key_begin, key_end, PskvDtype<Val>::value, mode,
                                    overflow_slots, &shard_),
               "pskv_shard_create");
  }
  ~HipStorage() override { pskv_shard_destroy(shard_); }
  HipStorage(const HipStorage&) = delete;
  HipStorage& operator=(const HipStorage&) = delete;

  void SubAdd(const third_party::SArray<Key>& typed_keys,
              const third_party::SArray<char>& vals) override {
    auto typed_vals = third_party::SArray<Val>(vals);
    if (typed_keys.size() != typed_vals.size()) {
      std::fprintf(stderr, "Check failed: typed_keys.size() == typed_vals.size() (%zu vs %zu)\n",
                   (size_t)typed_keys.size(), (size_t)typed_vals.size());
      std::abort();
    }
    pskv_check(pskv_add(shard_, typed_keys.data(), typed_vals.data(), typed_keys.size(),
                        PSKV_HOST | PSKV_HOST_FRAME),
               "pskv_add");
  }

#ifndef PSKV_IN_REFERENCE_TREE
  // One staged copy and one grouped launch for a run of Add messages (BSP flush).
  void AddGrouped(std::vector<Message>& msgs) override {
    std::vector<pskv_batch> batches;
    std::vector<third_party::SArray<Key>> keep_k;
    std::vector<third_party::SArray<Val>> keep_v;
    batches.reserve(msgs.size());
    for (auto& m : msgs) {
      if (m.data.size() != 2) {
        std::fprintf(stderr, "Check failed: msg.data.size() == 2\n");
        std::abort();
      }
      keep_k.emplace_back(m.data[0]);
      keep_v.emplace_back(m.data[1]);
      if (keep_k.back().size() != keep_v.back().size()) {
        std::fprintf(stderr, "Check failed: typed_keys.size() == typed_vals.size()\n");
        std::abort();
      }
      batches.push_back(pskv_batch{keep_k.back().data(), keep_v.back().data(), keep_k.back().size()});
    }
    pskv_check(pskv_add_grouped(shard_, batches.data(), batches.size(), PSKV_HOST | PSKV_HOST_FRAME),
               "pskv_add_grouped");
  }
#endif

  third_party::SArray<char> SubGet(const third_party::SArray<Key>& typed_keys) override {
    // the reply is a page-locked frame: written in place by the kernel when the
    // request keys are a frame too, and sent zero-copy by the Sender
    auto reply_vals = FrameArray<Val>(typed_keys.size());
    pskv_check(pskv_get(shard_, typed_keys.data(), typed_keys.size(), reply_vals.data(),
                        PSKV_HOST | PSKV_HOST_FRAME),
               "pskv_get");
    return third_party::SArray<char>(reply_vals);
  }

  // The reference's FinishIter is a no-op (map_storage.hpp:47); here it is the
  // point where deferred device errors surface and the overflow table, which
  // grows on the device as keys arrive, is trimmed and its old arrays freed.
  void FinishIter() override { pskv_check(pskv_sync(shard_), "pskv_sync"); }

  pskv_shard* shard() const { return shard_; }

 private:
  pskv_shard* shard_ = nullptr;
};

}  // namespace csci5570
