// ps/host_frames.hpp — SArrays over page-locked frames from the pskv pool
// (pskv_host_alloc / pskv_host_free, include/pskv.h), for SURVEY.md §8f-3:
// the mailbox receives every data frame of a message into one
// (comm/mailbox.cpp:246-257 wraps each received frame in an SArray whose
// deleter releases it), and HipStorage allocates its Get replies from the same
// pool.  Storage calls then read and write the frames in place
// (PSKV_HOST_FRAME): no staging copy on the server thread, and an Add returns
// once its work is queued.  The frame is released when the last SArray copy
// of it goes away; the pool holds it back until the queued work has run.
#pragma once

#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "pskv.h"

#ifdef PSKV_IN_REFERENCE_TREE
#include "base/third_party/sarray.h"
#else
#include "ps/sarray.hpp"
#endif

namespace csci5570 {

// A frame-backed SArray of n values (uninitialised).
template <typename V>
third_party::SArray<V> FrameArray(size_t n) {
  void* p = nullptr;
  if (pskv_host_alloc((uint64_t)(n * sizeof(V)), &p) != PSKV_OK) {
    std::fprintf(stderr, "Check failed: pskv_host_alloc: %s\n", pskv_last_error());
    std::abort();
  }
  third_party::SArray<V> a;
  a.reset(static_cast<V*>(p), n, [](V* q) { pskv_host_free(q); });
  return a;
}

// The received bytes of one data frame, copied into a page-locked frame: the
// one copy Mailbox::Recv makes (on the mailbox thread) in place of the staging
// copy the storage call would otherwise make on the server thread.
inline third_party::SArray<char> RecvIntoFrame(const void* data, size_t size) {
  auto a = FrameArray<char>(size);
  if (size) std::memcpy(a.data(), data, size);
  return a;
}

}  // namespace csci5570
