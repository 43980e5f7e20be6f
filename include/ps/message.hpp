// ps/message.hpp — clean-room restatement of the payload types that cross the
// storage boundary: Key (base/magic.hpp:7), Flag / Meta / Message
// (base/message.hpp:14-58).
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ps/sarray.hpp"

#ifndef PS_CHECK
// glog CHECK restated: print and abort (the reference's error convention).
#define PS_CHECK(cond)                                                           \
  do {                                                                           \
    if (!(cond)) {                                                               \
      std::fprintf(stderr, "Check failed: %s (%s:%d)\n", #cond, __FILE__, __LINE__); \
      std::abort();                                                              \
    }                                                                            \
  } while (0)
#endif

namespace csci5570 {

using Key = uint32_t;

enum class Flag : char { kExit, kBarrier, kResetWorkerInModel, kClock, kAdd, kGet };

struct Meta {
  Flag flag = Flag::kExit;
  int sender = -1;
  int recver = -1;
  int model_id = -1;
};

struct Message {
  Meta meta;
  std::vector<third_party::SArray<char>> data;

  template <typename V>
  void AddData(const third_party::SArray<V>& val) {
    data.push_back(third_party::SArray<char>(val));
  }
};

}  // namespace csci5570
