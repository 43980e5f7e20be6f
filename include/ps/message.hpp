// ps/message.hpp — clean-room restatement of the payload types that cross the
// storage boundary: Key (base/magic.hpp:7), Flag / Meta / Message
// (base/message.hpp:14-58).
#pragma once

#include <cstdint>
#include <vector>

#include "ps/sarray.hpp"

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
