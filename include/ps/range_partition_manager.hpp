// ps/range_partition_manager.hpp — the range shard map, mirroring
// RangePartitionManager (base/range_partition_manager.hpp:14-77) through the
// pskv_range_slice C entry point.  Device d of a G-GPU node owns range d; the
// last range also receives every key the forward-only walk cannot place
// (keys beyond all ranges, and out-of-order keys), exactly as the reference.
// Slices are zero-copy segments of the caller's arrays (the reference copies
// them key by key with push_back, :33,37).
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

#include "pskv.h"
#include "ps/abstract_partition_manager.hpp"

namespace csci5570 {

class RangeShardMap : public AbstractPartitionManager {
 public:
  RangeShardMap(std::vector<uint32_t> server_thread_ids,
                std::vector<std::pair<uint64_t, uint64_t>> ranges)
      : AbstractPartitionManager(server_thread_ids) {
    for (auto& r : ranges) {
      rb_.push_back(r.first);
      re_.push_back(r.second);
    }
  }

  // Key range [begin, end) of the i-th server (in server order).
  std::pair<uint64_t, uint64_t> GetRange(size_t i) const { return std::make_pair(rb_[i], re_[i]); }

  // Zero-copy slices (segments of `keys`), in server order.
  void Slice(const Keys& keys, std::vector<std::pair<int, Keys>>* sliced) const override {
    sliced->clear();
    for (auto& c : Cuts(keys)) sliced->push_back(std::make_pair(c.server, keys.segment(c.b, c.e)));
  }

  // The same cut applied to the values (range_partition_manager.hpp:48-77).
  void Slice(const KVPairs& kvs, std::vector<std::pair<int, KVPairs>>* sliced) const override {
    sliced->clear();
    PS_CHECK(kvs.first.size() == kvs.second.size());
    for (auto& c : Cuts(kvs.first))
      sliced->push_back(std::make_pair(
          c.server, std::make_pair(kvs.first.segment(c.b, c.e), kvs.second.segment(c.b, c.e))));
  }

 private:
  struct Cut {
    int server;
    size_t b, e;
  };
  std::vector<Cut> Cuts(const Keys& keys) const {
    std::vector<int32_t> r(rb_.size());
    std::vector<uint64_t> s(rb_.size()), n(rb_.size());
    const int ns = pskv_range_slice(rb_.data(), re_.data(), (int)rb_.size(), keys.data(),
                                    keys.size(), r.data(), s.data(), n.data());
    std::vector<Cut> out;
    for (int i = 0; i < ns; ++i)
      out.push_back(Cut{(int)server_thread_ids_[r[i]], (size_t)s[i], (size_t)(s[i] + n[i])});
    return out;
  }
  std::vector<uint64_t> rb_, re_;
};

}  // namespace csci5570
