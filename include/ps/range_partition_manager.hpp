// ps/range_partition_manager.hpp — the range shard map, mirroring
// RangePartitionManager (base/range_partition_manager.hpp:14-77) through the
// pskv_range_slice C entry point.  Device d of a G-GPU node owns range d; the
// last range also receives every key the forward-only walk cannot place
// (keys beyond all ranges, and out-of-order keys), exactly as the reference.
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

#include "pskv.h"
#include "ps/sarray.hpp"

namespace csci5570 {

class RangeShardMap {
 public:
  using Keys = third_party::SArray<uint32_t>;
  RangeShardMap(std::vector<uint32_t> server_thread_ids,
                std::vector<std::pair<uint64_t, uint64_t>> ranges)
      : ids_(std::move(server_thread_ids)) {
    for (auto& r : ranges) {
      rb_.push_back(r.first);
      re_.push_back(r.second);
    }
  }

  size_t GetNumServers() const { return ids_.size(); }
  const std::vector<uint32_t>& GetServerThreadIds() const { return ids_; }
  // Key range [begin, end) of the i-th server (in server order).
  std::pair<uint64_t, uint64_t> GetRange(size_t i) const { return std::make_pair(rb_[i], re_[i]); }

  // Zero-copy slices (segments of `keys`), in server order.
  void Slice(const Keys& keys, std::vector<std::pair<int, Keys>>* sliced) const {
    sliced->clear();
    std::vector<int32_t> r(rb_.size());
    std::vector<uint64_t> s(rb_.size()), n(rb_.size());
    const int ns = pskv_range_slice(rb_.data(), re_.data(), (int)rb_.size(), keys.data(),
                                    keys.size(), r.data(), s.data(), n.data());
    for (int i = 0; i < ns; ++i)
      sliced->push_back(std::make_pair((int)ids_[r[i]], keys.segment(s[i], s[i] + n[i])));
  }

 private:
  std::vector<uint32_t> ids_;
  std::vector<uint64_t> rb_, re_;
};

}  // namespace csci5570
