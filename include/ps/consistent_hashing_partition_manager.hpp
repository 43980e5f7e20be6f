// ps/consistent_hashing_partition_manager.hpp — the reference Engine's DEFAULT
// partitioner (driver/engine.hpp:143-150), restated from
// base/consistent_hashing_partition_manager.hpp:9-90 over the pskv_jump_hash C
// entry point: every key goes to server_thread_ids[JumpHash(key, #servers)].
//
// Output order kept from the reference (its tests pin it,
// base/consistent_hashing_partition_manager_test.cpp:48-139): one slice per
// server that receives keys, slices in order of the server's FIRST appearance
// in the batch, keys (and values) in batch order inside a slice.  The
// reference finds a key's slice with a linear std::find_if per key (:28,59);
// here the buckets come from one pskv_jump_hash call and the slices are
// filled by a counting pass.
//
// Storage under this map: a hashed server receives keys from the whole key
// space, so its HipStorage covers [0, key_end) (CreateTable's ranges overload
// in ps/storage_factory.hpp); 288 GB of HBM holds even the full 2^32-key space
// (17.2 GB of float) per GPU.
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

#include "pskv.h"
#include "ps/abstract_partition_manager.hpp"

namespace csci5570 {

class ConsistentHashShardMap : public AbstractPartitionManager {
 public:
  explicit ConsistentHashShardMap(const std::vector<uint32_t>& server_thread_ids)
      : AbstractPartitionManager(server_thread_ids) {}

  void Slice(const Keys& keys, std::vector<std::pair<int, Keys>>* sliced) const override {
    sliced->clear();
    std::vector<int> order;
    std::vector<size_t> count;
    std::vector<int32_t> bucket = Buckets(keys, &order, &count);
    std::vector<Keys> out(count.size());
    std::vector<size_t> fill(count.size(), 0);
    for (int b : order) out[b] = Keys(count[b]);
    for (size_t i = 0; i < keys.size(); ++i) out[bucket[i]][fill[bucket[i]]++] = keys[i];
    for (int b : order) sliced->push_back(std::make_pair((int)server_thread_ids_[b], out[b]));
  }

  void Slice(const KVPairs& kvs, std::vector<std::pair<int, KVPairs>>* sliced) const override {
    sliced->clear();
    PS_CHECK(kvs.first.size() == kvs.second.size());
    std::vector<int> order;
    std::vector<size_t> count;
    std::vector<int32_t> bucket = Buckets(kvs.first, &order, &count);
    std::vector<KVPairs> out(count.size());
    std::vector<size_t> fill(count.size(), 0);
    for (int b : order) out[b] = std::make_pair(Keys(count[b]), third_party::SArray<double>(count[b]));
    for (size_t i = 0; i < kvs.first.size(); ++i) {
      const int b = bucket[i];
      out[b].first[fill[b]] = kvs.first[i];
      out[b].second[fill[b]++] = kvs.second[i];
    }
    for (int b : order) sliced->push_back(std::make_pair((int)server_thread_ids_[b], out[b]));
  }

 private:
  // Per-key bucket, the buckets in first-appearance order, and their sizes.
  std::vector<int32_t> Buckets(const Keys& keys, std::vector<int>* order, std::vector<size_t>* count) const {
    const int nb = (int)server_thread_ids_.size();
    PS_CHECK(nb > 0);
    std::vector<int32_t> bucket(keys.size());
    PS_CHECK(pskv_jump_hash(keys.data(), keys.size(), nb, bucket.data()) == PSKV_OK);
    count->assign(nb, 0);
    for (int32_t b : bucket)
      if ((*count)[b]++ == 0) order->push_back(b);
    return bucket;
  }
};

}  // namespace csci5570
