// ps/abstract_partition_manager.hpp — the worker-side slicing interface,
// restated from base/abstract_partition_manager.hpp:14-43: a partition manager
// owns the list of server thread ids and cuts a key batch (or a key/value batch,
// values carried as double) into <server id, slice> pairs.  RangeShardMap
// (ps/range_partition_manager.hpp) is the range implementation; KVClientTable
// (ps/kv_client_table.hpp) is the caller.
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

#include "ps/message.hpp"

namespace csci5570 {

class AbstractPartitionManager {
 public:
  using Keys = third_party::SArray<Key>;
  using KVPairs = std::pair<third_party::SArray<Key>, third_party::SArray<double>>;

  explicit AbstractPartitionManager(const std::vector<uint32_t>& server_thread_ids)
      : server_thread_ids_(server_thread_ids) {}
  virtual ~AbstractPartitionManager() = default;

  size_t GetNumServers() const { return server_thread_ids_.size(); }
  const std::vector<uint32_t>& GetServerThreadIds() const { return server_thread_ids_; }

  virtual void Slice(const Keys& keys, std::vector<std::pair<int, Keys>>* sliced) const = 0;
  virtual void Slice(const KVPairs& kvs, std::vector<std::pair<int, KVPairs>>* sliced) const = 0;

 protected:
  std::vector<uint32_t> server_thread_ids_;
};

}  // namespace csci5570
