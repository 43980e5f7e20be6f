// ps/storage_factory.hpp — table construction of Engine::CreateTable
// (driver/engine.hpp:93-131), restated with the HBM storage type:
// for every server thread, one storage and one consistency model, registered
// under the table id.  StorageType::Hip places server i's shard on GPU
// i % device_count with the key range the range map gives server i, so server
// thread i drives GPU i on a node with one server thread per GPU
// (simple_id_mapper.cpp:20-37).
//
// StorageType::Map / ::Vector are the reference's CPU storages: inside the
// reference tree (PSKV_IN_REFERENCE_TREE) they construct MapStorage /
// VectorStorage as CreateTable does; standalone, the caller supplies them
// (the tests pass the oracle restatement), since the CPU storages are not part
// of this package.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "ps/consistency.hpp"
#include "ps/consistent_hashing_partition_manager.hpp"
#include "ps/hip_storage.hpp"
#include "ps/range_partition_manager.hpp"
#include "ps/server_thread.hpp"

#ifdef PSKV_IN_REFERENCE_TREE
#include "server/map_storage.hpp"
#include "server/vector_storage.hpp"
#endif

namespace csci5570 {

enum class StorageType { Map, Vector, Hip };  // driver/engine.hpp:25, plus Hip
enum class ModelType { SSP, BSP, ASP };       // driver/engine.hpp:24

using CpuStorageMaker = std::function<std::unique_ptr<AbstractStorage>(StorageType)>;

using KeyRange = std::pair<uint64_t, uint64_t>;  // [begin, end), end <= 2^32

// The storage of the i-th server, owning key range r (server order = the
// partition manager's server order).
template <typename Val>
std::unique_ptr<AbstractStorage> MakeStorage(StorageType type, const KeyRange& r, size_t i,
                                             int mode = PSKV_ASSIGN,
                                             const CpuStorageMaker& cpu = nullptr) {
  if (type == StorageType::Hip) {
    const int ndev = pskv_device_count();
    PS_CHECK(ndev > 0);
    return std::unique_ptr<AbstractStorage>(
        new HipStorage<Val>((int)(i % (size_t)ndev), (uint32_t)r.first, r.second, mode));
  }
#ifdef PSKV_IN_REFERENCE_TREE
  if (type == StorageType::Map) return std::unique_ptr<AbstractStorage>(new MapStorage<Val>());
  return std::unique_ptr<AbstractStorage>(new VectorStorage<Val>());
#else
  PS_CHECK(cpu != nullptr);  // standalone: the CPU storages come from the caller
  return cpu(type);
#endif
}

inline std::unique_ptr<AbstractModel> MakeModel(ModelType type, uint32_t model_id,
                                                std::unique_ptr<AbstractStorage>&& storage,
                                                int staleness, ReplyQueue* replies) {
  switch (type) {
    case ModelType::SSP:
      return std::unique_ptr<AbstractModel>(new SSPModel(model_id, std::move(storage), staleness, replies));
    case ModelType::BSP:
      return std::unique_ptr<AbstractModel>(new BSPModel(model_id, std::move(storage), replies));
    default:
      return std::unique_ptr<AbstractModel>(new ASPModel(model_id, std::move(storage), replies));
  }
}

// Engine::CreateTable for a group of server threads: threads[i] gets a storage
// owning ranges[i] and a consistency model.  Returns the storages (still owned
// by the models) in server order, for inspection.
template <typename Val>
std::vector<AbstractStorage*> CreateTable(std::vector<std::unique_ptr<ServerThread>>& threads,
                                          const std::vector<KeyRange>& ranges, uint32_t model_id,
                                          ModelType model_type, StorageType storage_type,
                                          int staleness, ReplyQueue* replies,
                                          int mode = PSKV_ASSIGN,
                                          const CpuStorageMaker& cpu = nullptr) {
  PS_CHECK(threads.size() == ranges.size());
  std::vector<AbstractStorage*> out;
  for (size_t i = 0; i < threads.size(); ++i) {
    auto st = MakeStorage<Val>(storage_type, ranges[i], i, mode, cpu);
    out.push_back(st.get());
    threads[i]->RegisterModel(model_id, MakeModel(model_type, model_id, std::move(st), staleness, replies));
  }
  return out;
}

// Range partitioning (base/range_partition_manager.hpp): server i owns map range i.
template <typename Val>
std::vector<AbstractStorage*> CreateTable(std::vector<std::unique_ptr<ServerThread>>& threads,
                                          const RangeShardMap& map, uint32_t model_id,
                                          ModelType model_type, StorageType storage_type,
                                          int staleness, ReplyQueue* replies,
                                          int mode = PSKV_ASSIGN,
                                          const CpuStorageMaker& cpu = nullptr) {
  PS_CHECK(threads.size() == map.GetNumServers());
  std::vector<KeyRange> ranges;
  for (size_t i = 0; i < threads.size(); ++i) ranges.push_back(map.GetRange(i));
  return CreateTable<Val>(threads, ranges, model_id, model_type, storage_type, staleness, replies, mode,
                          cpu);
}

// Consistent hashing (the reference default, driver/engine.hpp:143-150): any
// server may receive any key below key_end, so every storage covers
// [0, key_end).
template <typename Val>
std::vector<AbstractStorage*> CreateTable(std::vector<std::unique_ptr<ServerThread>>& threads,
                                          const ConsistentHashShardMap& map, uint64_t key_end,
                                          uint32_t model_id, ModelType model_type,
                                          StorageType storage_type, int staleness, ReplyQueue* replies,
                                          int mode = PSKV_ASSIGN,
                                          const CpuStorageMaker& cpu = nullptr) {
  PS_CHECK(threads.size() == map.GetNumServers());
  std::vector<KeyRange> ranges(threads.size(), KeyRange(0, key_end));
  return CreateTable<Val>(threads, ranges, model_id, model_type, storage_type, staleness, replies, mode,
                          cpu);
}

}  // namespace csci5570
