// hip_storage_test.cpp — the reference's storage known-answer tests, restated
// against HipStorage<Val> through the AbstractStorage interface, the way a
// consistency model holds it (std::unique_ptr<AbstractStorage>,
// server/consistency/ssp_model.hpp:42).
//
//   AddGetInt / AddGetFloat / SubAddSubGet   server/vector_storage_test.cpp:19-78,
//                                            server/map_storage_test.cpp:19-75
//   LastWriteWins                            SURVEY.md §0.1 probe of both reference storages:
//                                            Add{5:1,5:2,7:3}; Add{7:10}; Get{5,7,9} -> {2,10,0}
//   SliceKeys / SliceKVs                     base/range_partition_manager_test.cpp:17-56
//   SliceFallthrough                         SURVEY.md §0.4 probes
//   FramedMessages                           SURVEY.md §8f-3: payloads received into page-locked
//                                            frames (ps/host_frames.hpp), read in place; the
//                                            frames dropped while their Adds may still be queued
//   CreateTableHip                           driver/engine.hpp:93-131 with StorageType::Hip
//                                            (ps/storage_factory.hpp): per-server ranges, the
//                                            last server also stores the fall-through keys
//
// Needs a GPU for the storage cases (run by tests/test_gpu_parity.py);
// `--host-only` runs the range-map cases alone.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <random>
#include <vector>

#include "ps/hip_storage.hpp"
#include "ps/host_frames.hpp"
#include "ps/consistent_hashing_partition_manager.hpp"
#include "ps/range_partition_manager.hpp"
#include "ps/storage_factory.hpp"

using namespace csci5570;

static int g_fail = 0, g_pass = 0;
#define EXPECT(cond)                                                            \
  do {                                                                          \
    if (cond) {                                                                 \
      ++g_pass;                                                                 \
    } else {                                                                    \
      ++g_fail;                                                                 \
      std::printf("  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);             \
    }                                                                           \
  } while (0)

template <typename V>
static void AddGet(const std::vector<V>& vals, const char* name) {
  std::printf("[ RUN ] %s\n", name);
  std::unique_ptr<AbstractStorage> s(new HipStorage<V>());
  Message m;
  third_party::SArray<Key> s_keys({13, 14, 15});
  third_party::SArray<V> s_vals(vals);
  m.AddData(s_keys);
  m.AddData(s_vals);
  s->Add(m);
  Message m2;
  m2.meta.sender = 7;
  m2.meta.recver = 1000;
  m2.meta.flag = Flag::kGet;
  m2.meta.model_id = 3;
  m2.AddData(s_keys);
  Message rep = s->Get(m2);
  EXPECT(rep.data.size() == 2);
  EXPECT(rep.meta.sender == 1000 && rep.meta.recver == 7);
  EXPECT(rep.meta.flag == Flag::kGet && rep.meta.model_id == 3);
  auto rep_keys = third_party::SArray<Key>(rep.data[0]);
  auto rep_vals = third_party::SArray<V>(rep.data[1]);
  EXPECT(rep_keys.size() == 3 && rep_vals.size() == 3);
  EXPECT(rep_keys.data() == s_keys.data());  // reply keys alias the request (abstract_storage.hpp:27)
  for (size_t i = 0; i < s_keys.size(); ++i) {
    EXPECT(rep_keys[i] == s_keys[i]);
    EXPECT(std::memcmp(&rep_vals[i], &s_vals[i], sizeof(V)) == 0);
  }
}

static void SubAddSubGet() {
  std::printf("[ RUN ] SubAddSubGet\n");
  HipStorage<float> s;
  third_party::SArray<Key> s_keys({13, 14, 15});
  third_party::SArray<float> s_vals({0.1f, 0.2f, 0.3f});
  s.SubAdd(s_keys, third_party::SArray<char>(s_vals));
  auto ret = third_party::SArray<float>(s.SubGet(s_keys));
  for (size_t i = 0; i < s_keys.size(); ++i) EXPECT(ret[i] == s_vals[i]);
  s.FinishIter();
}

template <typename V>
static void LastWriteWins(uint32_t key_begin, uint64_t key_end, const char* name) {
  std::printf("[ RUN ] %s [%u, %llu)\n", name, key_begin, (unsigned long long)key_end);
  std::unique_ptr<AbstractStorage> s(new HipStorage<V>(0, key_begin, key_end));
  {
    Message m;
    m.AddData(third_party::SArray<Key>({5, 5, 7}));
    m.AddData(third_party::SArray<V>({V(1), V(2), V(3)}));
    s->Add(m);
  }
  {
    Message m;
    m.AddData(third_party::SArray<Key>({7}));
    m.AddData(third_party::SArray<V>({V(10)}));
    s->Add(m);
  }
  Message g;
  g.AddData(third_party::SArray<Key>({5, 7, 9}));
  Message rep = s->Get(g);
  auto v = third_party::SArray<V>(rep.data[1]);
  EXPECT(v.size() == 3);
  EXPECT(v[0] == V(2) && v[1] == V(10) && v[2] == V(0));
  s->FinishIter();
}

static void SliceCases() {
  std::printf("[ RUN ] SliceKeys / SliceKVs / SliceFallthrough\n");
  {
    RangeShardMap pm({0, 1, 2}, {{2, 4}, {4, 7}, {7, 10}});
    std::vector<std::pair<int, RangeShardMap::Keys>> sl;
    pm.Slice(third_party::SArray<uint32_t>({2, 8, 9}), &sl);
    EXPECT(sl.size() == 2);
    EXPECT(sl[0].first == 0 && sl[1].first == 2);
    EXPECT(sl[0].second.size() == 1 && sl[0].second[0] == 2);
    EXPECT(sl[1].second.size() == 2 && sl[1].second[0] == 8 && sl[1].second[1] == 9);
  }
  {
    RangeShardMap pm({0, 1, 2}, {{0, 4}, {4, 8}, {8, 10}});
    std::vector<std::pair<int, RangeShardMap::Keys>> sl;
    pm.Slice(third_party::SArray<uint32_t>({2, 5, 9}), &sl);
    EXPECT(sl.size() == 3);
    for (int i = 0; i < 3; ++i) EXPECT(sl[i].first == i && sl[i].second.size() == 1);
  }
  {  // unsorted input misroutes: {5,1,9} over [0,4),[4,8),[8,12) -> srv1:5, srv2:1 9
    RangeShardMap pm({0, 1, 2}, {{0, 4}, {4, 8}, {8, 12}});
    std::vector<std::pair<int, RangeShardMap::Keys>> sl;
    pm.Slice(third_party::SArray<uint32_t>({5, 1, 9}), &sl);
    EXPECT(sl.size() == 2);
    EXPECT(sl[0].first == 1 && sl[0].second.size() == 1 && sl[0].second[0] == 5);
    EXPECT(sl[1].first == 2 && sl[1].second.size() == 2 && sl[1].second[0] == 1);
  }
  {  // below the first range falls to the last: [2,4),[4,8) keys {0,5} -> srv1: 0 5
    RangeShardMap pm({0, 1}, {{2, 4}, {4, 8}});
    std::vector<std::pair<int, RangeShardMap::Keys>> sl;
    pm.Slice(third_party::SArray<uint32_t>({0, 5}), &sl);
    EXPECT(sl.size() == 1 && sl[0].first == 1 && sl[0].second.size() == 2);
  }
}

// ConsistentHashShardMap (the Engine's default partitioner): the slices the
// reference's own test asserts, base/consistent_hashing_partition_manager_test.cpp:48-139
static void HashSliceCases() {
  std::printf("[ RUN ] HashSliceKeys / HashSliceKVs\n");
  ConsistentHashShardMap pm({0, 1, 2});
  {
    std::vector<std::pair<int, AbstractPartitionManager::Keys>> sl;
    pm.Slice(third_party::SArray<uint32_t>({2, 8, 9}), &sl);
    EXPECT(sl.size() == 2);
    EXPECT(sl[0].first == 0 && sl[0].second.size() == 2 && sl[0].second[0] == 2 && sl[0].second[1] == 8);
    EXPECT(sl[1].first == 2 && sl[1].second.size() == 1 && sl[1].second[0] == 9);
    pm.Slice(third_party::SArray<uint32_t>({2, 8, 9, 10, 11, 12, 13}), &sl);
    EXPECT(sl.size() == 3);
    EXPECT(sl[0].first == 0 && sl[0].second.size() == 3 && sl[0].second[2] == 13);
    EXPECT(sl[1].first == 2 && sl[1].second.size() == 3 && sl[1].second[0] == 9 && sl[1].second[1] == 10);
    EXPECT(sl[2].first == 1 && sl[2].second.size() == 1 && sl[2].second[0] == 12);
  }
  {
    std::vector<std::pair<int, AbstractPartitionManager::KVPairs>> sl;
    pm.Slice(std::make_pair(third_party::SArray<uint32_t>({2, 5, 9}), third_party::SArray<double>({.2, .5, .9})),
             &sl);
    EXPECT(sl.size() == 3);
    for (int i = 0; i < 3; ++i) EXPECT(sl[i].first == i && sl[i].second.first.size() == 1);
    EXPECT(sl[0].second.second[0] == .2 && sl[1].second.first[0] == 5 && sl[1].second.second[0] == .5);
  }
}

// Messages whose payloads sit in page-locked frames, as Mailbox::Recv delivers
// them after the §8f-3 change (RecvIntoFrame per data frame): Adds of 3 to
// 300 000 keys (sorted, unsorted with duplicates, out of range), each message
// dropped right after Add -- its frames return to the pool while the Add may
// still be queued -- and fresh frames of the same sizes scribbled over; then
// a framed Get against a host map.
template <typename V>
static void FramedMessages(const char* name) {
  std::printf("[ RUN ] %s\n", name);
  std::unique_ptr<AbstractStorage> s(new HipStorage<V>(0, 1000, 501000));
  std::mt19937 rng(11);
  std::map<uint32_t, V> want;
  const size_t sizes[] = {3, 1000, 5000, 70000, 300000};
  for (size_t n : sizes) {
    for (int form = 0; form < 2; ++form) {
      std::vector<uint32_t> k(n);
      std::vector<V> v(n);
      for (size_t i = 0; i < n; ++i) {
        k[i] = 900 + rng() % 500200;  // some below 1000 and past 501000: overflow keys
        v[i] = V(int(rng() % 2000) - 1000);
      }
      if (form == 0) std::sort(k.begin(), k.end());
      for (size_t i = 0; i < n; ++i) want[k[i]] = v[i];
      {
        Message m;
        m.meta.flag = Flag::kAdd;
        m.AddData(third_party::SArray<Key>(RecvIntoFrame(k.data(), n * sizeof(uint32_t))));
        m.AddData(RecvIntoFrame(v.data(), n * sizeof(V)));
        s->Add(m);
      }  // the message and its frames are gone; the Add may still be queued
      auto a = RecvIntoFrame(k.data(), n * sizeof(uint32_t));
      auto b = RecvIntoFrame(v.data(), n * sizeof(V));
      std::memset(a.data(), 0xA5, a.size());
      std::memset(b.data(), 0x5A, b.size());
    }
  }
  std::vector<uint32_t> q;
  for (uint32_t x = 0; x < 502000; x += 3) q.push_back(x);
  Message g;
  g.meta.flag = Flag::kGet;
  g.AddData(third_party::SArray<Key>(RecvIntoFrame(q.data(), q.size() * sizeof(uint32_t))));
  Message rep = s->Get(g);
  auto got = third_party::SArray<V>(rep.data[1]);
  EXPECT(got.size() == q.size());
  size_t bad = 0;
  for (size_t i = 0; i < q.size() && i < got.size(); ++i) {
    auto it = want.find(q[i]);
    const V w = it == want.end() ? V(0) : it->second;
    bad += std::memcmp(&got[i], &w, sizeof(V)) != 0;
  }
  EXPECT(bad == 0);
  s->FinishIter();
  uint64_t live = 0, cached = 0, held = 0;
  EXPECT(pskv_host_pool_stats(&live, &cached, &held) == PSKV_OK);
  EXPECT(held == 0);  // FinishIter synchronised the shard: every held frame is free
}

// CreateTable over three server threads: each server's HipStorage owns its
// range; keys the slicer routes to the last server beyond its range land in
// its overflow table.  Adds go through the models (ASP: immediate).
static void CreateTableHip() {
  std::printf("[ RUN ] CreateTableHip\n");
  RangeShardMap map({0, 1, 2}, {{0, 100}, {100, 200}, {200, 300}});
  std::vector<std::unique_ptr<ServerThread>> threads;
  for (uint32_t i = 0; i < 3; ++i) threads.emplace_back(new ServerThread(i));
  ReplyQueue replies;
  auto st = CreateTable<int>(threads, map, 7, ModelType::ASP, StorageType::Hip, 0, &replies);
  EXPECT(st.size() == 3);
  for (size_t i = 0; i < 3; ++i) {
    auto* hs = dynamic_cast<HipStorage<int>*>(st[i]);
    EXPECT(hs != nullptr);
    pskv_info info;
    EXPECT(pskv_shard_info(hs->shard(), &info) == PSKV_OK);
    EXPECT(info.key_begin == 100 * i && info.key_end == 100 * (i + 1));
  }
  // push {5, 150, 250, 4000} through the map and the models, then pull
  const std::vector<uint32_t> ks = {5, 150, 250, 4000};
  const std::vector<int> vs = {1, 2, 3, 4};
  std::vector<std::pair<int, RangeShardMap::Keys>> sl;
  third_party::SArray<uint32_t> ka(ks);
  map.Slice(ka, &sl);
  EXPECT(sl.size() == 3 && sl[2].second.size() == 2);  // 250 and 4000 -> the last server
  for (auto& s : sl) {
    const size_t off = s.second.data() - ka.data();
    Message m;
    m.meta.flag = Flag::kAdd;
    m.meta.model_id = 7;
    m.AddData(s.second);
    m.AddData(third_party::SArray<int>(std::vector<int>(vs.begin() + off, vs.begin() + off + s.second.size())));
    threads[s.first]->GetModel(7)->Add(m);
  }
  for (auto& s : sl) {
    Message m;
    m.meta.flag = Flag::kGet;
    m.meta.model_id = 7;
    m.meta.recver = s.first;
    m.AddData(s.second);
    threads[s.first]->GetModel(7)->Get(m);
  }
  std::vector<int> got;
  Message r;
  while (replies.Pop(&r)) {
    auto v = third_party::SArray<int>(r.data[1]);
    got.insert(got.end(), v.begin(), v.end());
  }
  EXPECT(got == vs);
}

int main(int argc, char** argv) {
  const bool host_only = argc > 1 && std::strcmp(argv[1], "--host-only") == 0;
  SliceCases();
  HashSliceCases();
  if (!host_only) {
    AddGet<int>({1, 2, 3}, "AddGetInt");
    AddGet<float>({0.1f, 0.2f, 0.3f}, "AddGetFloat");
    AddGet<double>({0.1, 0.2, 0.3}, "AddGetDouble");
    SubAddSubGet();
    LastWriteWins<int>(0, 1ull << 20, "LastWriteWinsInt");
    LastWriteWins<float>(0, 1ull << 20, "LastWriteWinsFloat");
    LastWriteWins<double>(6, 8, "LastWriteWinsDoubleOverflow");  // 5 and 9 live in the overflow table
    FramedMessages<float>("FramedMessagesFloat");
    FramedMessages<double>("FramedMessagesDouble");
    CreateTableHip();
  }
  std::printf("%d passed, %d failed\n", g_pass, g_fail);
  // every shard is gone; hand the cached page-locked frames back while the HIP
  // runtime is still up (not from a static destructor at exit)
  if (!host_only) (void)pskv_host_pool_trim();
  return g_fail ? 1 : 0;
}
