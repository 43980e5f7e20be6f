// pskv_oracle.cpp — TEST INFRASTRUCTURE ONLY.  CPU restatement of the
// reference's storage algorithms, used by tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg as the checker and the CPU baseline.  Nothing in
// the product (libpskv.so, include/, parameter_server_amd/) links or calls it.
//
// Parity pinning: the reference storages include glog/logging.h, which this
// image lacks, so the reference cannot be compiled here without a stand-in
// header (forbidden) — oracle/_ref is therefore not built.  This restatement is
// pinned instead by the reference's own known-answer tests
// (server/vector_storage_test.cpp:19-78, server/map_storage_test.cpp:19-75,
// base/range_partition_manager_test.cpp:17-56, the consistency-model tests)
// and by the reference probe outputs recorded in SURVEY.md §0, all committed as
// fixtures under tests/golden/ and checked by tests/test_oracle.py.
//
// Restated algorithms (same loops, same complexity, so the CPU timings are
// representative of the reference):
//   MapStorageRef     server/map_storage.hpp:17-45   std::map, assign, 0 if absent
//   VectorStorageRef  server/vector_storage.hpp:16-49 append on Add; Get scans every
//                     stored pair for every query, the LAST match wins, else 0
//   range slice       base/range_partition_manager.hpp:19-46
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

namespace {

template <typename V>
struct MapRef {
  std::map<uint32_t, V> storage;
  void add(const uint32_t* k, const V* v, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) storage[k[i]] = v[i];  // map_storage.hpp:22-23
  }
  void get(const uint32_t* k, uint64_t n, V* out) const {
    for (uint64_t i = 0; i < n; ++i) {  // map_storage.hpp:32-39
      auto it = storage.find(k[i]);
      out[i] = it != storage.end() ? it->second : V(0);
    }
  }
};

template <typename V>
struct VectorRef {
  // vector_storage.hpp:54-55 keeps keys as std::vector<int>; the comparison at
  // :36 converts back to unsigned, so uint32 storage is observably identical.
  std::vector<uint32_t> keys;
  std::vector<V> vals;
  void add(const uint32_t* k, const V* v, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) {  // vector_storage.hpp:21-29
      keys.push_back(k[i]);
      vals.push_back(v[i]);
    }
  }
  void get(const uint32_t* q, uint64_t n, V* out) const {
    for (uint64_t m = 0; m < n; ++m) out[m] = V(0);  // zero-filled reply (sarray.h resize)
    for (size_t i = 0; i < keys.size(); ++i)          // vector_storage.hpp:34-43
      for (uint64_t m = 0; m < n; ++m)
        if (keys[i] == q[m]) out[m] = vals[i];
  }
};

// dtype: 0 int32, 1 float, 2 double (same codes as pskv.h)
struct Handle {
  int kind;   // 0 map, 1 vector
  int dtype;
  void* impl;
};

template <template <typename> class S>
void* make(int dtype) {
  switch (dtype) {
    case 0: return new S<int32_t>();
    case 1: return new S<float>();
    case 2: return new S<double>();
  }
  return nullptr;
}

template <template <typename> class S>
void destroy(int dtype, void* p) {
  switch (dtype) {
    case 0: delete static_cast<S<int32_t>*>(p); break;
    case 1: delete static_cast<S<float>*>(p); break;
    case 2: delete static_cast<S<double>*>(p); break;
  }
}

template <template <typename> class S>
void add(int dtype, void* p, const uint32_t* k, const void* v, uint64_t n) {
  switch (dtype) {
    case 0: static_cast<S<int32_t>*>(p)->add(k, static_cast<const int32_t*>(v), n); break;
    case 1: static_cast<S<float>*>(p)->add(k, static_cast<const float*>(v), n); break;
    case 2: static_cast<S<double>*>(p)->add(k, static_cast<const double*>(v), n); break;
  }
}

template <template <typename> class S>
void get(int dtype, void* p, const uint32_t* k, uint64_t n, void* out) {
  switch (dtype) {
    case 0: static_cast<S<int32_t>*>(p)->get(k, n, static_cast<int32_t*>(out)); break;
    case 1: static_cast<S<float>*>(p)->get(k, n, static_cast<float*>(out)); break;
    case 2: static_cast<S<double>*>(p)->get(k, n, static_cast<double*>(out)); break;
  }
}

}  // namespace

extern "C" {

// kind: 0 = MapStorageRef, 1 = VectorStorageRef
void* oracle_create(int kind, int dtype) {
  if (dtype < 0 || dtype > 2 || kind < 0 || kind > 1) return nullptr;
  Handle* h = new Handle{kind, dtype, kind == 0 ? make<MapRef>(dtype) : make<VectorRef>(dtype)};
  return h;
}

void oracle_destroy(void* hp) {
  Handle* h = static_cast<Handle*>(hp);
  if (!h) return;
  if (h->kind == 0)
    destroy<MapRef>(h->dtype, h->impl);
  else
    destroy<VectorRef>(h->dtype, h->impl);
  delete h;
}

void oracle_add(void* hp, const uint32_t* keys, const void* vals, uint64_t n) {
  Handle* h = static_cast<Handle*>(hp);
  if (h->kind == 0)
    add<MapRef>(h->dtype, h->impl, keys, vals, n);
  else
    add<VectorRef>(h->dtype, h->impl, keys, vals, n);
}

void oracle_get(void* hp, const uint32_t* keys, uint64_t n, void* out) {
  Handle* h = static_cast<Handle*>(hp);
  if (h->kind == 0)
    get<MapRef>(h->dtype, h->impl, keys, n, out);
  else
    get<VectorRef>(h->dtype, h->impl, keys, n, out);
}

// Number of distinct keys held (map) or pairs appended (vector).
uint64_t oracle_size(void* hp) {
  Handle* h = static_cast<Handle*>(hp);
  if (h->kind == 0) {
    switch (h->dtype) {
      case 0: return static_cast<MapRef<int32_t>*>(h->impl)->storage.size();
      case 1: return static_cast<MapRef<float>*>(h->impl)->storage.size();
      default: return static_cast<MapRef<double>*>(h->impl)->storage.size();
    }
  }
  switch (h->dtype) {
    case 0: return static_cast<VectorRef<int32_t>*>(h->impl)->keys.size();
    case 1: return static_cast<VectorRef<float>*>(h->impl)->keys.size();
    default: return static_cast<VectorRef<double>*>(h->impl)->keys.size();
  }
}

// base/range_partition_manager.hpp:19-46, one pass with a forward-only range
// pointer: a key joins the current range if it lies in it or the current range
// is the last; otherwise the pointer advances and the key is re-examined.
// Writes the range index of every key; returns 0.
int oracle_range_assign(const uint64_t* rb, const uint64_t* re, int nr, const uint32_t* keys,
                        uint64_t n, int32_t* range_of_key) {
  int range = 0;
  for (uint64_t i = 0; i < n; ++i) {
    for (;;) {
      const uint64_t k = keys[i];
      if ((k >= rb[range] && k < re[range]) || range + 1 >= nr) {
        range_of_key[i] = range;
        break;
      }
      ++range;
    }
  }
  return 0;
}

}  // extern "C"
