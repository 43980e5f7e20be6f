// pskv_kernels.hip — CDNA4 (gfx950) kernels of the parameter-shard Add/Get path.
//
// The reference does this work in libstdc++ containers on one CPU thread per
// server (server/map_storage.hpp:17-45, server/vector_storage.hpp:16-49).  These
// kernels are new, written for MI355X: 64-lane waves, 16-byte-per-lane HBM
// accesses, LDS for per-workgroup duplicate resolution, no atomics on the
// sorted path, and grouped launches so many push/pull batches share one
// dispatch.  The work is HBM-bound byte movement (no MFMA); DESIGN.md prices
// every kernel against the 8 TB/s HBM roofline.
//
//   K1  k_gather          Get: out[i] = value(keys[i])                 (map_storage.hpp:29-45)
//   K2  k_assign_sorted   Add, one batch, sorted keys: the last element of
//                         each equal-key run stores, nothing else does
//   K2g k_assign_group    Add, grouped sorted batches: one workgroup owns a
//                         key tile and applies the batches in call order
//   K4a k_general_mark    Add, any order: per-workgroup LDS hash dedup, then
//                         (assign) u64 last-writer stamps / (accumulate) one
//                         atomic add per distinct key per workgroup
//   K4b k_general_commit  Add, any order: the stamped winner of each key stores
//   K5  k_rb_bin/resolve  Add, any order: key buckets, no global atomics
//   K6  k_dense_check     accumulate: prove every batch a dense in-range window
//   K7  k_acc_dense       accumulate over dense windows: one RMW per key, sums in
//                         call order, no atomics
//
// Semantics restated from the reference: last write wins within a call (index
// order) and across calls (stream order) — map_storage.hpp:22-23 assigns in a
// sequential loop; vector_storage.hpp:34-43 returns the LAST appended match.
// A never-written key reads 0 (map_storage.hpp:33-37).
#include <type_traits>

#include "pskv_internal.h"

namespace pskv {
namespace {

// ---------------------------------------------------------------- helpers

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// 16-byte accesses through clang vector types; NT = non-temporal (streamed
// once: keys/values of a push, outputs of a pull).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const void* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<const u32x4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st16(void* p, u32x4 v) {
  if (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  else
    *reinterpret_cast<u32x4*>(p) = v;
}

// A 16-byte load from a DWORD-aligned address (global_load_dwordx4 needs only
// dword alignment): K5b reads 8-byte run entries two at a time from any entry.
typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
template <bool NT>
__device__ __forceinline__ void ld16a4(const uint32_t* p, uint32_t (&v)[4]) {
  const u32x4 t = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4a4*>(p))
                     : *reinterpret_cast<const u32x4a4*>(p);
  v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}
// ... and a 16-byte STORE to a dword-aligned address (K2g's own-range chunks store
// a window's elements where they land, whatever the window's phase).
template <bool NT>
__device__ __forceinline__ void st16a4(uint32_t* p, const uint32_t (&v)[4]) {
  const u32x4 t = u32x4{v[0], v[1], v[2], v[3]};
  if (NT)
    __builtin_nontemporal_store(t, reinterpret_cast<u32x4a4*>(p));
  else
    *reinterpret_cast<u32x4a4*>(p) = t;
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ void ld8_keys(const uint32_t* p, uint32_t (&k)[2]) {
  const u32x2 t = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p))
                     : *reinterpret_cast<const u32x2*>(p);
  k[0] = t.x;
  k[1] = t.y;
}

// Two 8-byte values as one 16-byte access.  Streams of 8-byte values go two
// per lane (a wave covers 1 KiB contiguously per instruction) rather than four
// per lane as two 16-byte accesses 32 bytes apart (each instruction then
// touches every line of a 2 KiB span for half its bytes).
struct Vec2x8 {
  using T = unsigned long long;
  template <bool NT = false>
  static __device__ __forceinline__ void load(const T* p, T (&v)[2]) {
    const u32x4 a = ld16<NT>(p);
    v[0] = (T)a.x | ((T)a.y << 32);
    v[1] = (T)a.z | ((T)a.w << 32);
  }
  template <bool NT = false>
  static __device__ __forceinline__ void store(T* p, const T (&v)[2]) {
    st16<NT>(p, u32x4{(uint32_t)v[0], (uint32_t)(v[0] >> 32), (uint32_t)v[1], (uint32_t)(v[1] >> 32)});
  }
};

template <typename VT>
struct Vec4;

template <>
struct Vec4<uint32_t> {
  template <bool NT = false>
  static __device__ __forceinline__ void load(const uint32_t* p, uint32_t (&v)[4]) {
    const u32x4 t = ld16<NT>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  template <bool NT = false>
  static __device__ __forceinline__ void store(uint32_t* p, const uint32_t (&v)[4]) {
    st16<NT>(p, u32x4{v[0], v[1], v[2], v[3]});
  }
};

template <>
struct Vec4<unsigned long long> {
  using T = unsigned long long;
  template <bool NT = false>
  static __device__ __forceinline__ void load(const T* p, T (&v)[4]) {
    const u32x4 a = ld16<NT>(p), b = ld16<NT>(p + 2);
    v[0] = (T)a.x | ((T)a.y << 32); v[1] = (T)a.z | ((T)a.w << 32);
    v[2] = (T)b.x | ((T)b.y << 32); v[3] = (T)b.z | ((T)b.w << 32);
  }
  template <bool NT = false>
  static __device__ __forceinline__ void store(T* p, const T (&v)[4]) {
    st16<NT>(p, u32x4{(uint32_t)v[0], (uint32_t)(v[0] >> 32), (uint32_t)v[1], (uint32_t)(v[1] >> 32)});
    st16<NT>(p + 2, u32x4{(uint32_t)v[2], (uint32_t)(v[2] >> 32), (uint32_t)v[3], (uint32_t)(v[3] >> 32)});
  }
};

// The widest lane layout of a value stream: N values per 16-byte access.
template <typename BT>
struct VecN;
template <>
struct VecN<uint32_t> : Vec4<uint32_t> {
  static constexpr int N = 4;
};
template <>
struct VecN<unsigned long long> : Vec2x8 {
  static constexpr int N = 2;
};

// Which batch of a grouped launch this workgroup serves: the last batch whose
// first workgroup is at or before `wg` (the prefix table in the kernarg
// segment is non-decreasing; empty batches repeat a prefix; nb <= 64).  A
// binary search: at most 6 dependent scalar loads, where a scan that stops at
// the batch waits for one per batch it passes (~63 for the last batch of a
// full group) before the workgroup's first memory access.  (Loading the whole
// table at once needs ~100 SGPRs and costs the gather a wave per SIMD.)
// Group-wide index of batch j's first element (the K4 stamps' element index):
// a scalar sum over the batches before it (the kernarg segment holds no prefix
// table: 512 B less to copy per launch, for the stamps variant only).
__device__ __forceinline__ uint64_t elem_prefix(const GroupArgs& ga, int j) {
  uint64_t e = 0;
  for (int i = 0; i < j; ++i) e += ga.b[i].n;
  return e;
}

__device__ __forceinline__ int batch_of(const GroupArgs& ga, uint32_t wg) {
  int lo = 0, hi = ga.nb;  // prefix[lo] <= wg (prefix[0] = 0); the answer is < hi
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (ga.wg_prefix[mid] <= wg)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// ------------------------------------------------------- overflow table
// Open addressing with linear probing over u64 slots (EMPTY = ~0, so every
// uint32 key is storable).  Keys are never deleted, so a non-EMPTY slot read
// without an atomic is final; a stale EMPTY is resolved by the CAS.

template <typename T>
__device__ __forceinline__ T sys_load(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ T agent_load(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// (readfirstlane returns int: each half goes through uint32_t, or a low word
// with its top bit set would sign-extend over the high word)
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// The table's current arrays, read from the control block (wave-uniform: kept
// in scalar registers).  FRESH: agent-scope loads, for a kernel in which a
// workgroup may have grown the table and switched the block over (the replays
// K4r / K1r, K5b, K8, K9): they reach L2 past any line an earlier read left
// in the CU.  Otherwise plain loads (the caches start clean at every launch).
template <bool FRESH = true>
__device__ __forceinline__ OvfTab ovf_tab(const Ovf& o) {
  OvfTab t;
  if (FRESH) {
    t.keys = reinterpret_cast<unsigned long long*>(
        uniform64(agent_load(reinterpret_cast<const uint64_t*>(&o.c->t.keys))));
    t.vals = reinterpret_cast<void*>(uniform64(agent_load(reinterpret_cast<const uint64_t*>(&o.c->t.vals))));
    t.mask = uniform64(agent_load(&o.c->t.mask));
  } else {
    t = o.c->t;
  }
  return t;
}

__device__ __forceinline__ long long ovf_find(const OvfTab& t, uint32_t key) {
  uint64_t h = fmix32(key) & t.mask;
  for (uint64_t p = 0; p <= t.mask; ++p) {
    const unsigned long long k = t.keys[h];
    if (k == (unsigned long long)key) return (long long)h;
    if (k == kEmpty64) return -1;
    h = (h + 1) & t.mask;
  }
  return -1;
}

// Insert (or find) `key`; counts a new key in stat[0].  A full table sets the
// sticky error bit: only a caller that skipped ovf_reserve can get there (the
// grow service did not answer within the wait bound, or its allocation failed).
__device__ long long ovf_insert(const OvfTab& t, uint32_t* stat, uint32_t key) {
  uint64_t h = fmix32(key) & t.mask;
  for (uint64_t p = 0; p <= t.mask; ++p) {
    const unsigned long long k = t.keys[h];
    if (k == (unsigned long long)key) return (long long)h;
    if (k == kEmpty64) {
      const unsigned long long old = atomicCAS(&t.keys[h], kEmpty64, (unsigned long long)key);
      if (old == kEmpty64) {
        atomicAdd(&stat[0], 1u);
        return (long long)h;
      }
      if (old == (unsigned long long)key) return (long long)h;
    }
    h = (h + 1) & t.mask;
  }
  atomicOr(&stat[1], kErrOverflowFull);
  return -1;
}
__device__ __forceinline__ long long ovf_insert(const Ovf& o, const OvfTab& t, uint32_t key) {
  return ovf_insert(t, o.c->stat, key);
}

// A key's slot in a table being filled by a rehash (room for every key, keys
// distinct): no count, no error.
__device__ __forceinline__ long long ovf_place(const OvfTab& t, uint32_t key) {
  uint64_t h = fmix32(key) & t.mask;
  for (;;) {
    const unsigned long long old = atomicCAS(&t.keys[h], kEmpty64, (unsigned long long)key);
    if (old == kEmpty64 || old == (unsigned long long)key) return (long long)h;
    h = (h + 1) & t.mask;
  }
}

// VB value bytes of slot i, copied (agent-scope loads: the values were stored
// by this workgroup earlier in the kernel, possibly behind a stale CU line).
template <int VB>
__device__ __forceinline__ void ovf_copy_val(const OvfTab& from, uint64_t i, const OvfTab& to, long long s) {
  if (VB == 8)
    reinterpret_cast<unsigned long long*>(to.vals)[s] =
        agent_load(reinterpret_cast<const unsigned long long*>(from.vals) + i);
  else
    reinterpret_cast<uint32_t*>(to.vals)[s] = agent_load(reinterpret_cast<const uint32_t*>(from.vals) + i);
}

// ---- growth on the device (round 6).  The reference's last range server
// stores every key the slicer cannot place, however many
// (range_partition_manager.hpp:26-27, map_storage.hpp:22-23).  A device-side
// Add's keys are never read on the host, so the table cannot be sized before
// the kernels run; instead every out-of-range insert happens in ONE workgroup
// (the replays K4r / K1r, the out-of-range bucket of K5b, K8, K9), which
// reserves room before each pass: when the pass could lift the load above 3/4,
// thread 0 posts a request to the shard's mailbox (coherent host memory) and
// polls for the answer; the library's grow service (a host thread) allocates
// arrays of the asked size and answers; the workgroup fills them, rehashes the
// table into them, switches the control block over and goes on.  Later
// kernels read the block, so work queued before the growth uses the new table.
// The wait is bounded (mailbox wait_ticks, from SYNC_TIMEOUT_MS): without an
// answer the workgroup goes on with the old table, and an insert that finds it
// full sets the sticky error (pskv_sync: PSKV_ESTATE), as before round 6.

// Thread 0: ask the grow service for `cap` slots; true with the new arrays in *out.
__device__ bool ovf_request(OvfMbox* m, uint64_t cap, OvfTab* out) {
  if (m == nullptr) return false;
  const uint32_t seq = sys_load(&m->req_seq) + 1u;
  __hip_atomic_store(&m->req_cap, cap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&m->req_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long t0 = wall_clock64(), lim = sys_load(&m->wait_ticks);
  for (;;) {
    if (__hip_atomic_load(&m->resp_seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == seq) break;
    if (wall_clock64() - t0 > lim) return false;
    __builtin_amdgcn_s_sleep(16);
  }
  if (sys_load(&m->resp_ok) == 0u) return false;
  out->keys = reinterpret_cast<unsigned long long*>(sys_load(reinterpret_cast<const uint64_t*>(&m->resp_tab.keys)));
  out->vals = reinterpret_cast<void*>(sys_load(reinterpret_cast<const uint64_t*>(&m->resp_tab.vals)));
  out->mask = sys_load(&m->resp_tab.mask);
  return out->keys != nullptr && out->vals != nullptr && out->mask + 1 == cap;
}

// Every thread of the workgroup, uniformly: make room for `extra` more keys
// (load <= 3/4 after them), growing the table if needed.  Orders every earlier
// insert of the workgroup before it (barrier).  VB: value bytes.
template <int VB>
__device__ void ovf_reserve(const Ovf& o, uint64_t extra) {
  __shared__ OvfTab s_new;
  __shared__ uint32_t s_go;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t go = 0;
    const OvfTab t = ovf_tab(o);
    const uint64_t cap = t.mask + 1;
    const uint64_t cnt = agent_load(&o.c->stat[0]);
    if (4 * (cnt + extra) > 3 * cap) {
      uint64_t want = 2 * cap;
      while (want < 2 * (cnt + extra)) want <<= 1;
      OvfTab n;
      if (ovf_request(o.c->mbox, want, &n)) {
        s_new = n;
        go = 1;
      }
    }
    s_go = go;
  }
  __syncthreads();
  if (!s_go) return;  // uniform
  const OvfTab from = ovf_tab(o);
  OvfTab to;  // (scalar registers: the caller's live values keep the vector ones)
  to.keys = reinterpret_cast<unsigned long long*>(uniform64(reinterpret_cast<uint64_t>(s_new.keys)));
  to.vals = reinterpret_cast<void*>(uniform64(reinterpret_cast<uint64_t>(s_new.vals)));
  to.mask = uniform64(s_new.mask);
  for (uint64_t i = threadIdx.x; i <= to.mask; i += blockDim.x) {
    to.keys[i] = kEmpty64;
    if (VB == 8)
      reinterpret_cast<unsigned long long*>(to.vals)[i] = 0ull;
    else
      reinterpret_cast<uint32_t*>(to.vals)[i] = 0u;
  }
  __threadfence();
  __syncthreads();
  for (uint64_t i = threadIdx.x; i <= from.mask; i += blockDim.x) {
    const unsigned long long k = agent_load(from.keys + i);
    if (k == kEmpty64) continue;
    ovf_copy_val<VB>(from, i, to, ovf_place(to, (uint32_t)k));
  }
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(&o.c->t.keys), reinterpret_cast<uint64_t>(to.keys),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<uint64_t*>(&o.c->t.vals), reinterpret_cast<uint64_t>(to.vals),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&o.c->t.mask, to.mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __threadfence();
  __syncthreads();
}

template <typename VT, bool FRESH = false>
__device__ __forceinline__ VT load_one(const DenseView& d, const Ovf& o, uint32_t key) {
  const uint32_t off = key - d.key_begin;
  if ((uint64_t)off < d.range) return reinterpret_cast<const VT*>(d.param)[off];
  const OvfTab t = ovf_tab<FRESH>(o);
  const long long s = ovf_find(t, key);
  return s >= 0 ? reinterpret_cast<const VT*>(t.vals)[s] : VT(0);
}

// An empty asm that reads x: the compiler's wait-count pass must have x's loads
// complete here.  Used to place the wait for a software-pipelined register set
// before the next set's loads are issued (see k_rb_bin, k_rb_resolve).
template <typename T, int N>
__device__ __forceinline__ void ready(const T (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" ::"v"(x[i]));
}

// Diagnostic build only (-DPSKV_STEP_STAMPS, tools/step_stamps.py): the
// real-time clock (s_memrealtime, 100 MHz, one clock for every XCD) at phase
// boundaries of every workgroup of the dense Add (K2g) and the Get (K1) of the
// most recent launch: [kernel][workgroup][phase], phase 0 = entry; K2g: 1 =
// prologue published, 2 = first chunk verified, 3 = last store issued; K1: 1 =
// keys loaded, 2 = last store issued.  Read back by pskv_diag_step_stamps.
#ifdef PSKV_STEP_STAMPS
__device__ unsigned long long g_step_stamps[2][8192][4];
#define STEP_STAMP(K, PH) \
  if (threadIdx.x == 0 && blockIdx.x < 8192u) g_step_stamps[K][blockIdx.x][PH] = __builtin_amdgcn_s_memrealtime()
#else
#define STEP_STAMP(K, PH) (void)0
#endif

// ------------------------------------------------------------- K1 gather

// Four keys of one lane: when they are four consecutive in-range keys (dense
// pulls), ONE 16-byte parameter load serves them, from a dword-aligned address
// when the run starts off a 16-byte slot (a pulled window may start at any
// key; cfg 4's producer windows do); otherwise four scalar gathers.  (Round 3
// loaded the two slots such a run straddles and selected: K1 ran 4-6 % slower
// at phases 1-3 than at phase 0, `profiles/r03_probes/align_probe_own_range.log`.)
template <typename VT, bool NTP = false, bool FRESH = false>
__device__ __forceinline__ void gather4(const DenseView& d, const Ovf& o, const uint32_t (&k)[4],
                                        VT (&v)[4]) {
  const uint32_t off0 = k[0] - d.key_begin;
  const bool run = (k[1] == k[0] + 1u) & (k[2] == k[0] + 2u) & (k[3] == k[0] + 3u) &
                   ((uint64_t)off0 + 3u < d.range);
  if (run && (off0 & 3u) == 0u) {
    Vec4<VT>::template load<NTP>(reinterpret_cast<const VT*>(d.param) + off0, v);
  } else if (sizeof(VT) == 4 && run) {
    uint32_t t[4];
    ld16a4<NTP>(reinterpret_cast<const uint32_t*>(d.param) + off0, t);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (VT)t[e];
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = load_one<VT, FRESH>(d, o, k[e]);
  }
}

// Two keys of one lane, 8-byte values: one 16-byte load when they are two
// consecutive in-range keys, from a dword-aligned address on an odd offset.
template <bool FRESH = false>
__device__ __forceinline__ void gather2(const DenseView& d, const Ovf& o, const uint32_t (&k)[2],
                                        unsigned long long (&v)[2]) {
  using T = unsigned long long;
  const uint32_t off0 = k[0] - d.key_begin;
  const bool run = (k[1] == k[0] + 1u) & ((uint64_t)off0 + 1u < d.range);
  if (run && (off0 & 1u) == 0u) {
    Vec2x8::load(reinterpret_cast<const T*>(d.param) + off0, v);
  } else if (run) {
    uint32_t t[4];
    ld16a4<false>(reinterpret_cast<const uint32_t*>(reinterpret_cast<const T*>(d.param) + off0), t);
    v[0] = (T)t[0] | ((T)t[1] << 32);
    v[1] = (T)t[2] | ((T)t[3] << 32);
  } else {
    v[0] = load_one<T, FRESH>(d, o, k[0]);
    v[1] = load_one<T, FRESH>(d, o, k[1]);
  }
}

// One K1 chunk (CH = 1024 * U keys of one batch): chunk `wg` of the group.
// go() is asked once, after the chunk's key loads are issued and before any
// parameter is read: false abandons the chunk (K1r's tag check, whose scalar
// load then waits behind the key loads instead of in front of them).
struct GoAlways {
  __device__ bool operator()() const { return true; }
};
template <typename VT, bool VEC, int U, bool NT, typename Go = GoAlways, bool FRESH = false>
__device__ __forceinline__ void gather_chunk(const GroupArgs& ga, const DenseView& d, const Ovf& o,
                                             uint32_t wg, Go go = Go()) {
  constexpr int CH = kBlock * 4 * U;
  const int j = batch_of(ga, wg);
  const uint32_t* __restrict__ keys = ga.b[j].keys;
  VT* __restrict__ out = reinterpret_cast<VT*>(const_cast<void*>(ga.b[j].vals));
  const uint64_t n = ga.b[j].n;
  const uint64_t base = (uint64_t)(wg - ga.wg_prefix[j]) * CH;
  const int tid = threadIdx.x;
  if constexpr (sizeof(VT) == 8) {
    if (VEC && base + CH <= n) {
      // two keys per lane per step (see Vec2x8): 8-byte key loads, 16-byte
      // value loads and stores, every instruction one contiguous span.  (A
      // form with 16-byte key loads and values moved as pairs over each wave's
      // span measured no faster and needed 202 VGPRs against 80.)
      constexpr int UU = 2 * U;
      uint32_t k[UU][2];
#pragma unroll
      for (int u = 0; u < UU; ++u) ld8_keys<NT>(keys + base + (uint64_t)(u * kBlock + tid) * 2, k[u]);
      if (!go()) return;
      VT v[UU][2];
#pragma unroll
      for (int u = 0; u < UU; ++u) gather2<FRESH>(d, o, k[u], v[u]);
#pragma unroll
      for (int u = 0; u < UU; ++u) Vec2x8::store<NT>(out + base + (uint64_t)(u * kBlock + tid) * 2, v[u]);
      return;
    }
  }
  STEP_STAMP(1, 0);
  if (VEC && base + CH <= n) {
    uint32_t k[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
      Vec4<uint32_t>::load<NT>(keys + base + (uint64_t)(u * kBlock + tid) * 4, k[u]);
    if (!go()) return;
#ifdef PSKV_STEP_STAMPS
    ready(k[0]);
    STEP_STAMP(1, 1);
#endif
    VT v[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) gather4<VT, false, FRESH>(d, o, k[u], v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u)
      Vec4<VT>::template store<NT>(out + base + (uint64_t)(u * kBlock + tid) * 4, v[u]);
    STEP_STAMP(1, 2);
  } else {
    // a partial (or unaligned) chunk: eight keys per lane loaded together,
    // then their gathers, then the stores — one dependent round trip per
    // eight elements instead of per element (it matters when the keys sit in
    // host memory: the zero-copy Get runs K1 over pinned staging)
    if (!go()) return;
    const uint64_t end = n < base + CH ? n : base + CH;
    for (uint64_t i0 = base + tid; i0 < end; i0 += 8ull * kBlock) {
      uint32_t kk[8];
      VT vv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t i = i0 + (uint64_t)q * kBlock;
        kk[q] = i < end ? keys[i] : 0u;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        vv[q] = i0 + (uint64_t)q * kBlock < end ? load_one<VT, FRESH>(d, o, kk[q]) : VT(0);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t i = i0 + (uint64_t)q * kBlock;
        if (i < end) out[i] = vv[q];
      }
    }
  }
}

template <typename VT, bool VEC, int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_gather(GroupArgs ga, DenseView d, Ovf o) {
  gather_chunk<VT, VEC, U, NT>(ga, d, o, blockIdx.x);
}

// ----------------------------------------------------- K2 sorted assign
// In a non-decreasing batch the duplicates of a key are adjacent, so the last
// occurrence is the element whose successor differs (or that has none).  Only
// that element stores: deterministic last-write-wins without atomics.  Every
// element also checks that it is in [lo, hi) and not greater than its
// successor; a violation tags `flag` with the call's epoch and the general path
// (launched behind it, conditional on the tag) recomputes every key of the
// batch, so a wrong sorted hint costs time, never correctness.

template <typename VT>
__device__ __forceinline__ bool scalar_elem(const uint32_t* __restrict__ keys,
                                            const VT* __restrict__ vals, uint64_t n, uint64_t i,
                                            const DenseView& d, uint64_t lo, uint64_t hi) {
  const uint32_t k = keys[i];
  const bool hn = i + 1 < n;
  const uint32_t nk = hn ? keys[i + 1] : 0u;
  const uint64_t off = (uint32_t)(k - d.key_begin);
  bool bad = hn && k > nk;
  if (off < lo || off >= hi)
    bad = true;
  else if (!hn || k != nk)
    reinterpret_cast<VT*>(d.param)[off] = vals[i];
  return bad;
}

template <typename VT>
__device__ __forceinline__ bool scatter4_sorted(const DenseView& d, const uint32_t (&k)[4],
                                                const VT (&v)[4], uint32_t nk, bool has_next,
                                                uint64_t lo, uint64_t hi) {
  VT* __restrict__ param = reinterpret_cast<VT*>(d.param);
  const uint32_t off0 = k[0] - d.key_begin;
  const bool run = (k[1] == k[0] + 1u) & (k[2] == k[0] + 2u) & (k[3] == k[0] + 3u) &
                   ((off0 & 3u) == 0u) & ((uint64_t)off0 >= lo) & ((uint64_t)off0 + 3u < hi);
  bool bad = false;
  if (run && !(has_next && nk <= k[3])) {
    Vec4<VT>::store(param + off0, v);  // four distinct consecutive keys, last one ends its run
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool hn = e < 3 || has_next;
      const uint32_t nx = e < 3 ? k[e + 1 < 4 ? e + 1 : 3] : nk;
      const uint64_t off = (uint32_t)(k[e] - d.key_begin);
      if (hn && k[e] > nx) bad = true;
      if (off < lo || off >= hi)
        bad = true;
      else if (!hn || k[e] != nx)
        param[off] = v[e];
    }
  }
  return bad;
}

template <typename VT, bool VEC>
__global__ __launch_bounds__(kBlock) void k_assign_sorted(const uint32_t* __restrict__ keys,
                                                          const VT* __restrict__ vals, uint64_t n,
                                                          DenseView d, uint32_t* flag,
                                                          uint32_t epoch) {
  const uint64_t base = (uint64_t)blockIdx.x * kSortedChunk;
  const int tid = threadIdx.x;
  bool bad = false;
  if (VEC && base + kSortedChunk <= n) {
    uint32_t k[kSortedUnroll][4];
    VT v[kSortedUnroll][4];
    uint32_t nk[kSortedUnroll];
    bool hn[kSortedUnroll];
#pragma unroll
    for (int u = 0; u < kSortedUnroll; ++u) {
      const uint64_t i = base + (uint64_t)(u * kBlock + tid) * 4;
      Vec4<uint32_t>::load(keys + i, k[u]);
      Vec4<VT>::load(vals + i, v[u]);
      hn[u] = i + 4 < n;
      nk[u] = hn[u] ? keys[i + 4] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kSortedUnroll; ++u)
      bad |= scatter4_sorted<VT>(d, k[u], v[u], nk[u], hn[u], 0, d.range);
  } else {
    const uint64_t end = n < base + kSortedChunk ? n : base + kSortedChunk;
    for (uint64_t i = base + tid; i < end; i += kBlock)
      bad |= scalar_elem<VT>(keys, vals, n, i, d, 0, d.range);
  }
  if (bad) *flag = epoch;
}

// --------------------------------------------- K2g grouped sorted assign
// Grouped batches may share keys (a later batch must win), so the elementwise
// K2 cannot run them concurrently.  Instead the key range is cut into tiles of
// 2^tile_shift keys; ONE workgroup owns a tile and applies, in call order, the
// slice of every batch that falls into it (a contiguous segment of a sorted
// batch, found by interpolation + binary search).  A workgroup barrier between
// batches orders the stores of one CU to one address; different tiles touch
// disjoint keys, so no cross-workgroup ordering is needed and the stores stay
// plain, coalesced and atomic-free.
//
// Verification: tile t of batch j gets segment [lb(lo_t), lb(hi_t)) with the
// SAME deterministic search for a shared boundary, so the segments of one batch
// chain without gaps from 0 (first tile) to n (last tile).  Each element checks
// that it lies in its tile and does not exceed its successor; if every check
// passes the whole batch was sorted.  Any failure tags `flag` for the repair.

__device__ __forceinline__ uint64_t lower_bound_interp(const uint32_t* __restrict__ keys,
                                                       uint64_t n, uint32_t x, uint32_t first,
                                                       uint32_t last) {
  // Called only when first < x <= last, so (for a sorted batch) the answer is
  // in [1, n-1].  All probes stay in [0, n-1] whatever the data.
  uint64_t lo = 1, hi = n - 1;
  if (n > 2 && last > first) {
    uint64_t g = (uint64_t)(x - first) * (n - 1) / (uint64_t)(last - first);
    g = g < lo ? lo : (g > hi ? hi : g);
    if (keys[g] >= x) {
      if (keys[g - 1] < x) return g;
      hi = g - 1;
    } else {
      lo = g + 1;
    }
  }
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (keys[mid] >= x)
      hi = mid;
    else
      lo = mid + 1;
  }
  return lo;
}

template <typename VT, bool VEC>
__device__ __forceinline__ bool apply_segment(const DevBatch& b, uint64_t s, uint64_t e,
                                              const DenseView& d, uint64_t lo, uint64_t hi) {
  const uint32_t* __restrict__ keys = b.keys;
  const VT* __restrict__ vals = reinterpret_cast<const VT*>(b.vals);
  const uint64_t n = b.n;
  const int tid = threadIdx.x;
  bool bad = false;
  if (VEC) {
    const uint64_t a = (s + 3) & ~3ull;
    const uint64_t va = a < e ? a : e;
    const uint64_t z0 = e & ~3ull;
    const uint64_t vz = z0 > va ? z0 : va;
    if ((uint64_t)tid < va - s) bad |= scalar_elem<VT>(keys, vals, n, s + tid, d, lo, hi);
    if ((uint64_t)tid < e - vz) bad |= scalar_elem<VT>(keys, vals, n, vz + tid, d, lo, hi);
    for (uint64_t g = va + (uint64_t)tid * 4; g < vz; g += (uint64_t)kBlock * 4) {
      uint32_t k[4];
      VT v[4];
      Vec4<uint32_t>::load(keys + g, k);
      Vec4<VT>::load(vals + g, v);
      const bool hn = g + 4 < n;
      const uint32_t nk = hn ? keys[g + 4] : 0u;
      bad |= scatter4_sorted<VT>(d, k, v, nk, hn, lo, hi);
    }
  } else {
    for (uint64_t i = s + tid; i < e; i += kBlock)
      bad |= scalar_elem<VT>(keys, vals, n, i, d, lo, hi);
  }
  return bad;
}

// Mode A (all batches dense): batch j of the group is a contiguous run
// first_j .. first_j + n_j - 1 (the vector_storage push of a whole parameter
// slice).  "A later call wins" is then an interval test: key k of batch j is
// stored unless some later batch j' > j covers k.  Work is split by elements
// (8192 per chunk, one workgroup each), so the launch is balanced like the
// gather; each chunk intersects its key interval with the later batches'
// intervals once (a 64-lane ballot) and elements test only the few that
// overlap.  Every element verifies k == first_j + i; a batch whose endpoints
// look dense but whose keys are not is caught there and tagged for the repair.
// An element is stored at first_j + i only when ITS OWN key verified (a lane's
// group of four, or a wave's span for 8-byte values, as a whole): the replay
// behind a tagged group rewrites exactly the keys the group holds, so the
// sorted pass must never write any other key — a look-alike batch (same
// endpoints, a duplicate hiding a missing key) would otherwise leave a value
// at a key no batch of the group pushed.

// dense_chunk: 8-byte values, and batches not 16-byte aligned (4-byte values
// in aligned batches take dense_chunk_own below).
template <typename VT, bool VEC, int U, bool NT, bool NTP>
__device__ __forceinline__ bool dense_chunk(const GroupArgs& ga, const DenseView& d, uint32_t c,
                                            const uint32_t* s_first, const uint32_t* s_last) {
  constexpr int CH = kBlock * 4 * U;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int j = batch_of(ga, c);
  const uint32_t* __restrict__ keys = ga.b[j].keys;
  const VT* __restrict__ vals = reinterpret_cast<const VT*>(ga.b[j].vals);
  const uint64_t n = ga.b[j].n;
  const uint64_t base = (uint64_t)(c - ga.wg_prefix[j]) * CH;
  const uint64_t end = n < base + CH ? n : base + CH;
  const uint32_t first = s_first[j];
  const uint32_t p0 = first - d.key_begin;
  const uint32_t c_lo = first + (uint32_t)base, c_hi = first + (uint32_t)(end - 1);
  // later batches whose interval meets this chunk's interval (every wave computes it)
  const bool ov = lane > j && lane < ga.nb && s_first[lane] <= c_hi && s_last[lane] >= c_lo;
  const unsigned long long later = __ballot(ov);
  // one later batch covers the whole chunk: none of its values can survive, so
  // they are not even read (the keys still are: they prove batch j dense)
  const bool covered = __ballot(ov && s_first[lane] <= c_lo && s_last[lane] >= c_hi) != 0;
  VT* __restrict__ param = reinterpret_cast<VT*>(d.param);
  bool bad = false;
  auto shadowed = [&](uint32_t k) {
    unsigned long long m = later;
    bool sh = false;
    while (m) {
      const int q = __ffsll((long long)m) - 1;
      m &= m - 1;
      sh |= (k >= s_first[q]) & (k <= s_last[q]);
    }
    return sh;
  };
  if (sizeof(VT) == 8 && VEC && end - base == CH) {
    // 8-byte values: keys four per lane (16-byte loads; each lane checks its
    // own four against first + index), values and parameters as PAIRS over the
    // wave's 256-element span (lane l: elements 2l, 2l+1 and 128+2l, 128+2l+1),
    // so every access instruction covers one contiguous span.  The wave's keys
    // cover the same span as its stores: it stores only if all 256 verified.
    using T = unsigned long long;
    uint32_t k[U][4];
    T va[U][2], vb[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (uint64_t)(u * kBlock + tid) * 4;
      const uint64_t ew = base + (uint64_t)(u * kBlock + (tid & ~63)) * 4;
      Vec4<uint32_t>::load<NT>(keys + i, k[u]);
      if (!covered) {
        Vec2x8::load<NT>(reinterpret_cast<const T*>(vals) + ew + 2 * lane, va[u]);
        Vec2x8::load<NT>(reinterpret_cast<const T*>(vals) + ew + 128 + 2 * lane, vb[u]);
      }
    }
    T* __restrict__ p8 = reinterpret_cast<T*>(param);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (uint64_t)(u * kBlock + tid) * 4;
      const uint32_t k0 = first + (uint32_t)i;
      const bool lbad = (k[u][0] != k0) | (k[u][1] != k0 + 1u) | (k[u][2] != k0 + 2u) | (k[u][3] != k0 + 3u);
      bad |= lbad;
      if (covered || __ballot(lbad) != 0) continue;  // wave-uniform
      const uint32_t ka = first + (uint32_t)(base + (uint64_t)(u * kBlock + (tid & ~63)) * 4) + 2u * lane;
      const uint32_t offa = ka - d.key_begin;
      if (later == 0 && (offa & 1u) == 0u) {
        Vec2x8::store<NTP>(p8 + offa, va[u]);
        Vec2x8::store<NTP>(p8 + offa + 128, vb[u]);
      } else {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          if (!shadowed(ka + e)) p8[offa + e] = va[u][e];
          if (!shadowed(ka + 128u + e)) p8[offa + 128 + e] = vb[u][e];
        }
      }
    }
  } else {
    // a partial (or unaligned) chunk — the last one of every window: eight
    // elements per lane loaded together, then checked and stored, so the
    // chunk costs one dependent round trip per eight elements per lane rather
    // than one per element (a window's 576-key tail took three in a row)
    for (uint64_t i0 = base + tid; i0 < end; i0 += 8ull * kBlock) {
      uint32_t kk[8];
      VT vv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t i = i0 + (uint64_t)q * kBlock;
        kk[q] = i < end ? keys[i] : first + (uint32_t)i;
        vv[q] = i < end && !covered ? vals[i] : VT(0);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t i = i0 + (uint64_t)q * kBlock;
        const bool ebad = kk[q] != first + (uint32_t)i;
        bad |= ebad;
        if (i < end && !covered && !ebad && !shadowed(first + (uint32_t)i)) param[p0 + i] = vv[q];
      }
    }
  }
  return bad;
}

// 4-byte values in 16-byte aligned batches (dense_chunk_own): every chunk
// loads its own keys and values with aligned 16-byte loads and stores them
// where they land, a dword-aligned 16-byte store when the window starts off
// the 16-byte parameter slots (cfg 4's producer windows start at any key).
// Against the round-3 form that shifted each chunk down by the window's phase
// so the stores were slot-aligned (and the loads dword-aligned), this is as
// fast at phase 0 and 3-4 % faster at phases 1-3 (K2g 107.3-109.2 against
// 111.0-112.8 us per 64 x 1M keys, `profiles/r03_probes/align_own/`), and it
// has no head or tail special case.  Early mode (option EARLY, chosen per
// launch by the host) issues a workgroup's whole-chunk loads before its
// prologue (the first and last key of every batch) has come back; it cannot
// skip the values of a chunk a later window covers (they are already in
// flight), so it is for small launches whose windows rarely overlap (a rank's
// ~8 windows at N = 8).  PRE: k / v already hold the (whole) chunk.  (Round 4
// measured a keys-only early form, values still skipped for a covered chunk:
// K2g 115.4 against 112.7 us on the headline; removed.)
template <int U, bool NT, bool NTP, bool PRE>
__device__ __forceinline__ bool dense_chunk_own(const GroupArgs& ga, const DenseView& d, uint32_t c,
                                                const uint32_t* s_first, const uint32_t* s_last,
                                                uint32_t (&k)[U][4], uint32_t (&v)[U][4]) {
  constexpr int CH = kBlock * 4 * U;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int j = batch_of(ga, c);
  const uint32_t* __restrict__ keys = ga.b[j].keys;
  const uint32_t* __restrict__ vals = reinterpret_cast<const uint32_t*>(ga.b[j].vals);
  const uint64_t n = ga.b[j].n;
  const uint64_t base = (uint64_t)(c - ga.wg_prefix[j]) * CH;
  const uint64_t end = n < base + CH ? n : base + CH;
  const uint32_t first = s_first[j];
  const uint32_t p0 = first - d.key_begin;
  const uint32_t c_lo = first + (uint32_t)base, c_hi = first + (uint32_t)(end - 1);
  const bool ov = lane > j && lane < ga.nb && s_first[lane] <= c_hi && s_last[lane] >= c_lo;
  const unsigned long long later = __ballot(ov);
  const bool covered = __ballot(ov && s_first[lane] <= c_lo && s_last[lane] >= c_hi) != 0;
  uint32_t* __restrict__ param = reinterpret_cast<uint32_t*>(d.param);
  bool bad = false;
  auto shadowed = [&](uint32_t key) {
    unsigned long long m = later;
    bool sh = false;
    while (m) {
      const int q = __ffsll((long long)m) - 1;
      m &= m - 1;
      sh |= (key >= s_first[q]) & (key <= s_last[q]);
    }
    return sh;
  };
  if (end - base == CH) {
    const uint32_t* __restrict__ kc = keys + base;
    const uint32_t* __restrict__ vc = vals + base;
    uint32_t* __restrict__ pc = param + p0 + base;
    if (!PRE) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t o = (uint32_t)(u * kBlock + tid) * 4u;
        Vec4<uint32_t>::load<NT>(kc + o, k[u]);
        if (!covered) Vec4<uint32_t>::load<NT>(vc + o, v[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t o = (uint32_t)(u * kBlock + tid) * 4u;
      const uint32_t k0 = first + (uint32_t)base + o;
      const bool lbad = (k[u][0] != k0) | (k[u][1] != k0 + 1u) | (k[u][2] != k0 + 2u) | (k[u][3] != k0 + 3u);
      bad |= lbad;
      if (covered || lbad) continue;
      if (later == 0) {
        st16a4<NTP>(pc + o, v[u]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (!shadowed(k0 + (uint32_t)e)) pc[o + e] = v[u][e];
      }
    }
  } else {
    // a partial chunk (the last of a window): eight elements per lane loaded
    // together, then checked and stored
    for (uint64_t i0 = base + tid; i0 < end; i0 += 8ull * kBlock) {
      uint32_t kk[8], vv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t i = i0 + (uint64_t)q * kBlock;
        kk[q] = i < end ? keys[i] : first + (uint32_t)i;
        vv[q] = i < end && !covered ? vals[i] : 0u;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint64_t i = i0 + (uint64_t)q * kBlock;
        const bool ebad = kk[q] != first + (uint32_t)i;
        bad |= ebad;
        if (i < end && !covered && !ebad && !shadowed(first + (uint32_t)i)) param[p0 + i] = vv[q];
      }
    }
  }
  return bad;
}

// The prologue of a grouped sorted Add (K2g): lanes of
// waves 0 and 1 keep batch jb's endpoints for the whole launch; wave 0
// publishes them (s_first / s_last) and whether every batch is one dense
// in-range window (s_dense).  Endpoints out of range or inverted tag `flag`
// (workgroup 0 only).  The caller syncs the workgroup before reading them.
struct GroupEnds {
  uint32_t first = 0, last = 0;
  uint64_t n = 0;
  bool ok = false;
  const uint32_t* keys = nullptr;
};

__device__ __forceinline__ GroupEnds group_prologue(const GroupArgs& ga, const DenseView& d, uint32_t* flag,
                                                    uint32_t epoch, uint32_t* s_first, uint32_t* s_last,
                                                    int* s_dense) {
  const int tid = threadIdx.x;
  const int jb = tid & 63;
  GroupEnds g;
  if (tid < 128 && jb < ga.nb) {
    g.keys = ga.b[jb].keys;
    g.n = ga.b[jb].n;
    if (g.n > 0) {
      g.first = g.keys[0];
      g.last = g.keys[g.n - 1];
      const uint64_t fo0 = (uint32_t)(g.first - d.key_begin);
      const uint64_t lo0 = (uint32_t)(g.last - d.key_begin);
      g.ok = fo0 < d.range && lo0 < d.range && g.first <= g.last;
      if (!g.ok && blockIdx.x == 0 && tid < 64) *flag = epoch;  // out-of-range or inverted endpoints
    }
  }
  if (tid < 64) {
    const bool dense_j = jb >= ga.nb || (g.ok && (uint64_t)(g.last - g.first) == g.n - 1);
    if (jb < kMaxBatches) {
      s_first[jb] = g.first;
      s_last[jb] = g.last;
    }
    const unsigned long long m = __ballot(!dense_j);
    if (tid == 0) *s_dense = m == 0;
  }
  return g;
}

// Tile mode (general sorted batches): a workgroup owns key tiles t = wg,
// wg + nwg, ... and applies each batch's segment of the tile in call order.
template <typename VT, bool VEC>
__device__ __forceinline__ bool tile_mode(const GroupArgs& ga, const DenseView& d, const GroupEnds& g,
                                          uint32_t tile_shift, uint64_t ntiles, uint32_t wg, uint32_t nwg,
                                          uint64_t* s_seg_s, uint64_t* s_seg_e, unsigned long long* s_mask) {
  const int tid = threadIdx.x;
  const int jb = tid & 63;
  bool bad = false;
  const uint64_t fo = (uint32_t)(g.first - d.key_begin);
  const uint64_t lo_ = (uint32_t)(g.last - d.key_begin);
  for (uint64_t t = wg; t < ntiles; t += nwg) {
    const uint64_t tlo = t << tile_shift;
    const uint64_t tend = tlo + (1ull << tile_shift);
    const uint64_t thi = tend < d.range ? tend : d.range;
    const bool ov = g.ok && fo < thi && lo_ >= tlo;
    // wave 0 searches segment starts, wave 1 segment ends, concurrently
    if (tid < 64) {
      if (jb < kMaxBatches)
        s_seg_s[jb] = !ov ? 0 : (fo >= tlo ? 0 : lower_bound_interp(g.keys, g.n, d.key_begin + (uint32_t)tlo, g.first, g.last));
    } else if (tid < 128) {
      s_seg_e[jb] = !ov ? 0 : (lo_ < thi ? g.n : lower_bound_interp(g.keys, g.n, d.key_begin + (uint32_t)thi, g.first, g.last));
    }
    __syncthreads();
    if (tid < 64) {
      const uint64_t s = s_seg_s[jb], e = s_seg_e[jb];
      if (ov && s > e) bad = true;
      const unsigned long long m = __ballot(ov && s < e);
      if (tid == 0) *s_mask = m;
    }
    __syncthreads();
    unsigned long long m = *s_mask;
    while (m) {
      const int j = __ffsll((long long)m) - 1;
      m &= m - 1;
      bad |= apply_segment<VT, VEC>(ga.b[j], s_seg_s[j], s_seg_e[j], d, tlo, thi);
      __syncthreads();  // batch j's stores precede batch j+1's in this tile
    }
  }
  return bad;
}

// Mode B (general sorted batches): key-tile owner, static strided schedule.
template <typename VT, bool VEC, int U, bool NT, bool NTP, bool EARLY = false>
__global__ __launch_bounds__(kBlock) void k_assign_group(GroupArgs ga, DenseView d,
                                                         uint32_t tile_shift, uint64_t ntiles,
                                                         uint32_t* flag, uint32_t epoch) {
  constexpr bool OWN = sizeof(VT) == 4 && VEC;  // dense_chunk_own
  static_assert(!EARLY || OWN, "early loads: 4-byte values, aligned batches");
  constexpr int CH = kBlock * 4 * U;
  __shared__ uint64_t s_seg_s[kMaxBatches];
  __shared__ uint64_t s_seg_e[kMaxBatches];
  __shared__ uint32_t s_first[kMaxBatches];
  __shared__ uint32_t s_last[kMaxBatches];
  __shared__ unsigned long long s_mask;
  __shared__ int s_dense;
  const int tid = threadIdx.x;
  // early mode: this workgroup's first chunk, when whole, is requested now,
  // before the prologue below (its loads need no batch endpoint)
  uint32_t ek[OWN ? U : 1][4], ev[OWN ? U : 1][4];
  bool pre = false;
  if constexpr (EARLY) {
    if (blockIdx.x < ga.wg_prefix[ga.nb]) {
      const int j0 = batch_of(ga, blockIdx.x);
      const uint64_t base0 = (uint64_t)(blockIdx.x - ga.wg_prefix[j0]) * CH;
      if (ga.b[j0].n >= base0 + CH) {
        pre = true;
        const uint32_t* __restrict__ kc = ga.b[j0].keys + base0;
        const uint32_t* __restrict__ vc = reinterpret_cast<const uint32_t*>(ga.b[j0].vals) + base0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t o = (uint32_t)(u * kBlock + tid) * 4u;
          Vec4<uint32_t>::load<NT>(kc + o, ek[u]);
          Vec4<uint32_t>::load<NT>(vc + o, ev[u]);
        }
      }
    }
  }
  STEP_STAMP(0, 0);
  const GroupEnds g = group_prologue(ga, d, flag, epoch, s_first, s_last, &s_dense);
  __syncthreads();
  STEP_STAMP(0, 1);
  bool bad = false;
  if (s_dense) {
    const uint32_t nchunks = ga.wg_prefix[ga.nb];
    if constexpr (OWN) {
      uint32_t c = blockIdx.x;
      if (pre) {
        bad |= dense_chunk_own<U, NT, NTP, true>(ga, d, c, s_first, s_last, ek, ev);
        STEP_STAMP(0, 2);
        c += gridDim.x;
      }
      for (; c < nchunks; c += gridDim.x)
        bad |= dense_chunk_own<U, NT, NTP, false>(ga, d, c, s_first, s_last, ek, ev);
      STEP_STAMP(0, 3);
    } else {
      for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x)
        bad |= dense_chunk<VT, VEC, U, NT, NTP>(ga, d, c, s_first, s_last);
    }
    if (bad) *flag = epoch;
    return;
  }
  // (Round 4: re-deriving g here from LDS and the arguments instead takes the
  // dense path from 100 to 94 VGPRs, 4 -> 5 waves per SIMD, and measured
  // 1-3 % SLOWER on the headline and cold steps: profiles/r04_probes/k2g_waves5_noreg/;
  // forcing 5 waves with amdgpu_waves_per_eu spills and loses too, k2g_waves5/.)
  bad = tile_mode<VT, VEC>(ga, d, g, tile_shift, ntiles, blockIdx.x, gridDim.x, s_seg_s, s_seg_e, &s_mask);
  if (bad) *flag = epoch;
}

// a + b with two's-complement wrap for int32 (the reference's int values),
// plain IEEE addition for float/double
template <typename T>
__device__ __forceinline__ T add_wrap(T a, T b) {
  return a + b;
}
template <>
__device__ __forceinline__ int add_wrap<int>(int a, int b) {
  return (int)((uint32_t)a + (uint32_t)b);
}

template <typename T>
__device__ __forceinline__ unsigned long long to_bits(T v) {
  if (sizeof(T) == 8) return *reinterpret_cast<const unsigned long long*>(&v);
  return (unsigned long long)*reinterpret_cast<const uint32_t*>(&v);
}
template <typename T>
__device__ __forceinline__ T from_bits(unsigned long long b) {
  if (sizeof(T) == 8) return *reinterpret_cast<const T*>(&b);
  const uint32_t lo = (uint32_t)b;
  return *reinterpret_cast<const T*>(&lo);
}

// *p += v on an LDS word.  Integer adds are ds_add (full rate).  The LDS unit
// runs ds_add_f32 at ~1/40 of the integer atomics' rate on gfx950 (measured:
// 0.2 vs 8 T atomics/s chip-wide, tools/micro/lds_atomic.hip), so float and
// double sums first try an integer compare-and-swap (2.6 T/s uncontended);
// a lane that loses twice (a hot key shared within the wave) falls back to the
// hardware float atomic, whose cost does not grow with contention.  Both are
// atomic read-modify-writes of the LDS unit, so they mix safely.
template <typename T>
__device__ __forceinline__ void lds_add(T* p, T v) {
  if constexpr (std::is_integral<T>::value) {
    atomicAdd(p, v);
  } else {
    using U = typename std::conditional<sizeof(T) == 8, unsigned long long, uint32_t>::type;
    U* w = reinterpret_cast<U*>(p);
    U old = *w;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const U assumed = old;
      old = atomicCAS(w, assumed, (U)to_bits<T>(from_bits<T>(assumed) + v));
      if (old == assumed) return;
    }
    atomicAdd(p, v);
  }
}

// ------------------------------------------------ K4 general (any order)
// K4a: a workgroup takes 2048 consecutive elements of one batch and folds them
// into a 4096-slot LDS hash (key -> max element index, or key -> sum).  Then
// each distinct key of the chunk does ONE global operation:
//   assign:     atomicMax(owner[key], epoch<<32 | group index of its last occurrence)
//   accumulate: atomicAdd(param[key], chunk sum)
// so a Zipf-hot key costs one atomic per chunk, not one per occurrence.
// K4b (assign): every element whose stamp won stores its value — exactly one
// element per key, the last one in call order.  The stamp array is never reset:
// epochs increase, so an old stamp always loses.

// Out-of-range keys are not K4's: many workgroups insert at once here, and
// only a single workgroup can grow the table mid-kernel, so K4a tags `oor`
// and the oor_only replay behind K4 applies those keys in call order (assign:
// last wins; accumulate: sums), with room reserved as it goes.  Dense and
// overflow keys are disjoint, so the split changes no result.
template <typename AT>
__device__ __forceinline__ void global_accumulate(const DenseView& d, uint32_t* oor, uint32_t epoch,
                                                  uint32_t k, AT v) {
  const uint32_t off = k - d.key_begin;
  if ((uint64_t)off < d.range)
    atomicAdd(reinterpret_cast<AT*>(d.param) + off, v);
  else
    __hip_atomic_store(oor, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void global_stamp(const DenseView& d, uint32_t* oor, uint32_t epoch,
                                             unsigned long long* owner, uint32_t k,
                                             unsigned long long tag) {
  const uint32_t off = k - d.key_begin;
  if ((uint64_t)off < d.range)
    atomicMax(owner + off, tag);
  else
    __hip_atomic_store(oor, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename AT, int MODE>
__global__ __launch_bounds__(kBlock) void k_general_mark(GroupArgs ga, DenseView d, uint32_t* oor,
                                                         unsigned long long* owner,
                                                         const uint32_t* cond, uint32_t epoch) {
  if (cond != nullptr && *cond != epoch) return;  // repair launch, sorted path was right
  constexpr int R = kGeneralChunk / kBlock;        // elements per lane per chunk
  __shared__ uint32_t hk[kGeneralSlots];           // key (EMPTY = 0xFFFFFFFF)
  __shared__ uint32_t hfirst[kGeneralSlots];       // first chunk index of the key
  __shared__ uint32_t hidx[MODE == 0 ? kGeneralSlots : 1];  // assign: last chunk index
  __shared__ AT hsum[MODE == 1 ? kGeneralSlots : 1];        // accumulate: chunk sum
  const int tid = threadIdx.x;
  const uint32_t nvwg = ga.wg_prefix[ga.nb];
  // grid-stride over virtual workgroups (one 2048-key chunk each)
  for (uint32_t wg = blockIdx.x; wg < nvwg; wg += gridDim.x) {
    const int j = batch_of(ga, wg);
    const uint32_t* __restrict__ keys = ga.b[j].keys;
    const AT* __restrict__ vals = reinterpret_cast<const AT*>(ga.b[j].vals);
    const uint64_t n = ga.b[j].n;
    const uint64_t base = (uint64_t)(wg - ga.wg_prefix[j]) * kGeneralChunk;
    const uint64_t gbase = elem_prefix(ga, j) + base;
    for (int s = tid; s < kGeneralSlots; s += kBlock) {
      hk[s] = kEmpty32;
      hfirst[s] = kEmpty32;
      if (MODE == 0)
        hidx[s] = 0;
      else
        hsum[s] = AT(0);
    }
    __syncthreads();
    uint32_t slot[R];
    uint32_t key[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int li = r * kBlock + tid;
      const uint64_t i = base + li;
      slot[r] = kEmpty32;
      key[r] = 0;
      if (i < n) {
        const uint32_t k = keys[i];
        key[r] = k;
        if (k == kEmpty32) {  // the LDS sentinel itself: bypass the LDS table
          if (MODE == 0)
            global_stamp(d, oor, epoch, owner, k, ((unsigned long long)epoch << 32) | (gbase + li));
          else
            global_accumulate<AT>(d, oor, epoch, k, vals[i]);
        } else {
          uint32_t h = fmix32(k) & (kGeneralSlots - 1);
          for (;;) {
            const uint32_t old = atomicCAS(&hk[h], kEmpty32, k);
            if (old == kEmpty32 || old == k) break;
            h = (h + 1) & (kGeneralSlots - 1);
          }
          slot[r] = h;
          atomicMin(&hfirst[h], (uint32_t)li);
          if (MODE == 0)
            atomicMax(&hidx[h], (uint32_t)li);
          else
            lds_add(&hsum[h], vals[i]);
        }
      }
    }
    __syncthreads();
    // One global operation per distinct key, issued by the key's FIRST
    // occurrence in element order: for sorted or dense chunks consecutive lanes
    // then hit consecutive addresses, so the atomics coalesce.
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t h = slot[r];
      if (h == kEmpty32 || hfirst[h] != (uint32_t)(r * kBlock + tid)) continue;
      if (MODE == 0)
        global_stamp(d, oor, epoch, owner, key[r], ((unsigned long long)epoch << 32) | (gbase + hidx[h]));
      else
        global_accumulate<AT>(d, oor, epoch, key[r], hsum[h]);
    }
    __syncthreads();  // the table is re-initialised for the next chunk
  }
}

template <typename VT>
__global__ __launch_bounds__(kBlock) void k_general_commit(GroupArgs ga, DenseView d,
                                                           const unsigned long long* owner,
                                                           const uint32_t* cond, uint32_t epoch) {
  if (cond != nullptr && *cond != epoch) return;
  const int tid = threadIdx.x;
  const uint32_t nvwg = ga.wg_prefix[ga.nb];
  for (uint32_t wg = blockIdx.x; wg < nvwg; wg += gridDim.x) {
    const int j = batch_of(ga, wg);
    const uint32_t* __restrict__ keys = ga.b[j].keys;
    const VT* __restrict__ vals = reinterpret_cast<const VT*>(ga.b[j].vals);
    const uint64_t n = ga.b[j].n;
    const uint64_t base = (uint64_t)(wg - ga.wg_prefix[j]) * kGeneralChunk;
    const uint64_t gbase = elem_prefix(ga, j) + base;
#pragma unroll 2
    for (int r = 0; r < kGeneralChunk / kBlock; ++r) {
      const int li = r * kBlock + tid;
      const uint64_t i = base + li;
      if (i >= n) break;
      const uint32_t k = keys[i];
      const unsigned long long tag = ((unsigned long long)epoch << 32) | (gbase + li);
      const uint32_t off = k - d.key_begin;
      if ((uint64_t)off < d.range && owner[off] == tag) reinterpret_cast<VT*>(d.param)[off] = vals[i];
      // (out-of-range keys: the oor_only replay behind K4)
    }
  }
}

// Host growth (pskv_sync): the table in the control block, rehashed into `to`
// (keys EMPTY, values 0, room for every key); then k_ovf_set switches over.
template <typename VT>
__global__ __launch_bounds__(kBlock) void k_ovf_rehash(Ovf o, uint64_t from_cap, OvfTab to) {
  const OvfTab from = ovf_tab(o);
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < from_cap && i <= from.mask;
       i += (uint64_t)gridDim.x * kBlock) {
    const unsigned long long k = from.keys[i];
    if (k == kEmpty64) continue;
    reinterpret_cast<VT*>(to.vals)[ovf_place(to, (uint32_t)k)] = reinterpret_cast<const VT*>(from.vals)[i];
  }
}

__global__ void k_ovf_set(Ovf o, OvfTab to) {
  if (threadIdx.x == 0) o.c->t = to;
}

// ------------------------------------------- K5 key-bucket general path
// The general (any order) Add without random global atomics.  K4's stamps cost
// one random agent-scope atomic per distinct key per chunk, and those run at
// ~20 G/s chip-wide (memory-side atomics, MI355X_MICROARCH.md "Global float
// atomics": 64 lanes in 64 rows ≈ 17x slower).  K5 instead moves the data to
// where it can be resolved locally, in two launches.  Work unit of the first:
// a SUPER-CHUNK of 8 Ki keys of one batch (4 Ki for 8-byte values); key
// buckets (RbMap): the owned range is cut into windows of 2^wbits keys, dealt
// round-robin to nbd buckets (window w -> bucket w % nbd), plus one bucket for
// out-of-range keys.  Interleaved windows keep a batch that covers only part of
// the range — sorted or dense keys pushed without the hint — spread over every
// bucket; with one contiguous window per bucket such a batch lands in a few
// buckets and the resolve of each runs on one CU (2^32 sequential keys: over
// 3 minutes, against 1.4 s interleaved).
//   K5a k_rb_bin      per super-chunk: LDS hash dedup (one entry per distinct
//                     key: its last value / its sum), LDS counting sort of the
//                     entries by bucket, one coalesced write of the sorted
//                     entries to the super-chunk's region, one 16-bit row of
//                     bucket starts
//   K5b k_rb_resolve  one workgroup per bucket: gathers the bucket's run from
//                     every super-chunk region — an entry's position in the
//                     concatenation IS call order — resolves it in an LDS hash
//                     (largest position wins / values add) and stores the
//                     winners into the dense array or the overflow table.  A
//                     bucket is owned by one workgroup: no cross-workgroup
//                     ordering, no global atomics.
// Measured against the four-launch form it replaces (dedup per 2 Ki sub-chunk,
// entries appended, global scan, global radix move, apply): 198 -> 149 us per
// 8 M Zipf keys; the per-entry uncoalesced appends and the move's second pass
// over the entries were the cost, not the LDS work.

template <int VB>
struct RbEnt;
template <>
struct RbEnt<4> {
  uint32_t key;
  uint32_t val;
};
template <>
struct RbEnt<8> {
  uint32_t key;
  uint32_t pad;
  unsigned long long val;
};

// Window w = off >> wbits -> bucket w % nbd, and the bucket-local window index
// w / nbd.  Division by the invariant nbd: q = umulhi(w, ceil(2^32 / nbd)) is
// w / nbd or one more (w < 2^21, nbd < 2^12), fixed up by the remainder's sign.
// (A double-reciprocal division here cost ~10 % of K5 on cfg 3.)
__device__ __forceinline__ uint32_t rb_split(const RbMap& m, uint32_t off, uint32_t* j) {
  const uint32_t w = off >> m.wbits;
  if (m.nlog >= 0) {  // nbd a power of two: shifts only
    *j = w >> m.nlog;
    return w & (m.nbd - 1u);
  }
  uint32_t q = __umulhi(w, m.magic);
  int32_t r = (int32_t)(w - q * m.nbd);
  if (r < 0) {
    --q;
    r += (int32_t)m.nbd;
  }
  *j = q;
  return (uint32_t)r;
}

__device__ __forceinline__ uint32_t rb_bucket(const DenseView& d, uint32_t k, const RbMap& m) {
  const uint32_t off = k - d.key_begin;
  uint32_t j;
  return (uint64_t)off < d.range ? rb_split(m, off, &j) : m.nbd;  // nbd = the out-of-range bucket
}

// Bucket-local index of an in-range key offset (dense in [0, m.span)).
__device__ __forceinline__ uint32_t rb_local(const RbMap& m, uint32_t off) {
  uint32_t j;
  (void)rb_split(m, off, &j);
  return (j << m.wbits) | (off & ((1u << m.wbits) - 1u));
}

// Block-wide exclusive scan of a[0..n) in LDS, in place (n <= kRbMaxBuckets + 1).
// Returns the total.  Every thread of the block must call it, after a barrier
// behind the last write of a[] (a thread reads words other threads wrote).
template <int BLOCK>
__device__ __forceinline__ uint32_t block_exscan(uint32_t* a, uint32_t n, uint32_t* wtmp) {
  constexpr int PER = (kRbMaxBuckets + 1 + BLOCK - 1) / BLOCK;
  constexpr int NW = BLOCK / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t b0 = (uint32_t)tid * PER;
  uint32_t x[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    x[i] = b0 + i < n ? a[b0 + i] : 0u;
    sum += x[i];
  }
  uint32_t v = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (lane == 63) wtmp[w] = v;
  __syncthreads();
  // the wave totals as 16-byte broadcast reads (NW / 4 LDS reads, not NW)
  static_assert(NW % 4 == 0, "whole 16-byte groups of wave totals");
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int g = 0; g < NW / 4; ++g) {
    const u32x4 t4 = reinterpret_cast<const u32x4*>(wtmp)[g];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = g * 4 + e;
      if (q < w) before += t4[e];
      tot += t4[e];
    }
  }
  uint32_t run = before + v - sum;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    if (b0 + i < n) a[b0 + i] = run;
    run += x[i];
  }
  __syncthreads();
  return tot;
}

// Insert this lane's keys into an LDS open-addressing table (linear probing,
// SLOTS a power of two; the key 0xFFFFFFFF uses the side word *sent).  The
// first probe of every key is issued back to back (independent LDS atomics in
// flight); only keys that met another key probe further.  slot[q] = EMPTY for
// invalid keys; own bit q = this lane inserted the key.
template <int PER, int SLOTS>
__device__ __forceinline__ uint32_t lds_insert(uint32_t* hk, uint32_t* sent,
                                               const uint32_t (&key)[PER], uint32_t valid_mask,
                                               uint32_t (&slot)[PER]) {
  uint32_t old[PER];
  uint32_t own = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    slot[q] = kEmpty32;
    old[q] = 0;
    if (!(valid_mask >> q & 1u)) continue;
    if (key[q] == kEmpty32) {
      // the sentinel key owns the side word: the lane that sets it inserted
      // the key (its own value equals EMPTY, so it cannot mark a lost race)
      slot[q] = SLOTS;
      own |= atomicCAS(sent, 0u, 1u) == 0u ? (1u << q) : 0u;
      old[q] = key[q];
    } else {
      slot[q] = fmix32(key[q]) & (SLOTS - 1);
      old[q] = atomicCAS(&hk[slot[q]], kEmpty32, key[q]);
    }
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    if (!(valid_mask >> q & 1u) || key[q] == kEmpty32) continue;
    uint32_t o = old[q], h = slot[q];
    while (o != kEmpty32 && o != key[q]) {  // collision: probe on
      h = (h + 1) & (SLOTS - 1);
      o = atomicCAS(&hk[h], kEmpty32, key[q]);
    }
    slot[q] = h;
    own |= o == kEmpty32 ? (1u << q) : 0u;
  }
  return own;
}

// Hybrid insert (K5a, round 5): the first CAS of every
// key position issued back to back as in lds_insert, then ONE retry stream per
// lane over its collided positions (one CAS per step; a placed key hands the
// next step to the lane's next collided key) instead of a probe loop per
// position -- the wave pays the worst lane's total of retries, not the sum
// over positions of each position's worst lane.
template <int PER, int SLOTS>
__device__ __forceinline__ uint32_t lds_insert_hybrid(uint32_t* hk, uint32_t* sent,
                                                      const uint32_t (&key)[PER], uint32_t valid_mask,
                                                      uint32_t (&slot)[PER]) {
  uint32_t old[PER];
  uint32_t own = 0, pend = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    slot[q] = kEmpty32;
    old[q] = 0;
    if (!(valid_mask >> q & 1u)) continue;
    if (key[q] == kEmpty32) {
      slot[q] = SLOTS;
      own |= atomicCAS(sent, 0u, 1u) == 0u ? (1u << q) : 0u;
      old[q] = key[q];
    } else {
      slot[q] = fmix32(key[q]) & (SLOTS - 1);
      old[q] = atomicCAS(&hk[slot[q]], kEmpty32, key[q]);
    }
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    if (!(valid_mask >> q & 1u) || key[q] == kEmpty32) continue;
    if (old[q] == kEmpty32)
      own |= 1u << q;
    else if (old[q] != key[q])
      pend |= 1u << q;
  }
  // the retry stream: cq = the lowest collided position, h its next slot
  auto pick = [&](uint32_t cq, const uint32_t (&a)[PER]) {
    uint32_t x = a[0];
#pragma unroll
    for (int i = 1; i < PER; ++i) {
      asm volatile("" : "+v"(x));  // keep the select chain (an index by cq would go to scratch)
      x = cq == (uint32_t)i ? a[i] : x;
    }
    return x;
  };
  uint32_t cq = (uint32_t)__builtin_ctz(pend | (1u << PER));
  uint32_t ck = pick(cq, key);
  uint32_t h = (pick(cq, slot) + 1u) & (SLOTS - 1);
  while (pend) {
    const uint32_t o = atomicCAS(&hk[h], kEmpty32, ck);
    if (o == kEmpty32 || o == ck) {
#pragma unroll
      for (int i = 0; i < PER; ++i) slot[i] = cq == (uint32_t)i ? h : slot[i];
      own |= o == kEmpty32 ? (1u << cq) : 0u;
      pend &= pend - 1u;
      cq = (uint32_t)__builtin_ctz(pend | (1u << PER));
      ck = pick(cq, key);
      h = (pick(cq, slot) + 1u) & (SLOTS - 1);
    } else {
      h = (h + 1) & (SLOTS - 1);
    }
  }
  return own;
}

// K5a k_rb_bin: persistent workgroups of BINB threads over super-chunks of
// SC = 8 * BINB keys of one batch (4-byte values; 4 * BINB for 8-byte ones),
// the next super-chunk's loads in flight.  BINB = 1024: one workgroup per CU
// (~139 KiB LDS); BINB = 512: 4 Ki-key super-chunks in ~74 KiB, two
// workgroups per CU whose barrier-separated phases overlap.  Per super-chunk:
//   dedup  the SC keys go into ONE LDS hash of 2*SC slots (key -> largest
//          element index for assign, sum for accumulate): a key keeps one
//          entry per super-chunk, its last value or its sum
//   count  each kept entry takes a rank in its bucket's LDS counter
//   stage  the entries are written into LDS in bucket order (over the hash
//          table, which is no longer needed) and copied out to the
//          super-chunk's region of `tmp` with coalesced 16-byte stores
//   row    the bucket starts go out as one 16-bit row loff[sc][0..nbk]
//          (loff[sc][nbk] = the entry count)
// Every global access is a coalesced 16-byte stream; no global atomics.
// Diagnostic build only (-DPSKV_K5_STAMPS, tools/micro/k5_phases.cpp): the
// shader-clock time at each phase boundary of the first 8 passes of every K5a
// / K5b workgroup, read back through pskv_diag_k5_stamps.
#ifdef PSKV_K5_STAMPS
__device__ unsigned long long g_k5_stamps[2][512 * 8 * 8];
#define K5_STAMP(K, IT, PH) \
  if (threadIdx.x == 0 && (IT) < 8u) g_k5_stamps[K][(blockIdx.x * 8u + (IT)) * 8u + (PH)] = __builtin_readcyclecounter()
#else
#define K5_STAMP(K, IT, PH) (void)0
#endif

template <typename BT>
constexpr uint32_t rb_sc(int binb) {
  return (sizeof(BT) == 8 ? 4u : 8u) * (uint32_t)binb;
}

template <typename AT, typename BT, int MODE, int BINB>
__global__ __launch_bounds__(BINB) void k_rb_bin(GroupArgs ga, DenseView d, RbMap bm,
                                                 uint32_t nbk,
                                                 uint16_t* __restrict__ loff, uint32_t nsc,
                                                 RbEnt<sizeof(BT)>* __restrict__ tmp) {
  constexpr int kBinBlock = BINB;
  constexpr uint32_t SC = rb_sc<BT>(BINB);
  constexpr int KPT = (int)(SC / kBinBlock);  // keys per thread: 8 or 4
  constexpr int SLOTS = (int)(2 * SC);
  using Ent = RbEnt<sizeof(BT)>;
  using VT = typename std::conditional<MODE == 0, uint32_t, AT>::type;  // last index / sum
  constexpr size_t VBYTES = (size_t)(SLOTS + 1) * sizeof(VT);
  constexpr size_t VPAD = (VBYTES + 15) / 16 * 16;
  constexpr size_t TBL = VPAD + (size_t)(SLOTS + 1) * 4;
  static_assert(SC * sizeof(Ent) <= TBL, "the staging area fits over the table");
  __shared__ __attribute__((aligned(16))) unsigned char tbl[TBL];
  VT* hv = reinterpret_cast<VT*>(tbl);
  uint32_t* hk = reinterpret_cast<uint32_t*>(tbl + VPAD);
  Ent* stg = reinterpret_cast<Ent*>(tbl);
  __shared__ uint32_t cnt[kRbMaxBuckets + 1];  // bucket counters, then bucket starts
  __shared__ __attribute__((aligned(16))) uint32_t wtmp[kBinBlock / 64];
  __shared__ uint32_t sent;
  const int tid = threadIdx.x;
  auto clear = [&]() {
    for (uint32_t i = (uint32_t)tid * 16; i < (uint32_t)VPAD; i += kBinBlock * 16)
      *reinterpret_cast<u32x4*>(tbl + i) = u32x4{0u, 0u, 0u, 0u};
    for (int i = tid * 4; i < SLOTS; i += kBinBlock * 4)
      *reinterpret_cast<u32x4*>(&hk[i]) = u32x4{kEmpty32, kEmpty32, kEmpty32, kEmpty32};
    if (tid == 0) {
      hk[SLOTS] = kEmpty32;
      sent = 0;
    }
    for (uint32_t b = tid; b <= nbk; b += kBinBlock) cnt[b] = 0;
  };
  struct Task {
    int j;
    uint64_t base;
    uint32_t nvalid;
  };
  auto task = [&](uint32_t sc) {
    Task t;
    t.j = batch_of(ga, sc);
    t.base = (uint64_t)(sc - ga.wg_prefix[t.j]) * SC;
    const uint64_t n = ga.b[t.j].n;
    t.nvalid = n - t.base < SC ? (uint32_t)(n - t.base) : SC;
    return t;
  };
  auto li_of = [&](int q) { return (uint32_t)(((q / 4) * kBinBlock + tid) * 4 + (q % 4)); };
  auto load = [&](const Task& t, uint32_t (&k)[KPT], BT (&v)[KPT]) {
    const uint32_t* __restrict__ keys = ga.b[t.j].keys;
    const BT* __restrict__ vals = reinterpret_cast<const BT*>(ga.b[t.j].vals);
    const bool full = t.nvalid == SC && ((reinterpret_cast<uintptr_t>(keys) & 15u) == 0) &&
                      ((reinterpret_cast<uintptr_t>(vals) & 15u) == 0);
#pragma unroll
    for (int g = 0; g < KPT / 4; ++g) {
      const uint64_t i0 = t.base + li_of(g * 4);
      if (full) {
        uint32_t k4[4];
        BT v4[4];
        Vec4<uint32_t>::template load<true>(keys + i0, k4);
        Vec4<BT>::template load<true>(vals + i0, v4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          k[g * 4 + e] = k4[e];
          v[g * 4 + e] = v4[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool in = li_of(g * 4 + e) < t.nvalid;
          k[g * 4 + e] = in ? keys[i0 + e] : 0u;
          v[g * 4 + e] = in ? vals[i0 + e] : BT(0);
        }
      }
    }
  };
  clear();
  __syncthreads();
  uint32_t kc[KPT], kn[KPT];
  BT vc[KPT], vn[KPT];
  Task cur{}, nxt{};
  if (blockIdx.x < nsc) {
    cur = task(blockIdx.x);
    load(cur, kc, vc);
  }
  ready(kc);  // complete on entry as on the back edge: no wait at the loop top
  ready(vc);
  for (uint32_t sc = blockIdx.x, pass = 0; sc < nsc; sc += gridDim.x, ++pass) {
    K5_STAMP(0, pass, 0);
    // kc / vc are complete here (waited for at the end of the previous pass,
    // before its copy-out stores; the prologue's loads by the compiler): the
    // wait-count pass cannot count the next loads (their number depends on the
    // full / partial branch), so a first wait for kc AFTER them would be a
    // vmcnt(0) for the prefetch just issued
    ready(kc);
    ready(vc);
    if (sc + gridDim.x < nsc) {
      nxt = task(sc + gridDim.x);
      load(nxt, kn, vn);
    }
    uint32_t valid = 0;
#pragma unroll
    for (int q = 0; q < KPT; ++q) valid |= li_of(q) < cur.nvalid ? (1u << q) : 0u;
    uint32_t slot[KPT];
    // (Round 5 measured a streamed insert -- each lane walking its keys as one
    // stream of compare-and-swaps, a collided key retried in the next step
    // instead of in a probe round of its own: ~15 instead of ~27 CAS
    // instructions per wave in a model of the table, tools/k5_probe_model.py
    // -- and it LOST: insert 17.8 K against 15.5 K cycles per pass, K5 +2 %,
    // profiles/r05_probes/k5ab/.  Each step's dependent LDS round trip and
    // the ~50 VALU picking the lane's key and recording its slot cost more
    // than the probe instructions it saved.)
    // (round 5) the hybrid insert: insert phase 15.5 K -> 13.7 K cycles per
    // pass (assign; accumulate 18.3 K -> 17.1 K), K5 145.9 -> 142.8 us
    // (accumulate 195.1 -> 191.7) over 3 interleaved rounds,
    // profiles/r05_probes/k5ab_hybrid/
    const uint32_t own = lds_insert_hybrid<KPT, SLOTS>(hk, &sent, kc, valid, slot);
#pragma unroll
    for (int q = 0; q < KPT; ++q) {
      if (!(valid >> q & 1u)) continue;
      if (MODE == 0)
        atomicMax(reinterpret_cast<uint32_t*>(&hv[slot[q]]), li_of(q));
      else
        lds_add(reinterpret_cast<AT*>(&hv[slot[q]]), from_bits<AT>(to_bits<BT>(vc[q])));
    }
    __syncthreads();
    K5_STAMP(0, pass, 1);
    uint32_t emask = 0, rk[KPT], bk[KPT];  // bk: the kept entries' buckets
    BT kv[KPT];
#pragma unroll
    for (int q = 0; q < KPT; ++q) {
      bool keep;
      if (MODE == 0) {
        keep = (valid >> q & 1u) && *reinterpret_cast<const uint32_t*>(&hv[slot[q]]) == li_of(q);
        kv[q] = vc[q];
      } else {
        keep = (own >> q & 1u) != 0;
        kv[q] = keep ? from_bits<BT>(to_bits<AT>(*reinterpret_cast<const AT*>(&hv[slot[q]]))) : BT(0);
      }
      rk[q] = 0;
      bk[q] = 0;
      if (keep) {
        emask |= 1u << q;
        bk[q] = rb_bucket(d, kc[q], bm);
        rk[q] = atomicAdd(&cnt[bk[q]], 1u);
      }
    }
    __syncthreads();  // table read and every entry counted
    K5_STAMP(0, pass, 2);
    const uint32_t total = block_exscan<kBinBlock>(cnt, nbk + 1, wtmp);
    K5_STAMP(0, pass, 3);
    uint16_t* row = loff + (size_t)sc * (nbk + 1);
    for (uint32_t b = tid; b <= nbk; b += kBinBlock) row[b] = (uint16_t)cnt[b];
#pragma unroll
    for (int q = 0; q < KPT; ++q) {
      if (!(emask >> q & 1u)) continue;
      Ent e;
      e.key = kc[q];
      if (sizeof(BT) == 8) reinterpret_cast<uint32_t*>(&e)[1] = 0;
      e.val = kv[q];
      stg[cnt[bk[q]] + rk[q]] = e;
    }
    __syncthreads();
    K5_STAMP(0, pass, 4);
    // the staged, bucket-sorted entries out as one coalesced stream.  The
    // thread that copies a 16-byte piece also returns it to its cleared state
    // (hv zero, hk EMPTY; nobody else reads it), the pieces past the staged
    // ones are cleared in the same pass, and so are the bucket counters (last
    // read by the staging above): one barrier where copy and clear took two
    // the next super-chunk's registers complete HERE, before the copy-out
    // stores go out: waited for at the top of the next pass instead, the
    // in-order counter would also wait for those stores' acknowledgements
    ready(kn);
    ready(vn);
    const uint32_t n16 = (uint32_t)((total * sizeof(Ent) + 15) / 16);
    u32x4* dst = reinterpret_cast<u32x4*>(tmp + (size_t)sc * SC);
    u32x4* src = reinterpret_cast<u32x4*>(stg);
    constexpr uint32_t T16 = (uint32_t)((VPAD + (size_t)SLOTS * 4) / 16);
    static_assert((VPAD + (size_t)SLOTS * 4) % 16 == 0, "whole 16-byte pieces");
    for (uint32_t i = tid; i < T16; i += kBinBlock) {
      if (i < n16) dst[i] = src[i];
      const uint32_t z = (size_t)i * 16 < VPAD ? 0u : kEmpty32;
      src[i] = u32x4{z, z, z, z};
    }
    if (tid == 0) {
      hk[SLOTS] = kEmpty32;
      sent = 0;
    }
    for (uint32_t b = tid; b <= nbk; b += kBinBlock) cnt[b] = 0;
    __syncthreads();
    K5_STAMP(0, pass, 5);
#pragma unroll
    for (int q = 0; q < KPT; ++q) {
      kc[q] = kn[q];
      vc[q] = vn[q];
    }
    cur = nxt;
  }
}

// K5b k_rb_resolve: one 1024-thread workgroup per bucket (LDS: 128 KiB table,
// one workgroup per CU, 16 waves).  The bucket's entries are the runs
// [loff[sc][b], loff[sc][b+1]) of the super-chunk regions; thread t loads the
// run of super-chunk t straight into registers (one contiguous read; the few
// entries past RPT are read in a loop, and a bucket with a run longer than
// LONG takes the strided path below).  An LDS hash resolves the bucket — the largest position wins
// (assign) / values add (accumulate) — and the winners store into the dense
// array or the overflow table.  A bucket is owned by one workgroup: no
// cross-workgroup ordering, no global atomics.  Buckets are dealt XCD by XCD
// (workgroups b and b+8 share an XCD): one XCD's workgroups take consecutive
// buckets, so the loff lines they read stay in that XCD's L2; the next
// bucket's loff words are read while this one resolves.  Slot SLOTS belongs
// to the key 0xFFFFFFFF.
constexpr int kApplyBlock = 1024;
static_assert(kRbMaxSc <= (uint32_t)kApplyBlock, "one run per resolve thread");
template <typename AT, typename BT, int MODE, int LOGS>
__global__ __launch_bounds__(kApplyBlock) void k_rb_resolve(DenseView d, Ovf o, RbMap bm,
                                                            uint32_t nbk,
                                                            const uint16_t* __restrict__ loff,
                                                            uint32_t nsc, uint32_t SC,
                                                            const RbEnt<sizeof(BT)>* __restrict__ tmp) {
  // f64 sums take 8 B per slot: half the slots in the same LDS
  constexpr int SLOTS = (MODE == 1 && sizeof(AT) == 8) ? (1 << LOGS) / 2 : (1 << LOGS);
  constexpr uint32_t CAP = (uint32_t)SLOTS / 8 * 7;  // entries per round (load <= 7/8)
  // run entries held in registers: 10 for 4-byte values; 16-byte entries
  // (8-byte values) take 6, since 10 spilled (52-68 bytes of scratch a lane)
  constexpr int RPT = sizeof(BT) == 8 ? 6 : 10;
  constexpr uint32_t LONG = 4 * RPT;                  // longer runs: the strided path
  static_assert(LONG <= 64, "a run's winners fit one 64-bit mask");
  using Ent = RbEnt<sizeof(BT)>;
  // assign: keys ak[0..SLOTS] and 1 + max position abest[0..SLOTS] in one
  // array, which the direct path reuses whole as best[0..DSPAN)
  __shared__ __attribute__((aligned(16))) uint32_t ak[MODE == 0 ? 2 * SLOTS + 8 : SLOTS + 1];
  uint32_t* abest = ak + SLOTS + 4;  // 16-byte aligned
  __shared__ __attribute__((aligned(16))) AT asum[MODE == 1 ? SLOTS + 1 : 1];
  // Positions.  K5a keeps ONE entry per key per super-chunk (its last value /
  // its sum), so inside a run every key is distinct and the run's super-chunk
  // index alone orders two entries of a key: the later super-chunk is the
  // later write.  Assign therefore ranks entries by run index (no scan of the
  // run lengths is needed to order them); only the strided path scans, to
  // deal positions to threads.
  // assign, dense buckets: a direct-indexed table best[key offset in the
  // bucket's DSPAN-key window] = tag << kPosBits | (1 + run index); the tag
  // grows every pass, so stale values always lose and the table is never
  // cleared between buckets (only after a hash-path bucket used the memory)
  constexpr uint32_t DSPAN = MODE == 0 ? 2u * SLOTS : 1u;
  constexpr uint32_t kPosBits = 18;
  uint32_t* best = ak;
  // strided path: the starts of the nsc runs in position order (pre[nsc] =
  // entries)
  __shared__ uint32_t pre[kRbMaxSc + 1];
  __shared__ __attribute__((aligned(16))) uint32_t wtmp[kApplyBlock / 64];
  __shared__ uint32_t sent;
  // per-bucket totals (entries, longest virtual run), three slots in rotation:
  // iteration i adds into slot i % 3 and clears slot (i + 2) % 3, which was
  // last read in iteration i - 1, before this iteration's barrier
  __shared__ uint32_t s_tot[3], s_max[3];
  const int tid = threadIdx.x;
  const uint32_t nbd = bm.nbd;
  if (tid < 3) {
    s_tot[tid] = 0;
    s_max[tid] = 0;
  }
  __syncthreads();
  auto find = [&](uint32_t key) -> uint32_t {
    if (key == kEmpty32) return SLOTS;
    uint32_t h = fmix32(key) & (SLOTS - 1);
    while (ak[h] != key) h = (h + 1) & (SLOTS - 1);
    return h;
  };
  auto first_run = [&](uint32_t p) -> uint32_t {  // last run r with pre[r] <= p
    uint32_t lo = 0, hi = nsc;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pre[mid] <= p)
        lo = mid;
      else
        hi = mid;
    }
    return lo;
  };
  // the overflow table, loaded (after the room for it is reserved) when this
  // workgroup takes the out-of-range bucket
  OvfTab ot{};
  auto store_winner = [&](uint32_t b, uint32_t key, BT vbits) {
    const AT v = from_bits<AT>(to_bits<BT>(vbits));
    if (b != nbd) {
      reinterpret_cast<AT*>(d.param)[key - d.key_begin] = v;
    } else {
      const long long sl = ovf_insert(o, ot, key);
      if (sl >= 0) reinterpret_cast<AT*>(ot.vals)[sl] = v;
    }
  };
  auto accumulate_all = [&](uint32_t b) {
    // this workgroup owns every key of the bucket: plain read-modify-write
    if (b != nbd) {
      // dense bucket: every lane's parameter loads issued together, masked to
      // the used slots (~1 in 10 for cfg 3: unmasked clamped loads cost 7 %),
      // then the adds and stores
      constexpr int SPT = (SLOTS + 1 + kApplyBlock - 1) / kApplyBlock;
      AT* __restrict__ param = reinterpret_cast<AT*>(d.param);
      uint32_t off[SPT];
      uint32_t used = 0;
#pragma unroll
      for (int q = 0; q < SPT; ++q) {
        const int s = q * kApplyBlock + tid;
        const bool u = s < SLOTS ? ak[s] != kEmpty32 : (s == SLOTS && sent != 0);
        const uint32_t key = s < SLOTS ? ak[s] : kEmpty32;
        off[q] = u ? key - d.key_begin : 0u;
        used |= u ? (1u << q) : 0u;
      }
      AT cur[SPT];
#pragma unroll
      for (int q = 0; q < SPT; ++q)
        if (used >> q & 1u) cur[q] = param[off[q]];
#pragma unroll
      for (int q = 0; q < SPT; ++q)
        if (used >> q & 1u) param[off[q]] = add_wrap<AT>(cur[q], asum[q * kApplyBlock + tid]);
      return;
    }
    for (int s = tid; s <= SLOTS; s += kApplyBlock) {
      const bool used = s == SLOTS ? sent != 0 : ak[s] != kEmpty32;
      if (!used) continue;
      const uint32_t key = s == SLOTS ? kEmpty32 : ak[s];
      const long long sl = ovf_insert(o, ot, key);
      if (sl < 0) continue;
      AT* p = reinterpret_cast<AT*>(ot.vals) + sl;
      *p = add_wrap<AT>(*p, asum[s]);
    }
  };
  auto clear_table = [&]() {
    // 16-byte LDS writes (SLOTS is a multiple of 4 * kApplyBlock)
    for (int s = tid * 4; s < SLOTS; s += kApplyBlock * 4) {
      *reinterpret_cast<u32x4*>(&ak[s]) = u32x4{kEmpty32, kEmpty32, kEmpty32, kEmpty32};
      if (MODE == 0) {
        *reinterpret_cast<u32x4*>(&abest[s]) = u32x4{0u, 0u, 0u, 0u};
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) asum[s + e] = AT(0);
      }
    }
    if (tid == 0) {
      ak[SLOTS] = kEmpty32;
      if (MODE == 0)
        abest[SLOTS] = 0;
      else
        asum[SLOTS] = AT(0);
      sent = 0;
    }
  };
  auto insert_one = [&](uint32_t key, uint32_t pos, BT vbits) {
    uint32_t k1[1] = {key}, s1[1];
    lds_insert<1, SLOTS>(ak, &sent, k1, 1u, s1);
    if (MODE == 0)
      atomicMax(&abest[s1[0]], pos + 1u);
    else
      lds_add(&asum[s1[0]], from_bits<AT>(to_bits<BT>(vbits)));
  };
  // XCD-aware bucket schedule
  const uint32_t xcd = blockIdx.x & 7u;
  const uint32_t per_xcd = (gridDim.x + 7u - xcd) >> 3;  // workgroups in this XCD group
  const uint32_t b_hi = (uint32_t)((uint64_t)nbk * (xcd + 1) / 8);
  uint32_t b = (uint32_t)((uint64_t)nbk * xcd / 8) + (blockIdx.x >> 3);
  const bool has_run = (uint32_t)tid < nsc;
  const uint32_t rowo = has_run ? (uint32_t)tid * (nbk + 1) : 0u;  // this thread's loff row
  const uint32_t st0 = (uint32_t)tid * SC;                           // its region in tmp
  const uint32_t pos = (uint32_t)tid + 1u;  // its run index (the entries' position), plus one
  // software pipeline: the run of bucket b in registers, the run bounds of the
  // bucket after it in flight.  The bounds loads are unconditional (a thread
  // without a run, or past the last bucket, reads a valid word it then
  // ignores) so nothing waits for them until the next bucket uses them.
  auto bounds_ok = [&](uint32_t bb) { return bb < b_hi && has_run; };
  auto bounds = [&](uint32_t bb, uint32_t& a, uint32_t& e) {
    const uint32_t i = rowo + (bb < b_hi ? bb : 0u);
    a = loff[i];
    e = loff[i + 1];
  };
  // 8-byte entries go two per 16-byte load (dword alignment suffices): half
  // the load instructions, and each lane of one touches a line of its own
  // run, so the address unit's work per bucket halves too.  A run of odd
  // length reads one entry past its end: the next run's, or the scratch
  // buffer's tail pad (launch_rb_add's caller allocates kRbTmpPad bytes more).
  auto load_run = [&](uint32_t a, uint32_t e, Ent (&x)[RPT]) {
    if constexpr (sizeof(Ent) == 8) {
      static_assert(RPT % 2 == 0, "whole pairs");
#pragma unroll
      for (int q = 0; q < RPT; q += 2)
        if ((uint32_t)q < e - a) {
          uint32_t w[4];
          ld16a4<false>(reinterpret_cast<const uint32_t*>(tmp + st0 + a + q), w);
          x[q].key = w[0];
          reinterpret_cast<uint32_t*>(&x[q])[1] = w[1];
          x[q + 1].key = w[2];
          reinterpret_cast<uint32_t*>(&x[q + 1])[1] = w[3];
        }
    } else {
#pragma unroll
      for (int q = 0; q < RPT; ++q)
        if ((uint32_t)q < e - a) x[q] = tmp[st0 + a + q];
    }
  };
  uint32_t dlog = 0;
  while ((1u << dlog) < DSPAN) ++dlog;
  const uint32_t halves = (uint32_t)(((uint64_t)bm.span + DSPAN - 1) >> dlog);  // direct passes per bucket
  bool clean = false;  // best[] holds only values below tag << kPosBits
  uint32_t tag = 0;
  auto zero_best = [&]() {
    for (uint32_t i = (uint32_t)tid * 4; i < DSPAN; i += kApplyBlock * 4)
      *reinterpret_cast<u32x4*>(&best[i]) = u32x4{0u, 0u, 0u, 0u};
  };
  uint32_t ra, re, na, ne_;
  bounds(b, ra, re);
  if (!bounds_ok(b)) ra = re = 0;
  bounds(b + per_xcd, na, ne_);
  Ent xn[RPT];
  load_run(ra, re, xn);
  uint32_t it = 0;
  for (uint32_t pass = 0; b < b_hi; b += per_xcd, it = it == 2u ? 0u : it + 1u, ++pass) {
    K5_STAMP(1, pass, 0);
    const uint32_t len = re - ra, st = st0 + ra;
    Ent x[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) x[q] = xn[q];
    // next bucket: its run loads now, the bounds of the one after
    ra = bounds_ok(b + per_xcd) ? na : 0u;
    re = bounds_ok(b + per_xcd) ? ne_ : 0u;
    load_run(ra, re, xn);
    bounds(b + 2 * per_xcd, na, ne_);
    {
      uint32_t ws = len, wm = len;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        ws += __shfl_xor(ws, o, 64);
        wm = max(wm, (uint32_t)__shfl_xor(wm, o, 64));
      }
      if ((tid & 63) == 0 && ws != 0) {
        atomicAdd(&s_tot[it], ws);
        atomicMax(&s_max[it], wm);
      }
    }
    __syncthreads();
    K5_STAMP(1, pass, 1);
    const uint32_t ne = s_tot[it];
    const bool long_run = s_max[it] > LONG;
    if (tid == 0) {
      const uint32_t z = it == 0u ? 2u : it - 1u;  // (it + 2) % 3
      s_tot[z] = 0;
      s_max[z] = 0;
    }
    if (ne == 0) continue;  // uniform
    if (b == nbd) {  // uniform: the out-of-range bucket, at most ne new keys
      ovf_reserve<sizeof(AT)>(o, ne);
      ot = ovf_tab(o);
    }
    const bool direct = MODE == 0 && b != nbd && !long_run && halves <= 4;
    if (direct) {
      uint32_t rel[RPT];
#pragma unroll
      for (int q = 0; q < RPT; ++q) rel[q] = (uint32_t)q < len ? rb_local(bm, x[q].key - d.key_begin) : 0u;
      // every pass only marks this lane's winners (bit q of win); the stores
      // of all passes go out together afterwards, so the random parameter
      // stores of the whole bucket are in flight at once
      uint64_t win = 0;
      for (uint32_t h = 0; h < halves; ++h) {
        if (!clean || tag + 1 >= (1u << (32 - kPosBits))) {  // uniform
          zero_best();
          __syncthreads();
          clean = true;
          tag = 0;
        }
        const uint32_t tg = ++tag << kPosBits;
#pragma unroll
        for (int q = 0; q < RPT; ++q)
          if ((uint32_t)q < len && (rel[q] >> dlog) == h)
            atomicMax(&best[rel[q] & (DSPAN - 1)], tg | pos);
        for (uint32_t q = RPT; q < len; ++q) {  // a run's short tail, from memory
          const uint32_t rl = rb_local(bm, tmp[st + q].key - d.key_begin);
          if ((rl >> dlog) == h) atomicMax(&best[rl & (DSPAN - 1)], tg | pos);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < RPT; ++q)
          if ((uint32_t)q < len && (rel[q] >> dlog) == h && best[rel[q] & (DSPAN - 1)] == (tg | pos))
            win |= 1ull << q;
        for (uint32_t q = RPT; q < len; ++q) {
          const uint32_t rl = rb_local(bm, tmp[st + q].key - d.key_begin);
          if ((rl >> dlog) == h && best[rl & (DSPAN - 1)] == (tg | pos)) win |= 1ull << q;
        }
        if (h + 1 < halves) __syncthreads();  // the table is read before the next pass
      }
      K5_STAMP(1, pass, 2);
#pragma unroll
      for (int q = 0; q < RPT; ++q)
        if (win >> q & 1u) store_winner(b, x[q].key, (BT)x[q].val);
      for (uint32_t q = RPT; q < len; ++q)
        if (win >> q & 1u) {
          const Ent y = tmp[st + q];
          store_winner(b, y.key, (BT)y.val);
        }
      // the next bucket's first atomics come after its scan's barriers, so
      // the reads above are done before best[] changes again
      continue;
    }
    clean = false;  // the hash paths below overwrite best[]
    if (ne <= CAP && !long_run) {
      clear_table();
      __syncthreads();
      uint32_t key[RPT], slot[RPT], valid = 0;
#pragma unroll
      for (int q = 0; q < RPT; ++q) {
        valid |= (uint32_t)q < len ? (1u << q) : 0u;
        key[q] = (uint32_t)q < len ? x[q].key : 0u;
      }
      // the hybrid insert here too (round 5): accumulate K5 191.8 -> 190.0 us
      // over 3 interleaved rounds, assign (mostly the direct path) unchanged,
      // profiles/r05_probes/k5b_hybrid/
      lds_insert_hybrid<RPT, SLOTS>(ak, &sent, key, valid, slot);
#pragma unroll
      for (int q = 0; q < RPT; ++q) {
        if (!(valid >> q & 1u)) continue;
        if (MODE == 0)
          atomicMax(&abest[slot[q]], pos);
        else
          lds_add(&asum[slot[q]], from_bits<AT>(to_bits<BT>((BT)x[q].val)));
      }
      for (uint32_t q = RPT; q < len; ++q) {  // a run's short tail (<= LONG - RPT), from memory
        const Ent y = tmp[st + q];
        insert_one(y.key, pos - 1u, (BT)y.val);
      }
      __syncthreads();
      if (MODE == 0) {
#pragma unroll
        for (int q = 0; q < RPT; ++q)
          if ((valid >> q & 1u) && abest[slot[q]] == pos)
            store_winner(b, key[q], (BT)x[q].val);
        for (uint32_t q = RPT; q < len; ++q) {
          const Ent y = tmp[st + q];
          if (abest[find(y.key)] == pos) store_winner(b, y.key, (BT)y.val);
        }
      } else {
        accumulate_all(b);
      }
      __syncthreads();
    } else {
      // a run longer than the registers hold, or more entries than the table
      // holds: every thread takes positions tid, tid + 1024, ... (coalesced
      // inside long runs), found by binary search over the starts of the nsc
      // runs (pre, rewritten per run); rounds split an oversized bucket by key
      // hash.  Run j's entries start at j * SC + its loff word.
      pre[tid] = len;
      __syncthreads();  // block_exscan reads other threads' words first
      (void)block_exscan<kApplyBlock>(pre, kApplyBlock, wtmp);
      if (tid == 0) pre[nsc] = ne;
      __syncthreads();
      auto run_ent = [&](uint32_t j, uint32_t p) -> Ent {
        return tmp[j * SC + loff[j * (nbk + 1) + b] + (p - pre[j])];
      };
      const uint32_t R = (ne + CAP - 1) / CAP;
      for (uint32_t round = 0; round < R; ++round) {
        clear_table();
        __syncthreads();
        for (uint32_t p = tid; p < ne; p += kApplyBlock) {
          const uint32_t j = first_run(p);
          const Ent y = run_ent(j, p);
          if ((fmix32(y.key ^ 0x9E3779B9u) % R) == round) insert_one(y.key, j, (BT)y.val);
        }
        __syncthreads();
        if (MODE == 0) {
          // the entry holding its key's largest position is the last write
          for (uint32_t p = tid; p < ne; p += kApplyBlock) {
            const uint32_t j = first_run(p);
            const Ent y = run_ent(j, p);
            if ((fmix32(y.key ^ 0x9E3779B9u) % R) != round) continue;
            if (abest[find(y.key)] == j + 1u) store_winner(b, y.key, (BT)y.val);
          }
        } else {
          accumulate_all(b);
        }
        __syncthreads();
      }
    }
  }
}

// ------------------------------------------ K4r conditional group replay
// The safety net behind the sorted paths (K2 / K2g verify their hint on every
// element and tag `cond` with the call's epoch on any violation; K7 behind
// K6's density proof).  ONE workgroup replays the whole group in call order:
// batch by batch, 4 Ki elements per pass, each pass resolved in an LDS hash
// (assign: the largest element index of a key wins, map_storage.hpp:22-23;
// accumulate: the pass's sum of a key, added by the key's first occurrence),
// the passes separated by workgroup barriers, so later passes' stores land
// last (one CU: its vector memory operations reach L2 in order).  That
// overwrites every key the group touched with its sequential value, whatever
// the sorted pass wrote — a wrong hint costs time, never correctness.
// Why one workgroup: the launch sits behind EVERY hinted group and almost
// always exits at once, so what matters is its idle cost — one launch of one
// workgroup (the two-launch, grid-wide K4a/K4b repair it replaces cost two
// kernel boundaries per step) — not the speed of a repair that only a broken
// hint triggers (~1 GB/s: 64 M keys take ~0.3 s).
constexpr int kReplayBlock = 1024;

// BLOCK threads (K4r: 1024; K1r: 256), 4 * BLOCK elements per pass; G is
// GroupArgs or ReplayGroup (only nb and b[] are read).  The pass's table --
// hk[SLOTS], assign: hidx[SLOTS + 1] (1 + largest local index), accumulate:
// hsum[SLOTS + 1] (the pass's sums), the sentinel's word -- is K4r's LDS, or
// for K1r a small global scratch (its atomics resolve in this XCD's L2; the
// barriers order them within the workgroup), so that K1r, which almost never
// replays, allocates no LDS.
template <int BLOCK>
constexpr int replay_slots() {
  return 8 * BLOCK;
}
template <typename VT, int MODE, int BLOCK = kReplayBlock, typename G = GroupArgs, bool OOR_ONLY = false>
__device__ __forceinline__ void replay_group(const G& ga, const DenseView& d, const Ovf& o, uint32_t* hk,
                                             uint32_t* hidx, VT* hsum, uint32_t* sent_p) {
  constexpr int CHUNK = 4 * BLOCK, SLOTS = replay_slots<BLOCK>();
  constexpr int PER = CHUNK / BLOCK;
  uint32_t& sent = *sent_p;
  const int tid = threadIdx.x;
  // Room in the overflow table for the group's out-of-range keys, reserved once
  // before the passes: a read of the group's keys counts their occurrences (a
  // bound on the new keys; the replay runs at ~1 GB/s, the count is noise),
  // summed in the sentinel word, which the first pass then clears.  (Once, not
  // per pass: the reservation then holds no pass state live, and K1r keeps
  // its register count.)
  {
    uint32_t c = 0;
    for (int j = 0; j < ga.nb; ++j)
      for (uint64_t i = (uint64_t)tid; i < ga.b[j].n; i += BLOCK)
        c += (uint64_t)(uint32_t)(ga.b[j].keys[i] - d.key_begin) >= d.range ? 1u : 0u;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) c += (uint32_t)__shfl_xor((int)c, w, 64);
    if (tid == 0) __hip_atomic_store(&sent, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if ((tid & 63) == 0 && c != 0u) atomicAdd(&sent, c);
    __syncthreads();
    const uint32_t total = __hip_atomic_load(&sent, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();  // every wave has read it before the first pass clears the word
    if (total != 0u) ovf_reserve<sizeof(VT)>(o, total);  // uniform
  }
  const OvfTab ot = ovf_tab(o);
  for (int j = 0; j < ga.nb; ++j) {
    const uint32_t* __restrict__ keys = ga.b[j].keys;
    const VT* __restrict__ vals = reinterpret_cast<const VT*>(ga.b[j].vals);
    const uint64_t n = ga.b[j].n;
    for (uint64_t base = 0; base < n; base += CHUNK) {
      for (int s = tid; s < SLOTS; s += BLOCK) {
        hk[s] = kEmpty32;
        if (MODE == 0)
          hidx[s] = 0u;
        else
          hsum[s] = VT(0);
      }
      if (tid == 0) {
        sent = 0u;
        if (MODE == 0)
          hidx[SLOTS] = 0u;
        else
          hsum[SLOTS] = VT(0);
      }
      __syncthreads();  // also orders the previous pass's stores before this pass's
      uint32_t key[PER], slot[PER], valid = 0;
      VT v[PER];
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const uint64_t i = base + (uint64_t)(q * BLOCK + tid);
        const bool in = i < n;
        key[q] = in ? keys[i] : 0u;
        // OOR_ONLY (behind K4): only the out-of-range keys; K4 applied the rest
        const bool take = in && (!OOR_ONLY || (uint64_t)(uint32_t)(key[q] - d.key_begin) >= d.range);
        valid |= take ? (1u << q) : 0u;
        v[q] = take ? vals[i] : VT(0);
      }
      const uint32_t own = lds_insert<PER, SLOTS>(hk, &sent, key, valid, slot);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        if (!(valid >> q & 1u)) continue;
        if (MODE == 0)
          atomicMax(&hidx[slot[q]], (uint32_t)(q * BLOCK + tid) + 1u);
        else
          lds_add(&hsum[slot[q]], v[q]);
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        if (!(valid >> q & 1u)) continue;
        const uint32_t off = key[q] - d.key_begin;
        if (MODE == 0) {
          // (an atomic load: in K1r's global table the maxima were resolved in L2,
          // and a plain load could hit a line this CU's L1 holds from an
          // earlier pass)
          if (__hip_atomic_load(&hidx[slot[q]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
              (uint32_t)(q * BLOCK + tid) + 1u)
            continue;  // a later occurrence wins
          if ((uint64_t)off < d.range) {
            reinterpret_cast<VT*>(d.param)[off] = v[q];
          } else {
            const long long sl = ovf_insert(o, ot, key[q]);
            if (sl >= 0) reinterpret_cast<VT*>(ot.vals)[sl] = v[q];
          }
        } else {
          if (!(own >> q & 1u)) continue;  // the key's inserting lane adds the pass's sum
          VT* p = nullptr;
          if ((uint64_t)off < d.range) {
            p = reinterpret_cast<VT*>(d.param) + off;
          } else {
            const long long sl = ovf_insert(o, ot, key[q]);
            if (sl >= 0) p = reinterpret_cast<VT*>(ot.vals) + sl;
          }
          if (p) *p = add_wrap<VT>(*p, hsum[slot[q]]);
        }
      }
      __syncthreads();  // the table is read before the next pass clears it
    }
  }
}

template <typename VT, int MODE, bool OOR_ONLY>
__global__ __launch_bounds__(kReplayBlock) void k_replay(GroupArgs ga, DenseView d, Ovf o,
                                                         const uint32_t* cond, uint32_t epoch) {
  constexpr int SLOTS = replay_slots<kReplayBlock>();
  __shared__ uint32_t hk[SLOTS];
  __shared__ uint32_t hidx[MODE == 0 ? SLOTS + 1 : 1];
  __shared__ VT hsum[MODE == 1 ? SLOTS + 1 : 1];
  __shared__ uint32_t sent;
  if (*cond != epoch) return;  // the hint held / no out-of-range key (the usual case)
  replay_group<VT, MODE, kReplayBlock, GroupArgs, OOR_ONLY>(ga, d, o, hk, hidx, hsum, &sent);
}

// K1r: K1 carrying the conditional replay of the assign group just before it
// (pskv_add_get_grouped: the Add's last launch group, then the Get's first) --
// the idle K4r launch between K2g and K1 cost ~1 us of a rank's ~40 us step
// and ~3 us of the headline's 200 (profiles/r04_probes/no_replay/).  Almost
// always the hint held and every workgroup gathers its chunk as K1 does.  When
// the Add's verification tagged `cond`, no parameter may be read before the
// replay has rewritten the group's keys, and workgroups of one launch cannot
// safely wait for one another, so workgroup 0 does all of it -- the replay
// (256 threads, 1 Ki elements per pass) and then every chunk of the Get in
// turn -- while the others leave at once.  Slow (a broken hint already pays a
// one-workgroup replay), never a wait between workgroups.
template <typename VT, bool VEC, int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_gather_r(GroupArgs ga, DenseView d, Ovf o, ReplayGroup rg,
                                                     const uint32_t* cond, uint32_t epoch, uint32_t* tab) {
  const uint32_t tag = *cond;  // waited for after this chunk's key loads are issued
  bool tagged = false;
  gather_chunk<VT, VEC, U, NT>(ga, d, o, blockIdx.x, [&]() {
    tagged = tag == epoch;  // uniform
    return !tagged;
  });
  if (tagged && blockIdx.x == 0) {
    // the table in global scratch (kK1rTableWords words): hk, hidx, the sentinel word
    constexpr int SLOTS = replay_slots<kBlock>();
    static_assert(2 * SLOTS + 2 <= (int)kK1rTableWords, "K1r's replay table fits its scratch");
    replay_group<VT, 0, kBlock>(rg, d, o, tab, tab + SLOTS, static_cast<VT*>(nullptr), tab + 2 * SLOTS + 1);
    // (ends with a barrier: its stores precede the loads below)
    // (FRESH: the replay may have grown the overflow table in this kernel)
    for (uint32_t w = 0; w < gridDim.x; ++w) gather_chunk<VT, VEC, U, NT, GoAlways, true>(ga, d, o, w);
  }
}

// ------------------------------------------- K6/K7 dense accumulate
// Accumulate for grouped batches that are each one contiguous key window
// (first_j .. first_j + n_j - 1): no atomics and no duplicates to resolve.
// Every key gets exactly ONE read-modify-write, by the element of the
// EARLIEST batch that covers it, which adds that batch's value and then the
// values of every later covering batch in call order — so the result is the
// sequential sum p + v_0 + v_1 + ... bit for bit.  Because the RMW cannot be
// undone, density is proven BEFORE it runs:
//   K6 k_dense_check  reads the keys only; tags `flag` with the call's epoch
//                     unless every batch is exactly dense and in range
//   K7 k_acc_dense    skips when tagged; K4a accumulate (conditional on the
//                     tag) takes the group instead
// Host-staged batches are proven dense on the CPU while copied, so K6 and the
// K4a fallback are not launched for them.

template <int U>
__global__ __launch_bounds__(kBlock) void k_dense_check(GroupArgs ga, DenseView d, uint32_t* flag,
                                                        uint32_t epoch) {
  constexpr int CH = kBlock * 4 * U;
  const uint32_t wg = blockIdx.x;
  const int j = batch_of(ga, wg);
  const uint32_t* __restrict__ keys = ga.b[j].keys;
  const uint64_t n = ga.b[j].n;
  const uint64_t base = (uint64_t)(wg - ga.wg_prefix[j]) * CH;
  const int tid = threadIdx.x;
  const uint32_t first = keys[0];
  const uint64_t off = (uint32_t)(first - d.key_begin);
  bool bad = off >= d.range || off + n > d.range;
  if (base + CH <= n && (reinterpret_cast<uintptr_t>(keys) & 15u) == 0) {
    uint32_t k[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
      Vec4<uint32_t>::load<true>(keys + base + (uint64_t)(u * kBlock + tid) * 4, k[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k0 = first + (uint32_t)(base + (uint64_t)(u * kBlock + tid) * 4);
      bad |= (k[u][0] != k0) | (k[u][1] != k0 + 1u) | (k[u][2] != k0 + 2u) | (k[u][3] != k0 + 3u);
    }
  } else {
    const uint64_t end = n < base + CH ? n : base + CH;
    for (uint64_t i = base + tid; i < end; i += kBlock) bad |= keys[i] != first + (uint32_t)i;
  }
  if (__any(bad) && (tid & 63) == 0) *flag = epoch;
}

template <typename AT>
struct Bits;
template <>
struct Bits<int> {
  using T = uint32_t;
};
template <>
struct Bits<float> {
  using T = uint32_t;
};
template <>
struct Bits<double> {
  using T = unsigned long long;
};

template <typename AT, int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_acc_dense(GroupArgs ga, DenseView d,
                                                      const uint32_t* flag, uint32_t epoch) {
  using BT = typename Bits<AT>::T;
  constexpr int CH = kBlock * 4 * U;
  if (*flag == epoch) return;  // K6 found a batch that is not a dense window
  __shared__ uint32_t s_first[kMaxBatches];
  __shared__ uint32_t s_last[kMaxBatches];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  if (tid < 64) {
    uint32_t f = 0, l = 0;
    if (lane < ga.nb) {
      f = ga.b[lane].keys[0];
      l = f + (uint32_t)(ga.b[lane].n - 1);
    }
    s_first[lane] = f;
    s_last[lane] = l;
  }
  __syncthreads();
  AT* __restrict__ param = reinterpret_cast<AT*>(d.param);
  const uint32_t nchunks = ga.wg_prefix[ga.nb];
  for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int j = batch_of(ga, c);
    const AT* __restrict__ vals = reinterpret_cast<const AT*>(ga.b[j].vals);
    const uint64_t n = ga.b[j].n;
    const uint64_t base = (uint64_t)(c - ga.wg_prefix[j]) * CH;
    const uint64_t end = n < base + CH ? n : base + CH;
    const uint32_t first = s_first[j];
    const uint32_t c_lo = first + (uint32_t)base, c_hi = first + (uint32_t)(end - 1);
    const bool meets = lane < ga.nb && lane != j && s_first[lane] <= c_hi && s_last[lane] >= c_lo;
    const unsigned long long earlier = __ballot(meets && lane < j);
    const unsigned long long later = __ballot(meets && lane > j);
    // an earlier batch covering the whole chunk owns every key: nothing to load
    if (__ballot(meets && lane < j && s_first[lane] <= c_lo && s_last[lane] >= c_hi)) continue;
    // the single RMW of key k, issued by batch j's element when j is the
    // earliest batch covering k
    auto rmw = [&](uint32_t k, AT v) {
      unsigned long long m = earlier;
      bool owned_earlier = false;
      while (m) {
        const int q = __ffsll((long long)m) - 1;
        m &= m - 1;
        owned_earlier |= (k >= s_first[q]) & (k <= s_last[q]);
      }
      if (owned_earlier) return;
      const uint32_t off = k - d.key_begin;
      AT acc = add_wrap<AT>(param[off], v);
      m = later;
      while (m) {  // ascending batch index = call order
        const int q = __ffsll((long long)m) - 1;
        m &= m - 1;
        if ((k >= s_first[q]) & (k <= s_last[q]))
          acc = add_wrap<AT>(acc, reinterpret_cast<const AT*>(ga.b[q].vals)[k - s_first[q]]);
      }
      param[off] = acc;
    };
    const bool vec_ok = ((reinterpret_cast<uintptr_t>(vals) & 15u) == 0) && end - base == CH;
    if (vec_ok) {
      // N values per lane per 16-byte access: 4 (4-byte values) or 2 (8-byte,
      // see Vec2x8); UU steps keep the chunk at CH keys
      constexpr int N = VecN<BT>::N;
      constexpr int UU = U * 4 / N;
      BT v[UU][N];
#pragma unroll
      for (int u = 0; u < UU; ++u)
        VecN<BT>::template load<NT>(reinterpret_cast<const BT*>(vals) + base +
                                        (uint64_t)(u * kBlock + tid) * N,
                                    v[u]);
      if (earlier == 0 && ((first - d.key_begin) & (uint32_t)(N - 1)) == 0) {
        // no earlier batch meets this chunk (the common case), aligned: 16-B
        // RMW; later batches meeting it add their values in call order
        BT p[UU][N];
        BT* pb = reinterpret_cast<BT*>(param) + (first - d.key_begin) + base;
#pragma unroll
        for (int u = 0; u < UU; ++u) VecN<BT>::load(pb + (uint64_t)(u * kBlock + tid) * N, p[u]);
#pragma unroll
        for (int u = 0; u < UU; ++u) {
#pragma unroll
          for (int e = 0; e < N; ++e)
            p[u][e] = to_bits<AT>(add_wrap<AT>(from_bits<AT>(p[u][e]), from_bits<AT>(v[u][e])));
        }
        unsigned long long m = later;
        while (m) {
          const int q = __ffsll((long long)m) - 1;
          m &= m - 1;
          const uint32_t fq = s_first[q], lq = s_last[q];
          const BT* __restrict__ vq = reinterpret_cast<const BT*>(ga.b[q].vals);
#pragma unroll
          for (int u = 0; u < UU; ++u) {
            const uint32_t k0 = first + (uint32_t)(base + (uint64_t)(u * kBlock + tid) * N);
            BT w[N];
            if (k0 >= fq && k0 + (uint32_t)(N - 1) <= lq &&
                (((k0 - fq) & (uint32_t)(N - 1)) | (reinterpret_cast<uintptr_t>(vq) & 15u)) == 0) {
              VecN<BT>::template load<NT>(vq + (k0 - fq), w);
#pragma unroll
              for (int e = 0; e < N; ++e)
                p[u][e] = to_bits<AT>(add_wrap<AT>(from_bits<AT>(p[u][e]), from_bits<AT>(w[e])));
            } else {
#pragma unroll
              for (int e = 0; e < N; ++e)
                if (k0 + e >= fq && k0 + e <= lq)
                  p[u][e] = to_bits<AT>(add_wrap<AT>(from_bits<AT>(p[u][e]), from_bits<AT>(vq[k0 + e - fq])));
            }
          }
        }
#pragma unroll
        for (int u = 0; u < UU; ++u) VecN<BT>::store(pb + (uint64_t)(u * kBlock + tid) * N, p[u]);
      } else {
#pragma unroll
        for (int u = 0; u < UU; ++u) {
          const uint32_t k0 = first + (uint32_t)(base + (uint64_t)(u * kBlock + tid) * N);
#pragma unroll
          for (int e = 0; e < N; ++e) rmw(k0 + e, from_bits<AT>(v[u][e]));
        }
      }
    } else {
      for (uint64_t i = base + tid; i < end; i += kBlock) rmw(first + (uint32_t)i, vals[i]);
    }
  }
}


// ------------------------------------------------ K8 inline small messages
// The reference's live traffic is many small messages: a logistic-regression
// worker pushes and pulls one sample's features at a time (tens of keys,
// app/logistic_regression.cpp:411,490), sliced over the server threads.  For
// those the cost of a call is latency, not bandwidth: staging DMAs (H2D of keys
// and values, D2H of the reply) and their completion waits dominate.  Here the
// keys (and an Add's values) travel INSIDE the kernel arguments — the launch
// packet's kernarg segment is the only host->device transfer — and a Get writes
// its reply straight into page-locked host memory.  One workgroup does the
// whole message with the reference's sequential semantics:
//   assign      element i stores iff no later element has its key (last wins,
//               map_storage.hpp:22-23)
//   accumulate  the FIRST occurrence of a key adds every occurrence's value in
//               index order: ((p + v_a) + v_b) + ..., bit-identical to the
//               sequential loop
// Distinct threads write distinct keys, and calls are stream-ordered, so no
// atomics are needed on the dense array (the overflow table's insert uses its
// usual CAS).

template <typename VT, int MODE>
__global__ __launch_bounds__(kInlineMax) void k_inline_add(InlineAdd a, DenseView d, Ovf o) {
  // Every lane walks the whole message with a wave-UNIFORM index, so each key
  // and value is one scalar load from the kernarg segment shared by the wave
  // (a per-lane start index would turn the walk into dependent vector loads,
  // ~10 us at 256 keys).
  const int tid = threadIdx.x;
  const int n = (int)a.n;
  const uint32_t k = tid < n ? a.keys[tid] : 0u;
  using BT = typename std::conditional<sizeof(VT) == 8, unsigned long long, uint32_t>::type;
  const uint32_t off = k - d.key_begin;
  // room for the message's new out-of-range keys first (every thread: the
  // reservation is a workgroup step)
  const bool outside = tid < n && (uint64_t)off >= d.range;
  const int n_out = __syncthreads_count(outside);
  OvfTab ot{};
  if (n_out) {
    ovf_reserve<sizeof(VT)>(o, (uint64_t)n_out);
    ot = ovf_tab(o);
  }
  if (MODE == 0) {
    bool later = false;
#pragma unroll 16
    for (int j = 0; j < n; ++j) later |= (j > tid) & (a.keys[j] == k);
    if (tid >= n || later) return;  // a later occurrence wins
    const BT v = (BT)a.vals[tid];
    if (!outside) {
      reinterpret_cast<BT*>(d.param)[off] = v;
    } else {
      const long long slot = ovf_insert(o, ot, k);
      if (slot >= 0) reinterpret_cast<BT*>(ot.vals)[slot] = v;
    }
  } else {
    bool earlier = false;
#pragma unroll 16
    for (int j = 0; j < n; ++j) earlier |= (j < tid) & (a.keys[j] == k);
    if (tid >= n || earlier) return;  // the first occurrence sums them all
    VT* p;
    if (!outside) {
      p = reinterpret_cast<VT*>(d.param) + off;
    } else {
      const long long slot = ovf_insert(o, ot, k);
      if (slot < 0) return;
      p = reinterpret_cast<VT*>(ot.vals) + slot;
    }
    VT acc = *p;
#pragma unroll 16
    for (int j = 0; j < n; ++j)  // index order: the sequential loop's sum, bit for bit
      if ((j >= tid) & (a.keys[j] == k)) acc = add_wrap<VT>(acc, from_bits<VT>(a.vals[j]));
    *p = acc;
  }
}

// One wave: its own stores are the whole reply, so when `done` is given (the
// spin-wait reply) lane 0 can publish it with a system-scope release and a
// sequence number the host polls — no cross-wave hand-off to order.
template <typename VT>
__global__ __launch_bounds__(64) void k_inline_get(InlineGet a, DenseView d, Ovf o, VT* out,
                                                   unsigned int* done, unsigned int seq) {
  // every lane's gathers first (independent, all in flight), then the reply
  // stores: interleaved, each store would wait for its own load
  constexpr int PER = kInlineGetMax / 64;
  VT v[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const uint32_t i = threadIdx.x + 64u * q;
    v[q] = i < a.n ? load_one<VT>(d, o, a.keys[i]) : VT(0);
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const uint32_t i = threadIdx.x + 64u * q;
    if (i < a.n) out[i] = v[q];
  }
  if (done) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the reply before the flag
    // MI355X_MICROARCH.md "Compiler hazard": keep the wait after the write-back
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// K9 k_serve: the small-message server.  One resident workgroup polls the
// request ring (coherent page-locked host memory) and applies each request in
// ring order with K8's semantics: a small Add or Get then costs the host a
// ring slot and a sequence number instead of a kernel launch.  Lane 0 polls
// req_seq with system-scope loads that bypass the caches; up to kSrvBatch
// posted slots are then read in ONE round trip by all lanes (the host filled
// them before publishing their numbers), and applied one by one from LDS
// (assign: last occurrence by an LDS hash of the largest index; accumulate:
// the first occurrence sums in index order).  Add requests need no release: only this
// workgroup touches the parameters while it runs (the host stops it before any
// other work on the shard, and its end is a release), and it reads its own
// stores through its own L2.  A Get's reply goes to page-locked host memory,
// released at system scope before done_seq.  The loop ends on `stop` or after
// idle_ticks without a request, so the kernel always drains.
// Workgroup barrier for LDS only: the wave's LDS operations complete, then
// s_barrier.  __syncthreads emits the same two instructions here, but it is
// also a workgroup-scope release/acquire for global memory, so the compiler
// keeps global accesses on their side of it; this one only orders LDS.
// (Neither waits for outstanding global stores: on gfx950 outside
// thread-group-split mode a CU's vector memory operations reach L2 in order,
// so workgroup-scope ordering needs no vmcnt wait — checked in the ISA.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <typename VT, int MODE>
__global__ __launch_bounds__(kInlineMax) void k_serve(SrvRing* ring, DenseView d, Ovf o,
                                                      void* reply, uint32_t start,
                                                      unsigned long long idle_ticks, uint32_t gen) {
  using BT = typename std::conditional<sizeof(VT) == 8, unsigned long long, uint32_t>::type;
  __shared__ __attribute__((aligned(16))) uint32_t s_keys[kInlineGetMax];
  __shared__ __attribute__((aligned(16))) unsigned long long s_vals[kInlineMax];
  constexpr int kSrvHash = 2 * kInlineMax;  // assign dedup slots (load <= 1/2)
  __shared__ uint32_t h_key[MODE == 0 ? kSrvHash + 1 : 1], h_idx[MODE == 0 ? kSrvHash + 1 : 1];
  __shared__ uint32_t h_sent;
  __shared__ uint32_t s_cmd, s_avail;
  constexpr int kSrvBatch = 4;  // requests read per round trip
  const int tid = threadIdx.x;
  uint32_t next = start + 1;
  unsigned long long t_idle = wall_clock64();
  // tell the host this launch is running (a launch queued behind other work on
  // its hardware queue has not started: the host's wait for it is bounded)
  if (tid == 0) __hip_atomic_store(&ring->started, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    if (tid == 0) {
      // {req_seq, stop} in one 8-byte load: one PCIe round trip per poll
      const unsigned long long* rs = reinterpret_cast<const unsigned long long*>(&ring->req_seq);
      uint32_t cmd = 0, avail = 0;
      for (;;) {
        const unsigned long long w = sys_load(rs);
        const int32_t ahead = (int32_t)((uint32_t)w - next);
        if (ahead >= 0) {
          avail = ahead + 1 < kSrvBatch ? (uint32_t)ahead + 1u : (uint32_t)kSrvBatch;
          // pairs with the host's release store of req_seq: the slots it
          // published are read after this (system scope; the other lanes after
          // the barrier below)
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
          break;
        }
        if ((uint32_t)(w >> 32) != 0u || wall_clock64() - t_idle > idle_ticks) {
          cmd = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_cmd = cmd;
      s_avail = avail;
    }
    __syncthreads();
    if (s_cmd) break;
    const int m = (int)s_avail;
    // one round trip for up to kSrvBatch posted requests: every lane loads each
    // request's header and its share of the LARGEST payload at once (the unused
    // part is ignored), with 16-byte volatile loads (system-coherent,
    // cache-bypassing): lanes 0..127 take the keys, lanes 128..255 the values
    static_assert(kInlineGetMax * 4 == 128 * 16 && kInlineMax * 8 == 128 * 16, "one 16-byte piece per lane");
    u32x4 hdrs[kSrvBatch], pieces[kSrvBatch];
#pragma unroll
    for (int b = 0; b < kSrvBatch; ++b) {
      if (b < m) {
        const SrvSlot* sl = &ring->slot[(next + (uint32_t)b) % kSrvSlots];
        hdrs[b] = *reinterpret_cast<const volatile u32x4*>(&sl->kind);
        pieces[b] = tid < 128 ? *reinterpret_cast<const volatile u32x4*>(&sl->keys[4 * tid])
                              : *reinterpret_cast<const volatile u32x4*>(&sl->vals[2 * (tid - 128)]);
      }
    }
    uint32_t last_kind = 0;
#pragma unroll
    for (int b = 0; b < kSrvBatch; ++b) {
    if (b >= m) break;  // uniform
    const u32x4 hdr = hdrs[b], piece = pieces[b];
    const uint32_t kind = hdr[0];
    last_kind = kind;
    const int n = (int)(hdr[1] < (uint32_t)kInlineGetMax ? hdr[1] : (uint32_t)kInlineGetMax);
    const unsigned long long h1 = hdr[2];
    if (MODE == 0) {  // the assign dedup table, cleared for this request
      for (int i = tid; i <= kSrvHash; i += kInlineMax) {
        h_key[i] = kEmpty32;
        h_idx[i] = 0u;
      }
      if (tid == 0) h_sent = 0u;
    }
    if (tid < 128) {
      u32x4 k4v = piece;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * tid + e >= n) k4v[e] = 0u;  // zero past n: the walks read whole 16-byte groups
      reinterpret_cast<u32x4*>(s_keys)[tid] = k4v;
    } else {
      reinterpret_cast<u32x4*>(s_vals)[tid - 128] = piece;
    }
    // a full barrier: besides the staged message, the previous request's
    // parameter stores are ordered before this one's (workgroup-scope
    // release/acquire), so a later request's store to the same key lands last
    __syncthreads();
    const u32x4* k4 = reinterpret_cast<const u32x4*>(s_keys);
    const int ng = (n + 3) >> 2;
    if (kind == kSrvAdd) {
      uint32_t win_slot = 0;
      if (tid < n) {
        const uint32_t k = s_keys[tid];
        if (MODE == 0) {
          // last occurrence: the largest index per key in an LDS hash (two LDS
          // atomics per key; the O(n) walk of every lane over the message cost
          // ~6 us at 256 keys)
          uint32_t k1[1] = {k}, s1[1];
          (void)lds_insert<1, kSrvHash>(h_key, &h_sent, k1, 1u, s1);
          atomicMax(&h_idx[s1[0]], (uint32_t)tid + 1u);
          win_slot = s1[0];
        }
      }
      __syncthreads();
      // room for the request's new out-of-range keys (a workgroup step)
      const int n_out = __syncthreads_count(tid < n && (uint64_t)(uint32_t)(s_keys[tid] - d.key_begin) >= d.range);
      OvfTab ot{};
      if (n_out) {
        ovf_reserve<sizeof(VT)>(o, (uint64_t)n_out);
        ot = ovf_tab(o);
      }
      if (tid < n) {
        const uint32_t k = s_keys[tid];
        const uint32_t off = k - d.key_begin;
        if (MODE == 0) {
          if (h_idx[win_slot] == (uint32_t)tid + 1u) {  // the last occurrence stores
            const BT v = (BT)s_vals[tid];
            if ((uint64_t)off < d.range) {
              reinterpret_cast<BT*>(d.param)[off] = v;
            } else {
              const long long slot = ovf_insert(o, ot, k);
              if (slot >= 0) reinterpret_cast<BT*>(ot.vals)[slot] = v;
            }
          }
        } else {
          bool earlier = false;
          for (int g = 0; g < ng; ++g) {
            const u32x4 q = k4[g];
#pragma unroll
            for (int e = 0; e < 4; ++e) earlier |= (4 * g + e < tid) & (q[e] == k);
          }
          if (!earlier) {  // the first occurrence sums them all, in index order
            VT* p = nullptr;
            if ((uint64_t)off < d.range) {
              p = reinterpret_cast<VT*>(d.param) + off;
            } else {
              const long long slot = ovf_insert(o, ot, k);
              if (slot >= 0) p = reinterpret_cast<VT*>(ot.vals) + slot;
            }
            if (p) {
              VT acc = *p;
              for (int j = tid; j < n; ++j)
                if (s_keys[j] == k) acc = add_wrap<VT>(acc, from_bits<VT>(s_vals[j]));
              *p = acc;
            }
          }
        }
      }
      lds_barrier();  // the staged message is read before the next one is staged
    } else {
      __syncthreads();  // the parameter stores of earlier Adds are ordered before these loads
      constexpr int PER = kInlineGetMax / kInlineMax;
      const uint32_t roff = (uint32_t)h1;
      BT v[PER];
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int i = tid + kInlineMax * q;
        v[q] = i < n ? load_one<BT, true>(d, o, s_keys[i]) : BT(0);
      }
      BT* out = static_cast<BT*>(reply) + roff;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int i = tid + kInlineMax * q;
        if (i < n) out[i] = v[q];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the reply before done_seq
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    // a Get publishes its number (covering the Adds before it); Adds are
    // published once per batch, below: a store to host memory per request cost
    // its PCIe write acknowledgement at the next barrier
    if (kind != kSrvAdd && tid == 0)
      __hip_atomic_store(&ring->done_seq, next + (uint32_t)b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }  // request b
    if (tid == 0 && last_kind == kSrvAdd)
      __hip_atomic_store(&ring->done_seq, next + (uint32_t)m - 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    next += (uint32_t)m;
    t_idle = wall_clock64();
  }
  if (tid == 0) __hip_atomic_store(&ring->alive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

// ------------------------------------------------------- launch wrappers

template <typename VT, bool VEC>
static void gather_dispatch(int unroll, bool nt, uint32_t nwg, const GroupArgs& ga,
                            const DenseView& d, const Ovf& o, hipStream_t st) {
  // (K1 held to 6 or 4 workgroups per CU by an LDS reservation, as K2g is to
  // 3: no gain anywhere, profiles/r04_probes/k1_occupancy/)
  if (unroll == 8) {
    if (nt)
      k_gather<VT, VEC, 8, true><<<nwg, kBlock, 0, st>>>(ga, d, o);
    else
      k_gather<VT, VEC, 8, false><<<nwg, kBlock, 0, st>>>(ga, d, o);
  } else {
    if (nt)
      k_gather<VT, VEC, 4, true><<<nwg, kBlock, 0, st>>>(ga, d, o);
    else
      k_gather<VT, VEC, 4, false><<<nwg, kBlock, 0, st>>>(ga, d, o);
  }
}

hipError_t launch_gather(int vb, bool vec, int unroll, bool nt, const GroupArgs& ga,
                         uint32_t nwg, const DenseView& d, const Ovf& o, hipStream_t st) {
  if (nwg == 0) return hipSuccess;
  if (vb == 4) {
    if (vec)
      gather_dispatch<uint32_t, true>(unroll, nt, nwg, ga, d, o, st);
    else
      gather_dispatch<uint32_t, false>(unroll, nt, nwg, ga, d, o, st);
  } else {
    if (vec)
      gather_dispatch<unsigned long long, true>(unroll, nt, nwg, ga, d, o, st);
    else
      gather_dispatch<unsigned long long, false>(unroll, nt, nwg, ga, d, o, st);
  }
  return hipGetLastError();
}

template <typename VT, bool VEC>
static void gather_replay_dispatch(int unroll, bool nt, uint32_t nwg, const GroupArgs& ga, const DenseView& d,
                                   const Ovf& o, const ReplayGroup& rg, const uint32_t* cond, uint32_t epoch,
                                   uint32_t* tab, hipStream_t st) {
  if (unroll == 8) {
    if (nt)
      k_gather_r<VT, VEC, 8, true><<<nwg, kBlock, 0, st>>>(ga, d, o, rg, cond, epoch, tab);
    else
      k_gather_r<VT, VEC, 8, false><<<nwg, kBlock, 0, st>>>(ga, d, o, rg, cond, epoch, tab);
  } else {
    if (nt)
      k_gather_r<VT, VEC, 4, true><<<nwg, kBlock, 0, st>>>(ga, d, o, rg, cond, epoch, tab);
    else
      k_gather_r<VT, VEC, 4, false><<<nwg, kBlock, 0, st>>>(ga, d, o, rg, cond, epoch, tab);
  }
}

hipError_t launch_gather_replay(int vb, bool vec, int unroll, bool nt, const GroupArgs& ga, uint32_t nwg,
                                const DenseView& d, const Ovf& o, const ReplayGroup& rg,
                                const uint32_t* cond, uint32_t epoch, uint32_t* tab, hipStream_t st) {
  if (nwg == 0) return hipErrorInvalidValue;  // the replay must run: the caller launches K4r instead
  if (vb == 4) {
    if (vec)
      gather_replay_dispatch<uint32_t, true>(unroll, nt, nwg, ga, d, o, rg, cond, epoch, tab, st);
    else
      gather_replay_dispatch<uint32_t, false>(unroll, nt, nwg, ga, d, o, rg, cond, epoch, tab, st);
  } else {
    if (vec)
      gather_replay_dispatch<unsigned long long, true>(unroll, nt, nwg, ga, d, o, rg, cond, epoch, tab, st);
    else
      gather_replay_dispatch<unsigned long long, false>(unroll, nt, nwg, ga, d, o, rg, cond, epoch, tab, st);
  }
  return hipGetLastError();
}

hipError_t launch_assign_sorted(int vb, bool vec, const uint32_t* keys, const void* vals,
                                uint64_t n, const DenseView& d, uint32_t* flag, uint32_t epoch,
                                hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint32_t nwg = (uint32_t)((n + kSortedChunk - 1) / kSortedChunk);
  if (vb == 4) {
    auto v = reinterpret_cast<const uint32_t*>(vals);
    if (vec)
      k_assign_sorted<uint32_t, true><<<nwg, kBlock, 0, st>>>(keys, v, n, d, flag, epoch);
    else
      k_assign_sorted<uint32_t, false><<<nwg, kBlock, 0, st>>>(keys, v, n, d, flag, epoch);
  } else {
    auto v = reinterpret_cast<const unsigned long long*>(vals);
    if (vec)
      k_assign_sorted<unsigned long long, true><<<nwg, kBlock, 0, st>>>(keys, v, n, d, flag, epoch);
    else
      k_assign_sorted<unsigned long long, false><<<nwg, kBlock, 0, st>>>(keys, v, n, d, flag, epoch);
  }
  return hipGetLastError();
}

// Workgroups of the 4-byte K2g per CU: at most 3, held there by a dynamic LDS
// reservation the kernel never touches (static 1.5 KiB + 48 KiB: 3 fit the
// CU's 160 KiB).  Its registers allow 4; 3 per CU measured faster on the
// headline (K2g 108.5 against 109.8 us), equal on the cold form and a rank's
// share; 2 per CU lost 3 % cold (profiles/r04_probes/k2g_occupancy/; A/B builds
// set PSKV_K2G_LDS_CAP).
#ifndef PSKV_K2G_LDS_CAP
#define PSKV_K2G_LDS_CAP (48u << 10)
#endif
constexpr uint32_t kK2gLdsCap = PSKV_K2G_LDS_CAP;

template <typename VT, bool VEC, bool NTP>
static void group_dispatch2(int unroll, bool nt, bool early, uint32_t grid, const GroupArgs& ga,
                            const DenseView& d, uint32_t shift, uint64_t ntiles, uint32_t* flag,
                            uint32_t epoch, hipStream_t st) {
  const uint32_t cap = sizeof(VT) == 4 && VEC && unroll == 8 ? kK2gLdsCap : 0u;
  if constexpr (sizeof(VT) == 4 && VEC) {
    if (early && unroll == 8 && nt) {  // early mode: the default unroll and streams only
      k_assign_group<VT, VEC, 8, true, NTP, true><<<grid, kBlock, cap, st>>>(ga, d, shift, ntiles, flag, epoch);
      return;
    }
  }
  if (unroll == 8) {
    if (nt)
      k_assign_group<VT, VEC, 8, true, NTP><<<grid, kBlock, cap, st>>>(ga, d, shift, ntiles, flag, epoch);
    else
      k_assign_group<VT, VEC, 8, false, NTP><<<grid, kBlock, cap, st>>>(ga, d, shift, ntiles, flag, epoch);
  } else {
    if (nt)
      k_assign_group<VT, VEC, 4, true, NTP><<<grid, kBlock, 0, st>>>(ga, d, shift, ntiles, flag, epoch);
    else
      k_assign_group<VT, VEC, 4, false, NTP><<<grid, kBlock, 0, st>>>(ga, d, shift, ntiles, flag, epoch);
  }
}

template <typename VT, bool VEC>
static void group_dispatch(int unroll, bool nt, bool ntp, bool early, uint32_t grid, const GroupArgs& ga,
                           const DenseView& d, uint32_t shift, uint64_t ntiles, uint32_t* flag,
                           uint32_t epoch, hipStream_t st) {
  if (ntp)
    group_dispatch2<VT, VEC, true>(unroll, nt, early, grid, ga, d, shift, ntiles, flag, epoch, st);
  else
    group_dispatch2<VT, VEC, false>(unroll, nt, early, grid, ga, d, shift, ntiles, flag, epoch, st);
}

hipError_t launch_assign_group(int vb, bool vec, int unroll, bool nt, bool ntp, bool early,
                               const GroupArgs& ga,
                               const DenseView& d, uint32_t tile_shift, uint64_t ntiles,
                               uint32_t grid, uint32_t* flag, uint32_t epoch, hipStream_t st) {
  if (grid == 0) return hipSuccess;
  if (vb == 4) {
    if (vec)
      group_dispatch<uint32_t, true>(unroll, nt, ntp, early, grid, ga, d, tile_shift, ntiles, flag, epoch, st);
    else
      group_dispatch<uint32_t, false>(unroll, nt, ntp, early, grid, ga, d, tile_shift, ntiles, flag, epoch, st);
  } else {
    if (vec)
      group_dispatch<unsigned long long, true>(unroll, nt, ntp, early, grid, ga, d, tile_shift, ntiles, flag,
                                               epoch, st);
    else
      group_dispatch<unsigned long long, false>(unroll, nt, ntp, early, grid, ga, d, tile_shift, ntiles, flag,
                                                epoch, st);
  }
  return hipGetLastError();
}

// Grid of a general-path launch: a conditional (repair) launch usually exits at
// once, so it gets few workgroups; otherwise enough to fill 256 CUs several
// times over, each looping over 2048-key chunks.
static uint32_t general_grid(uint32_t nwg, const uint32_t* cond) {
  const uint32_t cap = cond ? 256u : 4096u;
  return nwg < cap ? nwg : cap;
}

hipError_t launch_general_mark(int dtype, int mode, const GroupArgs& ga, uint32_t nwg,
                               const DenseView& d, uint32_t* oor, unsigned long long* owner,
                               const uint32_t* cond, uint32_t epoch, hipStream_t st) {
  if (nwg == 0) return hipSuccess;
  nwg = general_grid(nwg, cond);
  if (mode == 0) {
    // assign: value bits are never read here; the AT parameter only sizes unused LDS
    k_general_mark<uint32_t, 0><<<nwg, kBlock, 0, st>>>(ga, d, oor, owner, cond, epoch);
  } else if (dtype == 0) {
    k_general_mark<int, 1><<<nwg, kBlock, 0, st>>>(ga, d, oor, owner, cond, epoch);
  } else if (dtype == 1) {
    k_general_mark<float, 1><<<nwg, kBlock, 0, st>>>(ga, d, oor, owner, cond, epoch);
  } else {
    k_general_mark<double, 1><<<nwg, kBlock, 0, st>>>(ga, d, oor, owner, cond, epoch);
  }
  return hipGetLastError();
}

hipError_t launch_general_commit(int vb, const GroupArgs& ga, uint32_t nwg, const DenseView& d,
                                 const unsigned long long* owner,
                                 const uint32_t* cond, uint32_t epoch, hipStream_t st) {
  if (nwg == 0) return hipSuccess;
  nwg = general_grid(nwg, cond);
  if (vb == 4)
    k_general_commit<uint32_t><<<nwg, kBlock, 0, st>>>(ga, d, owner, cond, epoch);
  else
    k_general_commit<unsigned long long><<<nwg, kBlock, 0, st>>>(ga, d, owner, cond, epoch);
  return hipGetLastError();
}

template <bool OOR_ONLY>
static void replay_dispatch(int dtype, int mode, const GroupArgs& ga, const DenseView& d, const Ovf& o,
                            const uint32_t* cond, uint32_t epoch, hipStream_t st) {
  if (mode == 0) {
    // assign moves value bits only: int32 and float share the 4-byte form
    if (dtype == 2)
      k_replay<unsigned long long, 0, OOR_ONLY><<<1, kReplayBlock, 0, st>>>(ga, d, o, cond, epoch);
    else
      k_replay<uint32_t, 0, OOR_ONLY><<<1, kReplayBlock, 0, st>>>(ga, d, o, cond, epoch);
  } else if (dtype == 0) {
    k_replay<int, 1, OOR_ONLY><<<1, kReplayBlock, 0, st>>>(ga, d, o, cond, epoch);
  } else if (dtype == 1) {
    k_replay<float, 1, OOR_ONLY><<<1, kReplayBlock, 0, st>>>(ga, d, o, cond, epoch);
  } else {
    k_replay<double, 1, OOR_ONLY><<<1, kReplayBlock, 0, st>>>(ga, d, o, cond, epoch);
  }
}

hipError_t launch_replay(int dtype, int mode, const GroupArgs& ga, const DenseView& d, const Ovf& o,
                         const uint32_t* cond, uint32_t epoch, hipStream_t st, bool oor_only) {
  if (ga.nb == 0) return hipSuccess;
  if (oor_only)
    replay_dispatch<true>(dtype, mode, ga, d, o, cond, epoch, st);
  else
    replay_dispatch<false>(dtype, mode, ga, d, o, cond, epoch, st);
  return hipGetLastError();
}

hipError_t launch_ovf_rehash(int vb, const Ovf& o, uint64_t from_cap, const OvfTab& to, hipStream_t st) {
  uint64_t g = (from_cap + kBlock - 1) / kBlock;
  if (g > 4096) g = 4096;
  if (g != 0) {
    if (vb == 4)
      k_ovf_rehash<uint32_t><<<(uint32_t)g, kBlock, 0, st>>>(o, from_cap, to);
    else
      k_ovf_rehash<unsigned long long><<<(uint32_t)g, kBlock, 0, st>>>(o, from_cap, to);
  }
  k_ovf_set<<<1, 64, 0, st>>>(o, to);
  return hipGetLastError();
}

template <typename AT, typename BT, int MODE>
static hipError_t rb_launch(const GroupArgs& ga, uint32_t nsc, const DenseView& d, const Ovf& o,
                            const RbMap& bm, int apply_log2, int bin_block, uint16_t* loff,
                            void* tmp, hipStream_t st) {
  const uint32_t nbk = bm.nbd + 1;
  auto* t = reinterpret_cast<RbEnt<sizeof(BT)>*>(tmp);
  // persistent grid: one 1024-thread workgroup per CU (~139 KiB LDS), or two
  // 512-thread ones (~74 KiB each)
  const uint32_t wgs = bin_block == 512 ? 512u : 256u;
  const uint32_t gb = nsc < wgs ? nsc : wgs;
  if (bin_block == 512)
    k_rb_bin<AT, BT, MODE, 512><<<gb, 512, 0, st>>>(ga, d, bm, nbk, loff, nsc, t);
  else
    k_rb_bin<AT, BT, MODE, 1024><<<gb, 1024, 0, st>>>(ga, d, bm, nbk, loff, nsc, t);
  const uint32_t sc = rb_sc<BT>(bin_block);
  if (apply_log2 == 13)  // 2^13 slots: two workgroups per CU
    k_rb_resolve<AT, BT, MODE, 13><<<512, kApplyBlock, 0, st>>>(d, o, bm, nbk, loff, nsc, sc, t);
  else
    k_rb_resolve<AT, BT, MODE, 14><<<256, kApplyBlock, 0, st>>>(d, o, bm, nbk, loff, nsc, sc, t);
  return hipGetLastError();
}

hipError_t launch_rb_add(int dtype, int mode, const GroupArgs& ga, uint32_t nsc,
                         const DenseView& d, const Ovf& o, const RbMap& bm,
                         int apply_log2, int bin_block, uint16_t* loff, void* tmp,
                         hipStream_t st) {
  if (nsc == 0) return hipSuccess;
  if (bm.nbd + 1 > (uint32_t)kRbMaxBuckets || nsc > kRbMaxSc || bm.nbd == 0 ||
      (bin_block != 512 && bin_block != 1024))
    return hipErrorInvalidValue;
#define PSKV_RB(AT, BT, M) rb_launch<AT, BT, M>(ga, nsc, d, o, bm, apply_log2, bin_block, loff, tmp, st)
  if (mode == 0) {
    if (dtype == 0) return PSKV_RB(int, uint32_t, 0);
    if (dtype == 1) return PSKV_RB(float, uint32_t, 0);
    return PSKV_RB(double, unsigned long long, 0);
  }
  if (dtype == 0) return PSKV_RB(int, uint32_t, 1);
  if (dtype == 1) return PSKV_RB(float, uint32_t, 1);
  return PSKV_RB(double, unsigned long long, 1);
#undef PSKV_RB
}

hipError_t launch_dense_check(const GroupArgs& ga, uint32_t nchunks, const DenseView& d,
                              uint32_t* flag, uint32_t epoch, hipStream_t st) {
  if (nchunks == 0) return hipSuccess;
  k_dense_check<8><<<nchunks, kBlock, 0, st>>>(ga, d, flag, epoch);
  return hipGetLastError();
}

hipError_t launch_acc_dense(int dtype, const GroupArgs& ga, uint32_t grid, const DenseView& d,
                            const uint32_t* flag, uint32_t epoch, hipStream_t st) {
  if (grid == 0) return hipSuccess;
  if (dtype == 0)
    k_acc_dense<int, 8, true><<<grid, kBlock, 0, st>>>(ga, d, flag, epoch);
  else if (dtype == 1)
    k_acc_dense<float, 8, true><<<grid, kBlock, 0, st>>>(ga, d, flag, epoch);
  else
    k_acc_dense<double, 8, true><<<grid, kBlock, 0, st>>>(ga, d, flag, epoch);
  return hipGetLastError();
}

// Super-chunk size (keys) and entry size of the K5 path for a value size.
uint32_t rb_superchunk(int vb, int bin_block) {
  return vb == 8 ? rb_sc<unsigned long long>(bin_block) : rb_sc<uint32_t>(bin_block);
}
size_t rb_entry_bytes(int vb) { return vb == 8 ? sizeof(RbEnt<8>) : sizeof(RbEnt<4>); }


hipError_t launch_inline_add(int dtype, int mode, const InlineAdd& a, const DenseView& d,
                             const Ovf& o, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  if (mode == 0) {
    // assign moves value bits only: int32 and float share the 4-byte form
    if (dtype == 2)
      k_inline_add<double, 0><<<1, kInlineMax, 0, st>>>(a, d, o);
    else
      k_inline_add<float, 0><<<1, kInlineMax, 0, st>>>(a, d, o);
  } else if (dtype == 0) {
    k_inline_add<int, 1><<<1, kInlineMax, 0, st>>>(a, d, o);
  } else if (dtype == 1) {
    k_inline_add<float, 1><<<1, kInlineMax, 0, st>>>(a, d, o);
  } else {
    k_inline_add<double, 1><<<1, kInlineMax, 0, st>>>(a, d, o);
  }
  return hipGetLastError();
}

hipError_t launch_serve(int dtype, int mode, SrvRing* ring, const DenseView& d, const Ovf& o,
                        void* reply, uint32_t start_seq, unsigned long long idle_ticks,
                        uint32_t gen, hipStream_t st) {
  if (mode == 0) {
    if (dtype == 2)
      k_serve<double, 0><<<1, kInlineMax, 0, st>>>(ring, d, o, reply, start_seq, idle_ticks, gen);
    else
      k_serve<float, 0><<<1, kInlineMax, 0, st>>>(ring, d, o, reply, start_seq, idle_ticks, gen);
  } else if (dtype == 0) {
    k_serve<int, 1><<<1, kInlineMax, 0, st>>>(ring, d, o, reply, start_seq, idle_ticks, gen);
  } else if (dtype == 1) {
    k_serve<float, 1><<<1, kInlineMax, 0, st>>>(ring, d, o, reply, start_seq, idle_ticks, gen);
  } else {
    k_serve<double, 1><<<1, kInlineMax, 0, st>>>(ring, d, o, reply, start_seq, idle_ticks, gen);
  }
  return hipGetLastError();
}

hipError_t launch_inline_get(int vb, const InlineGet& a, const DenseView& d, const Ovf& o,
                             void* out, unsigned int* done, unsigned int seq, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  if (vb == 8)
    k_inline_get<unsigned long long><<<1, 64, 0, st>>>(a, d, o, static_cast<unsigned long long*>(out),
                                                       done, seq);
  else
    k_inline_get<uint32_t><<<1, 64, 0, st>>>(a, d, o, static_cast<uint32_t*>(out), done, seq);
  return hipGetLastError();
}

}  // namespace pskv

#ifdef PSKV_STEP_STAMPS
// Diagnostic build only: copy out (then clear) the K2g / K1 step stamps,
// 2 x 8192 x 4 u64 ([K2g|K1][workgroup][phase], 0 = not reached).
extern "C" int pskv_diag_step_stamps(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pskv::g_step_stamps), sizeof(pskv::g_step_stamps)) != hipSuccess)
    return -2;
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(pskv::g_step_stamps)) != hipSuccess) return -2;
  return hipMemset(p, 0, sizeof(pskv::g_step_stamps)) == hipSuccess ? 0 : -2;
}
#endif

#ifdef PSKV_K5_STAMPS
// Diagnostic build only: copy out (then clear) the K5 phase stamps, 2 x 512 x 8
// x 8 u64 ([K5a|K5b][workgroup][pass][phase], 0 = not reached).
extern "C" int pskv_diag_k5_stamps(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pskv::g_k5_stamps), sizeof(pskv::g_k5_stamps)) != hipSuccess) return -2;
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(pskv::g_k5_stamps)) != hipSuccess) return -2;
  return hipMemset(p, 0, sizeof(pskv::g_k5_stamps)) == hipSuccess ? 0 : -2;
}
#endif
