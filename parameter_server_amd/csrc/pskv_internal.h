// pskv_internal.h — device-side data layout and kernel launch wrappers shared by
// pskv_kernels.hip (device code) and pskv_shard.cpp (the C ABI host logic).
//
// HBM layout of one shard (DESIGN.md "Data layout in HBM"):
//   dense[range]        value array, one slot per owned key, zero-initialised
//   owner[range]        u64 last-writer stamps (epoch<<32 | group index), general path only
//   ctl                 OvfCtl: the overflow table's current arrays, {occupied
//                       slots, sticky error bits}, the growth mailbox
//   keys[cap]           u64 overflow hash keys, EMPTY = ~0
//   vals[cap]           overflow values
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace pskv {

constexpr int kMaxBatches = 64;     // batches per grouped launch (kernarg budget)
constexpr int kBlock = 256;         // threads per workgroup (4 waves)
constexpr int kGatherVec = 4;       // keys per lane per step (16 B loads)
constexpr int kSortedUnroll = 2;
inline int stream_chunk(int unroll) { return kBlock * 4 * unroll; }  // keys per gather / dense chunk
constexpr int kSortedChunk = kBlock * 4 * kSortedUnroll;          // 2048 keys / workgroup
constexpr int kGeneralChunk = 2048;  // keys per workgroup in the dedup path
constexpr int kGeneralSlots = 4096;  // LDS hash slots (load factor <= 1/2)
constexpr int kRbMaxBuckets = 2064;  // key buckets incl. the out-of-range bucket (>= 2049)
// K5a workgroup (option RB_BIN_BLOCK): 1024 threads, one per CU.  Two
// 512-thread workgroups per CU on 4 Ki-key super-chunks bin at the same rate
// (K5a 55.0 against 56.0 us per 8 M cfg-3 Zipf keys): K5a is bound by the CU's
// LDS and issue throughput, not by its barrier phases.  With one run per
// resolve thread the 512 form needs two launch pieces per 8 M keys, and the
// whole Add is slower (assign 2 x (32.0 + 58.7) against 56.8 + 86.4 us;
// profiles/r03_probes/ztrace_k5_split_*.txt).
constexpr int kRbBinBlockDefault = 1024;
constexpr uint32_t kRbMaxSc = 1024;  // K5 super-chunks per launch (one run per resolve thread)
constexpr int kInlineMax = 256;      // keys of an inline (kernarg-carried) Add
constexpr int kInlineGetMax = 512;   // keys of an inline Get
constexpr int kInlineMaxChunks = 16;   // inline launches per call at most (reply buffer size)
constexpr unsigned long long kEmpty64 = ~0ull;
constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;

// Error bits in ovf.stat[1].
constexpr uint32_t kErrOverflowFull = 1u;

struct DevBatch {
  const uint32_t* keys;
  const void* vals;  // input values for Add, output for Get
  uint64_t n;
};

// Passed by value as the kernel argument (fits the 4 KiB kernarg segment).
struct GroupArgs {
  int nb;
  uint32_t wg_prefix[kMaxBatches + 1];  // first workgroup of each batch
  DevBatch b[kMaxBatches];
};
static_assert(sizeof(GroupArgs) <= 1800, "a group plus the other arguments fit the 4 KiB kernarg segment");

// The batches of an Add group whose conditional replay rides on the next Get's
// K1 launch (K1r, pskv_add_get_grouped): a second group in the same kernarg
// segment, without the workgroup prefix the replay does not read.
struct ReplayGroup {
  int nb;
  DevBatch b[kMaxBatches];
};
static_assert(sizeof(GroupArgs) + sizeof(ReplayGroup) <= 3500,
              "K1r's two groups plus its other arguments fit the 4 KiB kernarg segment");

// K8: a whole small message inside the kernel arguments (<= 4 KiB kernarg).
struct InlineAdd {
  uint32_t n;
  uint32_t keys[kInlineMax];
  unsigned long long vals[kInlineMax];  // value bits (4-byte values in the low word)
};
struct InlineGet {
  uint32_t n;
  uint32_t keys[kInlineGetMax];
};
static_assert(sizeof(InlineAdd) + 128 <= 4096 && sizeof(InlineGet) + 128 <= 4096,
              "inline messages must fit the kernarg segment with the other arguments");

// K9: the small-message server (PSKV_SERVE=1): one resident workgroup polls a
// ring of requests in coherent page-locked host memory and applies them in
// ring order, so a small Add or Get costs no kernel launch.
constexpr int kSrvSlots = 64;
constexpr uint32_t kSrvAdd = 1, kSrvGet = 2;
struct SrvSlot {  // the kernel reads {kind, n} and {reply_off, pad} as 8-byte words
  uint32_t kind;       // kSrvAdd / kSrvGet
  uint32_t n;          // keys: <= kInlineMax (Add) / kInlineGetMax (Get)
  uint32_t reply_off;  // Get: first reply element
  uint32_t pad;
  uint32_t keys[kInlineGetMax];
  unsigned long long vals[kInlineMax];  // value bits (4-byte values in the low word)
};
struct SrvRing {  // the kernel polls {req_seq, stop} as one 8-byte word
  uint32_t req_seq;    // host: number of the last request posted
  uint32_t stop;       // host: 1 = leave the loop
  uint32_t pad0[30];
  uint32_t done_seq;   // device: number of the last request applied
  uint32_t alive;      // host sets 1 at launch; device: 0 once the kernel has left its loop
  uint32_t started;    // device: the launch generation now running (stored on entry)
  uint32_t pad1[29];
  SrvSlot slot[kSrvSlots];
};
static_assert(sizeof(SrvSlot) % 8 == 0 && offsetof(SrvRing, slot) % 8 == 0, "8-byte words in the ring");

struct DenseView {
  void* param;
  uint32_t key_begin;
  uint64_t range;  // number of owned keys, <= 2^32
};

// The overflow table: open addressing over u64 key slots (EMPTY = ~0) for the
// keys outside the dense range (the last range server's fall-through keys,
// range_partition_manager.hpp:26-27).  Its arrays can be replaced while work
// is queued -- a single-workgroup inserter grows the table on the device
// (ovf_reserve, DESIGN.md §4 "Overflow growth") -- so kernels reach them
// through the shard's control block, whose address is fixed for the shard's
// life, and load them when they meet an out-of-range key.
struct OvfTab {
  unsigned long long* keys;
  void* vals;
  uint64_t mask;  // capacity - 1 (capacity is a power of two)
};
// Growth requests of device-side inserters: one per shard, in coherent
// page-locked host memory; the library's grow service (pskv_shard.cpp) answers
// each with fresh arrays of the asked capacity, the requesting workgroup fills
// and rehashes them itself and switches the control block over.
struct OvfMbox {
  uint32_t req_seq;   // device: number of the last request
  uint32_t pad0;
  uint64_t req_cap;   // device: slots asked for (a power of two)
  uint64_t wait_ticks;  // host: bound of a request's wait (device wall-clock ticks)
  uint64_t pad1[5];
  uint32_t resp_seq;  // host: number of the last request answered
  uint32_t resp_ok;   // host: 1 = resp_tab holds uninitialised arrays of req_cap slots
  OvfTab resp_tab;
  uint64_t pad2[4];
};
static_assert(sizeof(OvfMbox) == 128, "device and host words on separate 64-byte lines");
struct OvfCtl {  // device memory
  OvfTab t;          // the current table
  uint32_t stat[2];  // {occupied slots, sticky error bits}
  OvfMbox* mbox;     // growth requests
};
struct Ovf {  // kernel argument
  OvfCtl* c;
};

// Launch wrappers (pskv_kernels.hip).  vb = value bytes (4 or 8), vec = all
// pointers 16-byte aligned so 16 B vector accesses are legal.
// unroll: 4 or 8 groups of 4 keys per lane (chunk = 256*4*unroll keys);
// nt: non-temporal loads/stores of the streamed push/pull buffers.
hipError_t launch_gather(int vb, bool vec, int unroll, bool nt, const GroupArgs& ga,
                         uint32_t nwg, const DenseView& d, const Ovf& o, hipStream_t st);
hipError_t launch_assign_sorted(int vb, bool vec, const uint32_t* keys, const void* vals,
                                uint64_t n, const DenseView& d, uint32_t* flag, uint32_t epoch,
                                hipStream_t st);
// Grouped sorted Add.  `ga` must be built with stream_chunk(unroll) elements per chunk
// (used by the dense-window mode); the tile mode ignores the chunking.
// ntp: non-temporal parameter stores in the dense-window mode
hipError_t launch_assign_group(int vb, bool vec, int unroll, bool nt, bool ntp, bool early,
                               const GroupArgs& ga,
                               const DenseView& d, uint32_t tile_shift, uint64_t ntiles,
                               uint32_t grid, uint32_t* flag, uint32_t epoch, hipStream_t st);
// K4a: in-range keys only; an out-of-range key tags *oor with `epoch` for the
// oor_only replay behind K4.
hipError_t launch_general_mark(int dtype, int mode, const GroupArgs& ga, uint32_t nwg,
                               const DenseView& d, uint32_t* oor, unsigned long long* owner,
                               const uint32_t* cond, uint32_t epoch, hipStream_t st);
hipError_t launch_general_commit(int vb, const GroupArgs& ga, uint32_t nwg, const DenseView& d,
                                 const unsigned long long* owner,
                                 const uint32_t* cond, uint32_t epoch, hipStream_t st);
// Host growth of the table (pskv_sync keeps its load <= 1/2): rehash the
// current table (from_cap slots) into `to` (keys EMPTY, values 0), then
// switch the control block over.
hipError_t launch_ovf_rehash(int vb, const Ovf& o, uint64_t from_cap, const OvfTab& to, hipStream_t st);
// K4r: conditional replay of a group in call order by ONE workgroup (runs only
// when *cond == epoch: a sorted-path hint was broken); assign or accumulate.
// oor_only: only the group's out-of-range keys (behind K4, which leaves them
// to this single workgroup, the only kind of inserter that can grow the table).
hipError_t launch_replay(int dtype, int mode, const GroupArgs& ga, const DenseView& d, const Ovf& o,
                         const uint32_t* cond, uint32_t epoch, hipStream_t st, bool oor_only = false);
// K1r: K1 with an assign group's conditional replay folded in (the launch K4r
// would cost): when *cond == epoch, workgroup 0 replays `rg` and then gathers
// every chunk of `ga` itself while the other workgroups leave; otherwise K1.
// tab: kK1rTableWords words of device scratch (the replay's table, K1r has no LDS).
constexpr uint32_t kK1rTableWords = 4100;
hipError_t launch_gather_replay(int vb, bool vec, int unroll, bool nt, const GroupArgs& ga, uint32_t nwg,
                                const DenseView& d, const Ovf& o, const ReplayGroup& rg,
                                const uint32_t* cond, uint32_t epoch, uint32_t* tab, hipStream_t st);
// K5 key buckets: windows of 2^wbits keys of the owned range, window w in
// bucket w % nbd (1 <= nbd < 2^12, windows < 2^21: wbits >= 11 or a range
// below 2^32); magic = ceil(2^32 / nbd); span = keys per bucket at most
// (ceil(windows / nbd) << wbits), the extent of a bucket's local index.
struct RbMap {
  uint32_t wbits;
  uint32_t nbd;
  uint32_t magic;
  uint32_t span;
  int32_t nlog;  // log2(nbd) when nbd is a power of two (then magic is unused), else -1
};

// K5 radix-bucket general Add (2 launches: K5a bin, K5b resolve).  `ga`
// chunked by rb_superchunk(vb, bin_block) keys (nsc <= kRbMaxSc super-chunks);
// nbd dense buckets (RbMap) plus one out-of-range bucket.  bin_block: K5a's
// workgroup size, 1024 (one per CU) or 512 (two per CU, half the super-chunk).
// Scratch: loff: nsc * (nbd+2) u16 (each super-chunk's bucket starts); tmp:
// nsc * rb_superchunk(vb, bin_block) entries (rb_entry_bytes(vb) each).
// apply_log2: log2 of the resolve workgroup's LDS table slots (13: 64 KiB, two
// workgroups per CU, ~7 Ki entries per bucket in one pass; 14: 128 KiB, ~14 Ki).
hipError_t launch_rb_add(int dtype, int mode, const GroupArgs& ga, uint32_t nsc,
                         const DenseView& d, const Ovf& o, const RbMap& bm,
                         int apply_log2, int bin_block, uint16_t* loff, void* tmp,
                         hipStream_t st);
uint32_t rb_superchunk(int vb, int bin_block);
constexpr size_t kRbTmpPad = 16;  // bytes past the last entry K5b may read (paired loads)
// K8: one small host message carried in the kernarg segment (one workgroup).
// Get writes its n values to `out` (page-locked host memory or device memory);
// with `done` non-null it then stores `seq` there (system-scope release) for a
// host that polls instead of waiting on the stream.
hipError_t launch_inline_add(int dtype, int mode, const InlineAdd& a, const DenseView& d,
                             const Ovf& o, hipStream_t st);
hipError_t launch_inline_get(int vb, const InlineGet& a, const DenseView& d, const Ovf& o,
                             void* out, unsigned int* done, unsigned int seq, hipStream_t st);
// K9: start the request server on `st` (one workgroup; requests start_seq+1..
// are applied as they are posted).  It stores `gen` in ring->started on entry,
// leaves its loop when ring->stop is set or after idle_ticks wall-clock ticks
// without a request, and then clears alive.
hipError_t launch_serve(int dtype, int mode, SrvRing* ring, const DenseView& d, const Ovf& o,
                        void* reply, uint32_t start_seq, unsigned long long idle_ticks,
                        uint32_t gen, hipStream_t st);
size_t rb_entry_bytes(int vb);
// K6: tag `flag` with `epoch` unless every batch is a dense in-range window
// (chunk = kBlock * 4 * 8 keys per workgroup).
hipError_t launch_dense_check(const GroupArgs& ga, uint32_t nchunks, const DenseView& d,
                              uint32_t* flag, uint32_t epoch, hipStream_t st);
// K7: accumulate dense windows (skips when flag == epoch); chunk as K6.
hipError_t launch_acc_dense(int dtype, const GroupArgs& ga, uint32_t grid, const DenseView& d,
                            const uint32_t* flag, uint32_t epoch, hipStream_t st);

}  // namespace pskv
