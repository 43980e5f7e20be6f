/*
 * pskv.h — C ABI of the MI355X-native parameter-shard store (Add/Get hot path).
 *
 * This is the drop-in boundary that replaces the arithmetic of the reference's
 * storage plugins:
 *
 *   reference interface                                   replaced by
 *   ---------------------------------------------------  -----------------------------
 *   AbstractStorage::SubAdd  server/abstract_storage.hpp:35-36   pskv_add / pskv_add_grouped
 *   AbstractStorage::SubGet  server/abstract_storage.hpp:39      pskv_get / pskv_get_grouped
 *   AbstractStorage::FinishIter server/abstract_storage.hpp:41   pskv_sync (the reference's is a no-op)
 *   MapStorage<Val>()        server/map_storage.hpp:15           pskv_shard_create(..., PSKV_ASSIGN)
 *   VectorStorage<Val>()     server/vector_storage.hpp:14        pskv_shard_create(..., PSKV_ASSIGN)
 *   ~AbstractStorage (missing in the reference) pskv_shard_destroy
 *   RangePartitionManager::Slice base/range_partition_manager.hpp:19-46,48-77  pskv_range_slice
 *   ConsistentHashingPartitionManager::JumpConsistentHash
 *                     base/consistent_hashing_partition_manager.hpp:81-89       pskv_jump_hash
 *   zmq receive buffer of a data frame, Mailbox::Recv comm/mailbox.cpp:246-257,
 *   and SubGet's reply allocation server/map_storage.hpp:30     pskv_host_alloc / pskv_host_free
 *
 * Semantics (PSKV_ASSIGN, the reference semantics; map_storage.hpp:22-23,
 * vector_storage.hpp:21-43): a shard is a last-write-wins key/value store with
 * uint32 keys (base/magic.hpp:7).  Within one call the LAST occurrence of a key
 * wins (index order), across calls the later call wins (call order on the
 * shard's stream).  A key that was never written reads as 0
 * (map_storage.hpp:33-37; zero-filled SArray in vector_storage.hpp:33).  Values
 * are copied bit-for-bit, so parity is bit-exact for every value type.
 *
 * PSKV_ACCUMULATE is the north-star gradient-reduction mode (param[k] += v for
 * every occurrence).  It has no reference counterpart; float sums follow the
 * tolerance stated in DESIGN.md (recursive-summation bound), int32 is exact.
 *
 * Keys outside [key_begin, key_end) are legal (the reference's last range
 * server receives every out-of-range key, range_partition_manager.hpp:26-27):
 * they live in a device-side overflow hash table with the same semantics, and
 * there is no limit on how many (as the reference's std::map has none).  Every
 * out-of-range insert, from host or device inputs, is made by ONE workgroup
 * that first reserves room: when the table would pass 3/4 load it asks the
 * library's grow service (a host thread) for larger arrays and rehashes into
 * them on the device, in stream order, so device callers need no host step
 * and no sizing (round 6; DESIGN.md §4 "Overflow growth").  pskv_sync trims
 * the load back to <= 1/2.  Keys are dropped -- and the next pskv_sync returns
 * PSKV_ESTATE -- only if a growth request is not answered within
 * SYNC_TIMEOUT_MS or its allocation fails (device memory exhausted).
 *
 * Threading: one shard handle is used by one host thread at a time (the
 * reference calls a storage only from its ServerThread, server_thread.cpp:20-50);
 * distinct handles may be used concurrently.  Every call selects the shard's
 * device itself, so construction and use may happen on different threads
 * (Engine::CreateTable constructs storages on the engine thread,
 * driver/engine.hpp:100-109).
 *
 * Errors: every function returns 0 on success and a negative PSKV_E* code on
 * failure; pskv_last_error() returns this thread's message for the last
 * failure.  The C++ HipStorage adaptor (include/ps/hip_storage.hpp) turns a
 * non-zero status into an abort, keeping the reference's glog CHECK convention
 * (abstract_storage.hpp:15,20; map_storage.hpp:20).
 */
#ifndef PSKV_H_
#define PSKV_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSKV_ABI_VERSION 1

/* status codes */
#define PSKV_OK 0
#define PSKV_EINVAL (-1)   /* bad argument (null pointer, bad dtype, n mismatch ...) */
#define PSKV_EHIP (-2)     /* a HIP runtime call failed */
#define PSKV_ENOMEM (-3)   /* device or pinned allocation failed */
#define PSKV_ESTATE (-4)   /* sticky device-side error (overflow table exhausted) */

/* value types used by the reference (driver/engine.cpp:254,261; apps use double) */
enum pskv_dtype { PSKV_I32 = 0, PSKV_F32 = 1, PSKV_F64 = 2 };

/* update semantics */
enum pskv_mode {
  PSKV_ASSIGN = 0,     /* reference: last write wins (drop-in default) */
  PSKV_ACCUMULATE = 1  /* north star: scatter-accumulate (gradient reduction) */
};

/* call flags */
#define PSKV_HOST 0x0        /* keys/vals/out are host memory (the zmq buffers of comm/mailbox.cpp) */
#define PSKV_DEVICE 0x1      /* keys/vals/out are device memory on the shard's device */
#define PSKV_SORTED_HINT 0x2 /* caller believes keys are non-decreasing: take the sorted path.
                                The kernel verifies the claim and repairs the result on the
                                device if it was wrong, so a wrong hint costs time, never
                                correctness.  What it costs: the group is replayed in call
                                order by ONE workgroup (K4r), ~1 GB/s of keys and values --
                                64 M 4-byte keys take ~0.3 s -- on top of the sorted pass. */
#define PSKV_HOST_FRAME 0x4  /* host keys/vals/out that lie in pskv_host_alloc frames are
                                BORROWED until pskv_host_free: the call reads and writes them
                                in place (no staging copy) and an Add returns once its work
                                is queued, without waiting for it.  The caller must not
                                modify such a frame before freeing it; pskv_host_free holds
                                it back from reuse until every queued call that reads it has
                                run.  Host pointers outside frames ignore the flag. */
/* Any other flag bit, or PSKV_HOST_FRAME together with PSKV_DEVICE, is
 * rejected with PSKV_EINVAL (the call does nothing). */

typedef struct pskv_shard pskv_shard;

/* One push or pull batch of a grouped call.  For an Add `vals` is read
 * (n values), for a Get `vals` is the output (n values). */
typedef struct pskv_batch {
  const uint32_t* keys;
  void* vals;
  uint64_t n;
} pskv_batch;

typedef struct pskv_info {
  int device;
  int dtype;
  int mode;
  int value_bytes;
  uint32_t key_begin;
  uint64_t key_end;          /* exclusive, may be 2^32 */
  uint64_t dense_bytes;      /* HBM held by the dense parameter array */
  uint64_t overflow_capacity;/* slots of the overflow hash table */
  uint64_t overflow_count;   /* keys stored in the overflow table (as of the last sync) */
  uint64_t n_add_calls;
  uint64_t n_get_calls;
  uint64_t n_sorted_launches;   /* sorted-path kernel launches */
  uint64_t n_general_launches;  /* general (dedup) path launches, repairs included */
} pskv_info;

/* Kernel ids for pskv_kernel_time. */
enum pskv_kernel {
  PSKV_K_GATHER = 0,        /* K1: gather (Get) */
  PSKV_K_ASSIGN_SORTED = 1, /* K2: sorted last-wins scatter (single batch) */
  PSKV_K_ASSIGN_TILES = 2,  /* K2g: grouped sorted scatter, key-tile owner */
  PSKV_K_GENERAL_MARK = 3,  /* K4a: chunk dedup + stamps / accumulate */
  PSKV_K_GENERAL_COMMIT = 4,/* K4b: winner write */
  PSKV_K_RADIX = 5,         /* K5a-d: radix-bucket general Add (timed as one operation) */
  PSKV_K_DENSE_CHECK = 6,   /* K6: accumulate, prove the batches dense windows */
  PSKV_K_ACC_DENSE = 7,     /* K7: accumulate dense windows, one RMW per key */
  PSKV_K_INLINE_ADD = 8,    /* K8: small host Add carried in the kernel arguments */
  PSKV_K_INLINE_GET = 9,    /* K8: small host Get, reply written to page-locked memory */
  PSKV_K_REPLAY = 10,       /* K4r: conditional replay behind a verifying sorted-path group */
  PSKV_K_COUNT = 11
};

/* Create a shard owning keys [key_begin, key_end) on `device`.  The dense
 * array ((key_end-key_begin) values) is allocated in HBM and zero-filled.
 * key_end may be 2^32 (the whole key space: 17.2 GB for float). */
int pskv_shard_create(int device, uint32_t key_begin, uint64_t key_end, int dtype, int mode,
                      pskv_shard** out);
/* As pskv_shard_create, with an explicit overflow-table capacity (slots, rounded
 * up to a power of two; 0 = default). */
int pskv_shard_create_ex(int device, uint32_t key_begin, uint64_t key_end, int dtype, int mode,
                         uint64_t overflow_slots, pskv_shard** out);
int pskv_shard_destroy(pskv_shard* s);

/* Push: apply n (key, value) pairs.  Asynchronous on the shard's stream for
 * PSKV_DEVICE inputs (the caller keeps them alive until the stream passes the
 * call); host inputs are staged before return and may be reused immediately.
 * A host Add of at most 256 keys in all (grouped: summed over its batches)
 * travels inside the kernel arguments and returns once the launch is
 * enqueued; a host Get of at most 1024 keys likewise, 512 keys per launch,
 * its reply written by the kernels into page-locked memory (PSKV_INLINE=0
 * disables; PSKV_SERVE=1 sends them to a resident request-server kernel
 * instead).  Larger pageable host Adds below 32 MiB are copied
 * into pinned staging and return once the copy is queued for DMA. */
int pskv_add(pskv_shard* s, const uint32_t* keys, const void* vals, uint64_t n, int flags);
/* Pull: out[i] = value of keys[i] (0 if never written).  Synchronous for host
 * `out` (PSKV_HOST), stream-ordered for device `out` (PSKV_DEVICE). */
int pskv_get(pskv_shard* s, const uint32_t* keys, uint64_t n, void* out, int flags);

/* Grouped forms: nb batches in one call, semantically identical to nb
 * consecutive pskv_add / pskv_get calls in array order, executed in a small,
 * fixed number of kernel launches. */
int pskv_add_grouped(pskv_shard* s, const pskv_batch* batches, uint64_t nb, int flags);
int pskv_get_grouped(pskv_shard* s, const pskv_batch* batches, uint64_t nb, int flags);
/* pskv_add_grouped(adds) then pskv_get_grouped(gets) in one call (flags as
 * for both; PSKV_SORTED_HINT applies to the Adds): the BSP model's flush of
 * its deferred Adds followed by the Gets that flush releases
 * (server/consistency/bsp_model.cpp:14-31), or one worker round's push then
 * pull.  Identical results to the two calls.  Device batches, assign mode,
 * 4-byte values: the Add's conditional replay (K4r) rides on the Get's first
 * K1 launch (K1r), one launch fewer than the two calls (option FOLD_REPLAY).
 * (A single fused launch for the pair was built and measured slower than the
 * two launches) */
int pskv_add_get_grouped(pskv_shard* s, const pskv_batch* adds, uint64_t na, const pskv_batch* gets,
                         uint64_t ng, int flags);

/* Wait for the shard's stream, adopt the overflow table as the kernels left
 * it (freeing arrays a device-side growth replaced; trimming its load to
 * <= 1/2), report sticky device errors.  Every host wait of the library (this one, a host
 * Get's, the staging and scratch waits, destroy's) is bounded by the option
 * SYNC_TIMEOUT_MS (default 120000; 0 = unbounded): work that does not complete
 * in time fails the call with PSKV_ESTATE, and pskv_last_error() names the
 * stream or event waited for, the device and the last kernel the shard
 * queued.  Nothing is cancelled or restarted: after a call fails with
 * PSKV_ESTATE its queued work may still read the call's host inputs (a direct
 * DMA from the caller's buffers) or write its host outputs (a Get's values
 * into page-locked memory), so the caller keeps those buffers alive and
 * unmodified until a later pskv_sync succeeds.  (The library's own staging is
 * held back the same way: the next call waits for it, bounded.) */
int pskv_sync(pskv_shard* s);
/* Zero every value (dense array and overflow table). */
int pskv_clear(pskv_shard* s);

/* Run the shard's work on an external hipStream_t (NULL = the shard's own
 * stream, a blocking stream that orders against the legacy default stream). */
int pskv_set_stream(pskv_shard* s, void* hip_stream);
void* pskv_get_stream(pskv_shard* s);
/* Device pointer of the dense array (for zero-copy inspection by tests/benches). */
void* pskv_dense_ptr(pskv_shard* s);
int pskv_shard_info(pskv_shard* s, pskv_info* info);

/* Tuning and path options of one shard, by name (DESIGN.md §5 lists them and
 * what each selects): GENERAL (0 = K4 stamps, 1 = auto, 2 = K5 always),
 * UNROLL, GET_UNROLL (K1's keys per lane: 0 = by launch size, 4, 8), NT, NTP,
 * EARLY (K2g early loads: 0 never, 1 always, 2 auto),
 * PAGEABLE_DMA, DMA_MIN_BYTES, DMA_MIN_BYTES_GET,
 * DMA_MIN_BYTES_PINNED, ZC_MAX_BYTES, FRAME_ZC_MAX_BYTES, INLINE,
 * INLINE_ADD_CHUNKS, INLINE_GET_CHUNKS, ISPIN, SERVE, SERVE_IDLE_US,
 * TILE_SHIFT, TILE_GRID, RB_WBITS, RB_NBD, RB_TB, RB_APPLY_LOG2, RB_BIN_BLOCK,
 * SYNC_TIMEOUT_MS (the bound of every host wait, pskv_sync), FOLD_REPLAY
 * (pskv_add_get_grouped: the Add's conditional replay rides on the Get's
 * first K1 launch, K1r, instead of a K4r launch of its own; 1 = on).
 * Every option changes speed only, never results.  Some apply only together
 * with others (a value is accepted and echoed either way):
 *   EARLY = 1     K2g with UNROLL 8 and NT 1 (otherwise the default loads)
 *   SERVE = 1     only while the device's hardware queues hold the server
 *                 (DESIGN.md §8); INLINE_*_CHUNKS and ISPIN only on the K8 path
 *   RB_* options  only on the K5 path (unhinted Adds)
 * pskv_set_option returns PSKV_EINVAL for an unknown name or a value out of
 * range (the shard is unchanged).  The environment variable PSKV_<NAME> sets a
 * creation default; an invalid value there is reported on stderr and ignored
 * (the built-in default stays; creation does not fail); so is a retired
 * option's variable (RB_INSERT, GET_DEDUP, GET_NTP, FUSE). */
int pskv_set_option(pskv_shard* s, const char* name, int64_t value);
int pskv_get_option(pskv_shard* s, const char* name, int64_t* value);

/* Per-kernel timing with HIP events on the launch stream (off by default).
 * pskv_set_timing brackets every kernel; pskv_set_timing_mask only the kernels
 * whose bit (1 << pskv_kernel) is set. */
int pskv_set_timing(pskv_shard* s, int enable);
int pskv_set_timing_mask(pskv_shard* s, uint32_t kernel_mask);
int pskv_kernel_time(pskv_shard* s, int kernel, uint64_t* launches, double* total_ms,
                     uint64_t* elements);
int pskv_reset_timing(pskv_shard* s);

/* Mirror of RangePartitionManager::Slice (base/range_partition_manager.hpp:19-46):
 * walk `keys` once; a key goes to the current range if it lies in it or the
 * current range is the last one, otherwise the range pointer advances.  Emits
 * contiguous slices (range index, first key index, length) in order; at most
 * nranges slices.  Returns the number of slices, or a negative error. */
int pskv_range_slice(const uint64_t* range_begin, const uint64_t* range_end, int nranges,
                     const uint32_t* keys, uint64_t n, int32_t* slice_range,
                     uint64_t* slice_start, uint64_t* slice_len);

/* Bucket of every key under jump consistent hashing over `nbuckets` servers:
 * the bucket function of ConsistentHashingPartitionManager::Slice, the
 * reference Engine's default partitioner
 * (base/consistent_hashing_partition_manager.hpp:18-42,81-89;
 * driver/engine.hpp:143-150).  out_bucket[i] in [0, nbuckets); the slice of key
 * i goes to server_thread_ids[out_bucket[i]].  Host memory, any n. */
int pskv_jump_hash(const uint32_t* keys, uint64_t n, int32_t nbuckets, int32_t* out_bucket);

/* Page-locked host frames for message payloads (the mailbox
 * receives data frames, comm/mailbox.cpp:211-261, into memory the GPU reads
 * directly).  Pooled by power-of-two size class, so steady traffic allocates
 * nothing; thread-safe; usable by every device.  *out is 4 KiB-aligned.  A
 * freed frame whose queued reads (PSKV_HOST_FRAME Adds) have not run yet is
 * held back until they have.  Free frames beyond PSKV_FRAME_CACHE_BYTES
 * (default 1 GiB) are returned to the system. */
int pskv_host_alloc(uint64_t bytes, void** out);
int pskv_host_free(void* p);
/* Bytes held by live frames, by cached free frames, and by freed frames still
 * awaiting their queued reads. */
int pskv_host_pool_stats(uint64_t* live_bytes, uint64_t* cached_bytes, uint64_t* held_bytes);
/* Return every cached free frame to the system (waits for held ones first). */
int pskv_host_pool_trim(void);

const char* pskv_last_error(void);
int pskv_abi_version(void);
/* Number of HIP devices visible (0 when there is no GPU). */
int pskv_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* PSKV_H_ */
