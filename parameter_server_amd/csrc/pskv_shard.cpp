// pskv_shard.cpp — host side of the C ABI declared in include/pskv.h.
//
// One pskv_shard is what the reference calls a storage: the object
// Engine::CreateTable builds per server thread (driver/engine.hpp:100-109) and
// the consistency model drives through AbstractStorage::Add/Get
// (server/abstract_storage.hpp:14-32).  Here it owns a dense HBM array for its
// key range, an overflow hash table for every other key, a stream, and
// pinned/device staging for host (zmq-buffer) inputs.
//
// Call flow of an assign-mode Add:
//   small host messages → K8 (kernarg-carried) or the K9 request server.
//   host inputs   → copy into pinned staging (or DMA / read in place when
//                   page-locked) while checking "sorted and in range" on the
//                   CPU → K2 / K2g if verified, else K5.
//   device inputs → PSKV_SORTED_HINT: K2 (one batch) or K2g (group), each
//                   verifying on device, followed by the one-workgroup K4r
//                   replay, which exits at once unless the verification
//                   tagged the call.  No hint: K5 (key buckets).
// Accumulate-mode Add: K6 density proof + K7 for dense windows, else K5.
// Get: K1 (one launch per group of <= 64 batches), K8 for small messages.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pskv.h"
#include "pskv_frames.h"
#include "pskv_internal.h"
#include "pskv_queues.h"

using namespace pskv;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define PSKV_HIP(call)                                                                     \
  do {                                                                                     \
    hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(PSKV_EHIP, std::string(#call) + ": " + hipGetErrorString(e_));           \
  } while (0)

int value_bytes(int dtype) {
  switch (dtype) {
    case PSKV_I32:
    case PSKV_F32:
      return 4;
    case PSKV_F64:
      return 8;
    default:
      return 0;
  }
}

uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

constexpr uint64_t kDefaultOverflowSlots = 1ull << 16;
// see tune_dma_min_bytes: measured per call (tools/micro/small_latency.cpp,
// f64): Add via the pinned copy 6-7 us up to 4 Ki keys, 338 us at 1 Mi keys
// (direct DMA 48 / 366 us), DMA ahead from ~4 Mi keys; Get via the copy 18 us
// up to 2 Ki keys (DMA 26), DMA ahead from 4 Ki keys
constexpr size_t kDefaultDmaMinBytes = 32ull << 20;
constexpr size_t kDefaultDmaMinBytesGet = 32ull << 10;

struct TimedLaunch {
  int kernel;
  hipEvent_t a, b;
  uint64_t elems;
};

// ---------------------------------------------------------------- host pool
// A small persistent pool for the host side of the path: copying zmq-buffer
// inputs into pinned staging (with the sorted/in-range check) and pinned
// outputs back to the caller.  One parallel section at a time; the caller
// thread works too.  Size: PSKV_HOST_THREADS (default min(8, cores)).
class HostPool {
 public:
  static HostPool& get() {
    static HostPool p;
    return p;
  }
  size_t size() const { return workers_.size() + 1; }
  // Runs fn(0..n-1), blocking until all are done.
  void run(size_t n, const std::function<void(size_t)>& fn) {
    if (n == 0) return;
    if (n == 1 || workers_.empty()) {
      for (size_t i = 0; i < n; ++i) fn(i);
      return;
    }
    std::lock_guard<std::mutex> section(section_);
    Job job(&fn, n);
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = &job;
      ++gen_;
    }
    cv_.notify_all();
    work(job);
    std::unique_lock<std::mutex> lk(m_);
    // a worker that joined late may still hold the job: wait for it to let go
    done_.wait(lk, [&] { return job.left == 0 && job.refs == 0; });
    job_ = nullptr;
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  // One parallel section; lives on the stack of run() until every index is
  // done and no worker references it.
  struct Job {
    Job(const std::function<void(size_t)>* f, size_t count) : fn(f), n(count), left(count) {}
    const std::function<void(size_t)>* fn;
    size_t n;
    std::atomic<size_t> next{0};
    size_t left;  // guarded by m_
    int refs = 0;  // workers inside work(*this), guarded by m_
  };
  HostPool() {
    unsigned hw = std::thread::hardware_concurrency();
    unsigned n = std::min(8u, hw ? hw : 1u);
    if (const char* e = std::getenv("PSKV_HOST_THREADS")) n = (unsigned)std::max(1, std::atoi(e));
    for (unsigned i = 1; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  void work(Job& j) {
    for (;;) {
      const size_t i = j.next.fetch_add(1);
      if (i >= j.n) return;
      (*j.fn)(i);
      std::lock_guard<std::mutex> lk(m_);
      if (--j.left == 0) done_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      Job* j;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        j = job_;
        if (!j) continue;
        ++j->refs;
      }
      work(*j);
      std::lock_guard<std::mutex> lk(m_);
      if (--j->refs == 0 && j->left == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex section_, m_;
  std::condition_variable cv_, done_;
  Job* job_ = nullptr;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

constexpr size_t kPieceBytes = 1 << 20;   // one pool task
constexpr size_t kCheckPieceBytes = 256 << 10;  // one pool task of a check without copy
constexpr size_t kWindowBytes = 8 << 20;  // one H2D / D2H DMA while the next window is copied
constexpr size_t kInlineCopyBytes = 256 << 10;  // smaller windows are copied by the calling thread

// Run fn over pieces [b, e) of `pieces`: on the calling thread when they are
// small (waking the pool costs more than copying a few hundred KiB), on the
// pool otherwise.
template <typename PieceT, typename Fn>
void run_pieces(std::vector<PieceT>& pieces, size_t b, size_t e, const Fn& fn) {
  size_t bytes = 0;
  for (size_t i = b; i < e; ++i) bytes += pieces[i].bytes;
  if (bytes < kInlineCopyBytes) {
    for (size_t i = b; i < e; ++i) fn(pieces[i]);
    return;
  }
  HostPool::get().run(e - b, [&](size_t t) { fn(pieces[b + t]); });
}

}  // namespace

struct pskv_shard {
  int device = 0;
  int dtype = PSKV_F32;
  int mode = PSKV_ASSIGN;
  int vb = 4;
  uint32_t key_begin = 0;
  uint64_t range = 0;
  void* dense = nullptr;
  unsigned long long* owner = nullptr;  // u64 stamps, allocated on first general-path use
  // overflow table: the control block (device memory; the kernels' argument),
  // its growth mailbox (coherent page-locked), the table as of the last
  // adoption (read_overflow_stat) and every table array set allocated for this
  // shard, by the host or by the grow service (freed once superseded and the
  // stream is idle).  tab_m guards `tables` (the service appends to it).
  Ovf ovf{};
  OvfMbox* mbox = nullptr;
  OvfTab cur{};
  std::mutex tab_m;
  std::vector<OvfTab> tables;
  uint32_t mbox_served = 0;  // grow service: number of the last request answered
  uint64_t ocap = 0;
  uint64_t ocount_known = 0;
  // device words: [0] verification tag
  uint32_t* flag = nullptr;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  uint32_t epoch = 0;
  // staging for host inputs/outputs
  void* hstage = nullptr;
  size_t hstage_bytes = 0;
  hipEvent_t hstage_free = nullptr;
  bool hstage_pending = false;
  hipEvent_t h2d_done = nullptr;  // pinned caller buffers: their DMA has completed
  void* dstage = nullptr;
  size_t dstage_bytes = 0;
  std::vector<hipEvent_t> win_events;  // per-window D2H completion (pull to host)
  // page-locked Get: values DMA'd out on their own stream, window by window
  hipStream_t out_stream = nullptr;
  std::vector<hipEvent_t> out_events;
  // timing
  uint32_t timing_mask = 0;  // bit k: bracket kernel k with events
  std::vector<TimedLaunch> pending;
  std::vector<hipEvent_t> event_pool;
  uint64_t t_launches[PSKV_K_COUNT] = {};
  double t_ms[PSKV_K_COUNT] = {};
  uint64_t t_elems[PSKV_K_COUNT] = {};
  // stats
  uint64_t n_add = 0, n_get = 0, n_sorted = 0, n_general = 0;
  // K5 radix-bucket scratch (grown on demand)
  uint16_t* rb_loff = nullptr;
  size_t rb_loff_bytes = 0;
  void* rb_ent = nullptr;
  size_t rb_ent_bytes = 0;
  int general_path = 1;  // PSKV_GENERAL: stamps = 0 (K4 always), auto = 1, radix = 2 (K5 always)
  // tuning knobs (environment, read at creation): PSKV_TILE_SHIFT, PSKV_TILE_GRID
  uint32_t tune_tile_shift = 0;
  // grid cap of K2g / K7: one workgroup per dense-mode chunk up to 512 Mi keys
  // (round 4: at 4096 a workgroup took two of cfg 2's 8192 chunks, K2g 112.7
  // against 111.4 us; 2048 / 1024: 116.5 / 117.3; profiles/r04_probes/k2g_tune/)
  uint32_t tune_tile_grid = 65536;
  int tune_unroll = 8;   // PSKV_UNROLL: 4 or 8 (8: measured +5 % on the dense Add)
  int tune_get_unroll = 0;  // PSKV_GET_UNROLL: K1's keys per lane, 4 or 8, 0 = by launch size
  bool tune_nt = true;   // PSKV_NT: non-temporal streams (measured +12-15 % on K1 / K2g)
  // PSKV_NTP: non-temporal parameter stores in the dense Add (K2g).  On
  // since round 4: cached stores leave the Add's parameter lines dirty in the
  // Infinity Cache, and the next Get pays their write-back; the headline step
  // 5.74-5.86 -> 6.11-6.22 TB/s, its Get (K1) 114-116 -> 91 us
  // (profiles/r04_probes/ntp_ab/)
  bool tune_ntp = true;
  int tune_early = 2;    // PSKV_EARLY: K2g early loads (0 never, 1 always, 2 when the group's keys cover < 1/4 of the range)
  // PSKV_PAGEABLE_DMA: DMA pageable host buffers directly (the runtime moves
  // them at the PCIe rate, measured 55 GB/s) instead of copying them into
  // pinned staging first; 0 selects the staging path.  cfg-2-shaped Add of
  // 8 x 1M keys: 1.43 ms against 1.75 ms staged, Get 1.37 against 1.44 ms.
  bool tune_pageable_dma = true;
  // PSKV_DMA_MIN_BYTES / PSKV_DMA_MIN_BYTES_GET: pageable host Adds / Gets of
  // at least this many bytes (keys + values) take the direct DMA; smaller ones
  // the pinned staging copy
  size_t tune_dma_min_bytes = kDefaultDmaMinBytes;
  size_t tune_dma_min_bytes_get = kDefaultDmaMinBytesGet;
  // PSKV_DMA_MIN_BYTES_PINNED: page-locked host Adds of at least this many
  // bytes are DMA'd straight from the caller's buffers (and wait for it);
  // smaller ones take the pinned staging copy, which returns before its DMA.
  // Measured (tools/micro/small_latency.cpp, f64): 16 Ki keys 9 us copied
  // against 29 us DMA'd, 256 Ki keys 95 against 90
  size_t tune_dma_min_bytes_pinned = 2ull << 20;
  // PSKV_ZC_MAX_BYTES: pageable host Gets of at most this many bytes (keys +
  // values) past the inline size go zero-copy through pinned staging (0: off).
  // Measured (tools/micro/small_latency.cpp, f64): 4 Ki keys 18 us, 16 Ki 23,
  // 64 Ki 43 against 28 / 40 / 63 us by DMA; DMA ahead at 256 Ki (101 vs 152)
  size_t tune_zc_max_bytes = 1ull << 20;
  // PSKV_FRAME_ZC_MAX_BYTES: PSKV_HOST_FRAME Adds and page-locked Gets of at
  // most this many bytes (keys + values) run the kernels on the host buffers
  // in place; larger ones DMA
  size_t tune_frame_zc_max_bytes = 8ull << 20;
  uint32_t tune_rb_tb = 0; // PSKV_RB_TB: K5 bucket bits (0 = by element count)
  uint32_t tune_rb_wbits = 0; // PSKV_RB_WBITS: K5 window bits (0 = 11; >= bucket shift: contiguous buckets)
  uint32_t tune_rb_nbd = 0;   // PSKV_RB_NBD: K5 dense bucket count (0 = by the rule; tuning)
  // PSKV_INLINE: host calls of <= kInlineMax (Add) / kInlineGetMax (Get) keys in
  // all travel inside the kernel arguments (K8); 0 sends them through staging
  bool tune_inline = true;
  // PSKV_INLINE_ADD_CHUNKS / PSKV_INLINE_GET_CHUNKS: K8 launches per call at
  // most (1..kInlineMaxChunks).  Measured (tools/micro/small_latency.cpp): an
  // Add launch costs ~3-7 us of enqueue, and the pinned staging copy returns
  // in 6-8 us up to 4 Ki keys (its DMA and kernels run on), so one launch;
  // a Get launch beyond the first ~4-12 us against ~20 us through the copy
  // (1024 keys: 16 us), so up to 2 (1024 keys).
  int tune_inline_add_chunks = 1;
  int tune_inline_get_chunks = 2;
  void* ireply = nullptr;  // page-locked reply buffer of inline Gets (kInlineGetMax values)
  bool tune_ispin = true;  // PSKV_ISPIN: poll the reply's sequence word instead of a stream wait
  unsigned int ireply_seq = 0;
  int tune_rb_apply_log2 = 0; // PSKV_RB_APPLY_LOG2: 13 or 14 (0 = by bucket size)
  int tune_rb_bin_block = kRbBinBlockDefault;  // PSKV_RB_BIN_BLOCK: K5a workgroup, 512 or 1024
  // K9 request server (PSKV_SERVE=1): the inline-size messages go to a ring in
  // coherent page-locked memory that one resident workgroup polls
  // (PSKV_SERVE_IDLE_US: it leaves after this long without a request)
  bool tune_serve = false;
  uint32_t tune_serve_idle_us = 20000;
  SrvRing* srv = nullptr;
  uint32_t srv_gen = 0;  // launch generation (the kernel stores it in ring->started on entry)
  hipStream_t srv_stream = nullptr;
  hipEvent_t srv_dep = nullptr;  // the shard's stream up to the server's launch
  bool srv_running = false;
  uint32_t srv_posted = 0;
  unsigned long long srv_idle_ticks = 0;
  bool counted = false;  // in g_queues (pskv_queues.h)
  bool add_chunks_set = false;  // INLINE_ADD_CHUNKS chosen explicitly
  int wall_khz = 0;             // device wall-clock rate (the server's idle timer)
  // bounded host waits (round 5): PSKV_SYNC_TIMEOUT_MS, 0 = unbounded.  A wait
  // for the shard's stream, an event or the request server that outlasts it
  // fails the call with PSKV_ESTATE naming what it waited for; nothing is
  // restarted.  The longest legitimate wait measured (one 2^32 + 2^20-key
  // unhinted batch) is ~1.4 s.
  uint32_t tune_sync_timeout_ms = 120000;
  int last_kernel = -1;           // the last kernel this shard queued (PSKV_K_*), for the report
  uint64_t launches = 0;          // kernels this shard queued
  hipEvent_t sync_ev = nullptr;   // marks the end of a stream for a bounded wait
  uint32_t* stat_host = nullptr;  // page-locked read-back of the overflow table's {count, err}
  // pskv_add_get_grouped (round 5): the Add's last conditional replay (K4r)
  // held back and folded into the Get's first K1 launch (K1r) instead of a
  // launch of its own; option FOLD_REPLAY
  int tune_fold_replay = 1;
  bool defer_replay = false;  // inside add_get: replay() holds the group instead of launching
  bool pend_replay = false;   // a held replay: pend_rg, pend_epoch, pend_elems
  ReplayGroup pend_rg{};
  uint32_t pend_epoch = 0;
  uint64_t pend_elems = 0;

  DenseView dview() const { return DenseView{dense, key_begin, range}; }
};

namespace {

// K1's keys per lane (8 x 4 or 4 x 4, i.e. 8 Ki- or 4 Ki-key chunks) for a
// launch of `elems` keys.  Option GET_UNROLL: 4 or 8, or 0 = by size (round 5):
// a launch of under kGetSmallKeys keys takes 4 x 4 -- a cfg-4 rank's Get at
// N = 8 (~8 M keys) ran K1 in 17.5 against 18.4 us with the smaller chunks
// (ranks 0 and 1 emulated, twice each, profiles/r05_probes/emu_u48/), where
// the dense Add's K2g lost with them (22.0 against 21.2 us), so the two are
// chosen apart; UNROLL = 4 still forces 4 x 4 on both.
constexpr uint64_t kGetSmallKeys = 24ull << 20;
int gather_unroll(const pskv_shard* s, uint64_t elems) {
  if (s->tune_get_unroll) return s->tune_get_unroll;
  if (s->tune_unroll == 4) return 4;
  return elems < kGetSmallKeys ? 4 : 8;
}

int use_device(pskv_shard* s) {
  PSKV_HIP(hipSetDevice(s->device));
  return PSKV_OK;
}

hipEvent_t take_event(pskv_shard* s) {
  if (!s->event_pool.empty()) {
    hipEvent_t e = s->event_pool.back();
    s->event_pool.pop_back();
    return e;
  }
  // timing-only events: no system-scope release fence (an L2 writeback + invalidate
  // per record, measured at ~4 us each between the cfg-2 kernels)
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}

// Bracket one kernel launch with events when timing is on.
struct LaunchTimer {
  pskv_shard* s;
  int kernel;
  uint64_t elems;
  hipEvent_t a = nullptr, b = nullptr;
  LaunchTimer(pskv_shard* s_, int k, uint64_t e) : s(s_), kernel(k), elems(e) {
    s->last_kernel = k;
    ++s->launches;
    if (s->timing_mask & (1u << k)) {
      a = take_event(s);
      b = take_event(s);
      if (a && b) (void)hipEventRecord(a, s->stream);
    }
  }
  void done() {
    if (a && b) {
      (void)hipEventRecord(b, s->stream);
      s->pending.push_back(TimedLaunch{kernel, a, b, elems});
    }
    a = b = nullptr;
  }
};

// ------------------------------------------------------ bounded host waits
// Every host wait of the library polls a HIP event instead of blocking in
// hipStreamSynchronize / hipEventSynchronize, so that work which never
// completes -- a kernel that does not finish, a stream held behind another
// process's queue -- fails the call after PSKV_SYNC_TIMEOUT_MS with
// PSKV_ESTATE and a message naming the stream or event, the device and the
// last kernel the shard queued, instead of hanging its caller (VERDICT r4
// item 1).  Nothing is restarted or cancelled: the work stays queued.  Polls
// spin for the first millisecond (a small call's latency), then yield, then
// sleep 100 us between polls after 50 ms.
const char* const kKernelNames[PSKV_K_COUNT] = {
    "k_gather (K1 Get)",          "k_assign_sorted (K2)",          "k_assign_group (K2g)",
    "k_general_mark (K4a)",       "k_general_commit (K4b)",        "k_rb_bin + k_rb_resolve (K5 Add)",
    "k_dense_check (K6)",         "k_acc_dense (K7)",              "k_inline_add (K8)",
    "k_inline_get (K8)",          "k_replay (K4r)"};

std::string wait_report(const pskv_shard* s, const char* what, const void* handle, double ms) {
  char buf[384];
  std::snprintf(buf, sizeof(buf),
                "%s (%p) on device %d not complete after %.0f ms (PSKV_SYNC_TIMEOUT_MS); last kernel this shard "
                "queued: %s (%llu launches); the work stays queued",
                what, handle, s->device, ms,
                s->last_kernel >= 0 && s->last_kernel < PSKV_K_COUNT ? kKernelNames[s->last_kernel] : "none",
                (unsigned long long)s->launches);
  return buf;
}

int wait_event(pskv_shard* s, hipEvent_t ev, const char* what, const void* handle) {
  if (!s->tune_sync_timeout_ms) {  // unbounded: the runtime's own blocking wait
    const hipError_t e = hipEventSynchronize(ev);
    return e == hipSuccess ? PSKV_OK : fail(PSKV_EHIP, std::string(what) + ": " + hipGetErrorString(e));
  }
  using Clock = std::chrono::steady_clock;
  const auto t0 = Clock::now();
  for (uint64_t it = 0;; ++it) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return PSKV_OK;
    if (e != hipErrorNotReady) return fail(PSKV_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    if ((it & 15u) != 15u) continue;
    const double ms = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    if (s->tune_sync_timeout_ms && ms > (double)s->tune_sync_timeout_ms)
      return fail(PSKV_ESTATE, wait_report(s, what, handle ? handle : ev, ms));
    if (ms > 50.0)
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    else if (ms > 1.0)
      std::this_thread::yield();
  }
}

// Wait for everything queued on `st` so far (hipStreamSynchronize, bounded).
// The marker event keeps the default system-scope release, as the stream
// synchronisation it replaces: host reads of pinned results see the writes.
int wait_stream(pskv_shard* s, hipStream_t st, const char* what) {
  if (!s->tune_sync_timeout_ms) {  // unbounded: the runtime's own blocking wait
    const hipError_t e = hipStreamSynchronize(st);
    return e == hipSuccess ? PSKV_OK : fail(PSKV_EHIP, std::string(what) + ": " + hipGetErrorString(e));
  }
  if (!s->sync_ev) PSKV_HIP(hipEventCreateWithFlags(&s->sync_ev, hipEventDisableTiming));
  PSKV_HIP(hipEventRecord(s->sync_ev, st));
  return wait_event(s, s->sync_ev, what, st);
}

int drain_timing(pskv_shard* s) {
  for (auto& t : s->pending) {
    if (int rc = wait_event(s, t.b, "timing event of the shard's stream", t.b)) return rc;
    float ms = 0.f;
    PSKV_HIP(hipEventElapsedTime(&ms, t.a, t.b));
    s->t_launches[t.kernel] += 1;
    s->t_ms[t.kernel] += ms;
    s->t_elems[t.kernel] += t.elems;
    s->event_pool.push_back(t.a);
    s->event_pool.push_back(t.b);
  }
  s->pending.clear();
  return PSKV_OK;
}

// ------------------------------------------------------- K9 request server
// Protocol (host side).  Requests are numbered 1, 2, ...; the host fills slot
// q % kSrvSlots, then publishes q in req_seq (release).  The kernel applies
// requests in order and publishes each number in done_seq after it (a Get
// after its reply is released).  The kernel runs ALONE on the shard: before
// any other work is queued on the shard's stream (srv_stop: every posted
// request applied, then `stop`, then the kernel's end, which releases its
// stores), and it starts behind everything already queued on that stream
// (srv_launch: stream wait on an event), so stream order is kept both ways.
// A kernel that left on its idle timer is restarted from done_seq (srv_wait).

// A resident server holds the hardware queue its stream maps to (the
// accounting per device, pskv_queues.h): the server engages on a device only
// while 2 * shards + 1 + extra streams fit its GPU_MAX_HW_QUEUES queues (one
// shard at the default 4) — it then holds a queue of its own, provided the
// process creates no further streams on the device (torch's default stream is
// the null stream).  Beyond that the K8 launches serve.  A launch that is
// nevertheless queued behind other work does not hang its caller: srv_wait
// bounds the wait for it to start (kSrvStartTimeoutMs) and fails the call.
DeviceQueues g_queues;

bool serve_on(const pskv_shard* s) {
  if (!s->tune_serve) return false;
  static const int queues = hw_queues_from_env(std::getenv("GPU_MAX_HW_QUEUES"));
  return g_queues.serve_fits(s->device, queues);
}

constexpr int kSrvStartTimeoutMs = 2000;

int ensure_ireply(pskv_shard* s, size_t cap) {
  if (s->ireply) return PSKV_OK;
  // the reply values, then the K8 reply's sequence word on its own line.
  // Coherent (fine-grained) memory: the kernel's stores go straight to the
  // host.  Measured alternatives (tools/micro/small_latency.cpp):
  // non-coherent pinned memory the same, a device reply + D2H copy 3 us slower.
  if (hipHostMalloc(&s->ireply, cap + 128, hipHostMallocCoherent) != hipSuccess) {
    s->ireply = nullptr;
    return fail(PSKV_ENOMEM, "inline reply buffer allocation failed");
  }
  // the sequence word the host polls (ireply_seq counts from 1): page-locked
  // memory may come back holding a former owner's bytes, so clear it
  std::memset(static_cast<char*>(s->ireply) + cap, 0, 128);
  s->ireply_seq = 0;
  return PSKV_OK;
}

int srv_launch(pskv_shard* s) {
  SrvRing* r = s->srv;
  const uint32_t start = __atomic_load_n(&r->done_seq, __ATOMIC_ACQUIRE);
  __atomic_store_n(&r->stop, 0u, __ATOMIC_RELAXED);
  __atomic_store_n(&r->alive, 1u, __ATOMIC_RELEASE);
  ++s->srv_gen;
  // SERVE_IDLE_US may change between launches (pskv_set_option)
  s->srv_idle_ticks =
      (unsigned long long)s->tune_serve_idle_us * (unsigned long long)std::max(s->wall_khz, 1) / 1000ull;
  PSKV_HIP(hipEventRecord(s->srv_dep, s->stream));
  PSKV_HIP(hipStreamWaitEvent(s->srv_stream, s->srv_dep, 0));
  PSKV_HIP(launch_serve(s->dtype, s->mode, r, s->dview(), s->ovf, s->ireply, start, s->srv_idle_ticks,
                        s->srv_gen, s->srv_stream));
  s->srv_running = true;
  return PSKV_OK;
}

// The kernel has left (or is leaving) its loop: wait for its end.
int srv_reap(pskv_shard* s) {
  s->srv_running = false;
  if (int rc = wait_stream(s, s->srv_stream, "request-server stream (K9 end)")) return rc;
  return PSKV_OK;
}

// Wait until request `seq` has been applied.
int srv_wait(pskv_shard* s, uint32_t seq) {
  SrvRing* r = s->srv;
  // The start clock runs only once the server's own dependency (everything
  // queued on the shard's stream before its launch, srv_dep) has completed: a
  // launch still waiting for that work -- e.g. a long replay of a broken sorted
  // hint -- is not stuck, however long the work takes.
  auto t_start = std::chrono::steady_clock::now();
  const auto t_entry = t_start;
  bool dep_done = false;
  for (uint32_t it = 1;; ++it) {
    if ((int32_t)(__atomic_load_n(&r->done_seq, __ATOMIC_ACQUIRE) - seq) >= 0) return PSKV_OK;
    if ((it & 255u) == 0 && __atomic_load_n(&r->alive, __ATOMIC_ACQUIRE) == 0u) {
      // it left on its idle timer as requests were being posted: restart it
      if (int rc = srv_reap(s)) return rc;
      if ((int32_t)(__atomic_load_n(&r->done_seq, __ATOMIC_ACQUIRE) - seq) >= 0) return PSKV_OK;
      if (int rc = srv_launch(s)) return rc;
      dep_done = false;
      t_start = std::chrono::steady_clock::now();
    }
    if ((it & 65535u) == 0) {  // a faulted kernel never publishes: surface the error
      const hipError_t e = hipStreamQuery(s->srv_stream);
      if (e != hipSuccess && e != hipErrorNotReady) PSKV_HIP(e);
      // the overall bound (PSKV_SYNC_TIMEOUT_MS): a dependency that never
      // completes -- a kernel that does not finish, or work held behind
      // another queue -- fails the call instead of spinning without end
      const double ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_entry).count();
      if (s->tune_sync_timeout_ms && ms > (double)s->tune_sync_timeout_ms)
        return fail(PSKV_ESTATE, wait_report(s, dep_done ? "request-server request (server launched, request not "
                                                            "applied)"
                                                          : "request-server dependency (the shard's stream before "
                                                            "the server's launch)",
                                             dep_done ? static_cast<const void*>(s->srv_stream)
                                                      : static_cast<const void*>(s->srv_dep),
                                             ms));
      if (!dep_done) {
        const hipError_t d = hipEventQuery(s->srv_dep);
        if (d != hipSuccess && d != hipErrorNotReady) PSKV_HIP(d);
        dep_done = d == hipSuccess;
        t_start = std::chrono::steady_clock::now();  // re-armed while the dependency runs
        continue;
      }
      // the dependency is done and the launch has still not started: it is
      // queued behind other work on its hardware queue -- fail the call rather
      // than wait without bound
      if (__atomic_load_n(&r->started, __ATOMIC_ACQUIRE) != s->srv_gen &&
          std::chrono::steady_clock::now() - t_start > std::chrono::milliseconds(kSrvStartTimeoutMs))
        return fail(PSKV_ESTATE,
                    "request server did not start within 2 s: its hardware queue is held by other work "
                    "(more streams on the device than GPU_MAX_HW_QUEUES); run without PSKV_SERVE");
    }
  }
}

// Every posted request applied and the kernel ended (before any other work).
int srv_stop(pskv_shard* s) {
  if (!s->srv_running) return PSKV_OK;
  if (int rc = srv_wait(s, s->srv_posted)) return rc;
  __atomic_store_n(&s->srv->stop, 1u, __ATOMIC_RELEASE);
  return srv_reap(s);
}

int srv_ensure(pskv_shard* s) {
  if (!s->srv) {
    int rc = ensure_ireply(s, (size_t)kInlineGetMax * kInlineMaxChunks * 8);
    if (rc) return rc;
    void* p = nullptr;
    if (hipHostMalloc(&p, sizeof(SrvRing), hipHostMallocCoherent) != hipSuccess)
      return fail(PSKV_ENOMEM, "request ring allocation failed");
    std::memset(p, 0, sizeof(SrvRing));
    s->srv = static_cast<SrvRing*>(p);
    PSKV_HIP(hipStreamCreateWithFlags(&s->srv_stream, hipStreamNonBlocking));
    PSKV_HIP(hipEventCreateWithFlags(&s->srv_dep, hipEventDisableTiming | hipEventDisableSystemFence));
    PSKV_HIP(hipDeviceGetAttribute(&s->wall_khz, hipDeviceAttributeWallClockRate, s->device));
  }
  if (s->srv_running && __atomic_load_n(&s->srv->alive, __ATOMIC_ACQUIRE) == 0u)
    if (int rc = srv_reap(s)) return rc;
  if (!s->srv_running) return srv_launch(s);
  return PSKV_OK;
}

// The slot of the next request (waits while the ring is full).
int srv_slot(pskv_shard* s, SrvSlot** slot) {
  const uint32_t q = s->srv_posted + 1;
  if ((int32_t)(q - __atomic_load_n(&s->srv->done_seq, __ATOMIC_ACQUIRE)) > kSrvSlots)
    if (int rc = srv_wait(s, q - kSrvSlots)) return rc;
  *slot = &s->srv->slot[q % kSrvSlots];
  return PSKV_OK;
}

void srv_publish(pskv_shard* s) {
  const uint32_t q = ++s->srv_posted;
  __atomic_store_n(&s->srv->req_seq, q, __ATOMIC_RELEASE);
}

// ------------------------------------------------------- overflow table
// One array set of the table: keys EMPTY, values 0 (stream-ordered), tracked
// in s->tables.
int alloc_tab(pskv_shard* s, uint64_t cap, OvfTab* out) {
  OvfTab t{};
  if (hipMalloc(&t.keys, cap * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&t.vals, cap * (size_t)s->vb) != hipSuccess) {
    if (t.keys) (void)hipFree(t.keys);
    return fail(PSKV_ENOMEM, "overflow table allocation failed");
  }
  t.mask = cap - 1;
  {
    std::lock_guard<std::mutex> g(s->tab_m);
    s->tables.push_back(t);
  }
  PSKV_HIP(hipMemsetAsync(t.keys, 0xFF, cap * sizeof(unsigned long long), s->stream));
  PSKV_HIP(hipMemsetAsync(t.vals, 0, cap * (size_t)s->vb, s->stream));
  *out = t;
  return PSKV_OK;
}

// Free every array set but the current one.  Only with the shard's stream
// idle (no kernel can still hold a superseded table).
void free_stale_tables(pskv_shard* s) {
  std::lock_guard<std::mutex> g(s->tab_m);
  std::vector<OvfTab> keep;
  for (const auto& t : s->tables) {
    if (t.keys == s->cur.keys) {
      keep.push_back(t);
      continue;
    }
    (void)hipFree(t.keys);
    (void)hipFree(t.vals);
  }
  s->tables.swap(keep);
}

// Read the control block back (synchronises the stream): {count, err}, and
// adopt the table it names -- a device-side inserter may have grown it
// (ovf_reserve) -- freeing the superseded arrays.
int read_overflow_stat(pskv_shard* s, uint32_t* count, uint32_t* err) {
  if (int rc = srv_stop(s)) return rc;
  // into page-locked memory the shard owns: the copy is truly asynchronous (a
  // pageable destination would block inside the runtime, unbounded), and a
  // wait that times out leaves it writing into live memory, not a dead frame
  static_assert(sizeof(OvfCtl) <= 64, "the control block fits the read-back buffer");
  if (!s->stat_host) {
    void* p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocDefault) != hipSuccess)
      return fail(PSKV_ENOMEM, "overflow-stat read-back buffer allocation failed");
    s->stat_host = static_cast<uint32_t*>(p);
  }
  OvfCtl* st = reinterpret_cast<OvfCtl*>(s->stat_host);
  std::memset(st, 0, sizeof(OvfCtl));
  PSKV_HIP(hipMemcpyAsync(st, s->ovf.c, sizeof(OvfCtl), hipMemcpyDeviceToHost, s->stream));
  if (int rc = wait_stream(s, s->stream, "shard stream (overflow count read-back)")) return rc;
  *count = st->stat[0];
  *err = st->stat[1];
  s->ocount_known = st->stat[0];
  if (st->t.keys && st->t.keys != s->cur.keys) {
    s->cur = st->t;
    s->ocap = st->t.mask + 1;
  }
  free_stale_tables(s);
  return PSKV_OK;
}

// Grow the overflow table to at least `need` occupied slots at load <= 1/2
// (after read_overflow_stat: the stream is idle and s->cur current).
int grow_overflow(pskv_shard* s, uint64_t need) {
  if (int rc = srv_stop(s)) return rc;
  uint64_t cap = s->ocap;
  while (cap < 2 * need) cap <<= 1;
  if (cap == s->ocap) return PSKV_OK;
  OvfTab n{};
  if (int rc = alloc_tab(s, cap, &n)) return rc;
  // rehash, then the control block names the new arrays (its counts and
  // sticky bits stay where they are)
  PSKV_HIP(launch_ovf_rehash(s->vb, s->ovf, s->ocap, n, s->stream));
  if (int rc = wait_stream(s, s->stream, "shard stream (overflow table growth)")) return rc;
  s->cur = n;
  s->ocap = cap;
  free_stale_tables(s);
  return PSKV_OK;
}

// Device wait bound of a growth request (SYNC_TIMEOUT_MS in device wall-clock
// ticks; 0 = unbounded host waits still bounds the device at 10 minutes, so a
// grow service that is gone cannot hold a workgroup forever).
void refresh_grow_wait(pskv_shard* s) {
  if (!s->mbox) return;
  const uint64_t ms = s->tune_sync_timeout_ms ? s->tune_sync_timeout_ms : 600000u;
  const uint64_t ticks = ms * (uint64_t)std::max(s->wall_khz, 1);
  __atomic_store_n(&s->mbox->wait_ticks, ticks, __ATOMIC_RELEASE);
}

// The grow service: ONE host thread per process that answers the growth
// requests device-side inserters post to their shard's mailbox (ovf_reserve in
// pskv_kernels.hip).  It polls every registered mailbox (100 us apart while
// requests come, backing off to 1 ms after a quiet second), allocates arrays of
// the asked capacity on the shard's device -- only allocation: the requesting
// workgroup fills them and rehashes the table itself, so nothing here waits for
// a queue the requester may be blocking -- records them in the shard's table
// list, and answers.  A shard unregisters (under the service's lock) before its
// mailbox goes.
class GrowService {
 public:
  static GrowService& get() {
    static GrowService g;
    return g;
  }
  void add(pskv_shard* s) {
    std::lock_guard<std::mutex> g(m_);
    shards_.push_back(s);
    if (!th_.joinable()) th_ = std::thread([this] { loop(); });
    cv_.notify_all();
  }
  void remove(pskv_shard* s) {
    std::lock_guard<std::mutex> g(m_);
    shards_.erase(std::remove(shards_.begin(), shards_.end(), s), shards_.end());
  }
  ~GrowService() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }

 private:
  GrowService() = default;
  void serve(pskv_shard* s) {
    OvfMbox* m = s->mbox;
    const uint32_t seq = __atomic_load_n(&m->req_seq, __ATOMIC_ACQUIRE);
    if (seq == s->mbox_served) return;
    const uint64_t cap = __atomic_load_n(&m->req_cap, __ATOMIC_RELAXED);
    OvfTab t{};
    uint32_t ok = 0;
    if (cap >= 2 && (cap & (cap - 1)) == 0 && hipSetDevice(s->device) == hipSuccess &&
        hipMalloc(&t.keys, cap * sizeof(unsigned long long)) == hipSuccess) {
      if (hipMalloc(&t.vals, cap * (size_t)s->vb) == hipSuccess) {
        t.mask = cap - 1;
        ok = 1;
        std::lock_guard<std::mutex> g(s->tab_m);
        s->tables.push_back(t);
      } else {
        (void)hipFree(t.keys);
        t = OvfTab{};
      }
    }
    (void)hipGetLastError();
    m->resp_tab = t;
    m->resp_ok = ok;
    __atomic_store_n(&m->resp_seq, seq, __ATOMIC_RELEASE);
    s->mbox_served = seq;
    ++served_;
  }
  void loop() {
    auto quiet_since = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || !shards_.empty(); });
      if (stop_) return;
      const uint64_t before = served_;
      for (pskv_shard* s : shards_) serve(s);
      const auto now = std::chrono::steady_clock::now();
      if (served_ != before) quiet_since = now;
      const bool busy = now - quiet_since < std::chrono::seconds(1);
      cv_.wait_for(lk, std::chrono::microseconds(busy ? 100 : 1000), [&] { return stop_; });
      if (stop_) return;
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::vector<pskv_shard*> shards_;
  std::thread th_;
  bool stop_ = false;
  uint64_t served_ = 0;
};

// A call that gives up on a wait (PSKV_ESTATE) or fails after queueing work
// that still reads or writes the pinned staging buffer (H2D from it, D2H or K1
// stores into it): mark the buffer busy until the stream's current end, so the
// next host call waits (bounded) before its CPU copy touches the buffer or a
// regrowth frees it.
void hold_hstage(pskv_shard* s) {
  if (hipEventRecord(s->hstage_free, s->stream) == hipSuccess) s->hstage_pending = true;
}

int ensure_hstage(pskv_shard* s, size_t bytes) {
  if (s->hstage_pending) {
    if (int rc = wait_event(s, s->hstage_free, "pinned staging release event", s->hstage_free)) return rc;
    s->hstage_pending = false;
  }
  if (s->hstage_bytes >= bytes) return PSKV_OK;
  if (s->hstage) (void)hipHostFree(s->hstage);
  s->hstage = nullptr;
  size_t nb = std::max<size_t>(bytes + bytes / 2, 1 << 20);
  if (hipHostMalloc(&s->hstage, nb, hipHostMallocDefault) != hipSuccess) {
    s->hstage_bytes = 0;
    return fail(PSKV_ENOMEM, "pinned staging allocation failed");
  }
  s->hstage_bytes = nb;
  return PSKV_OK;
}

int ensure_dstage(pskv_shard* s, size_t bytes) {
  if (s->dstage_bytes >= bytes) return PSKV_OK;
  if (s->dstage) {
    // stream-ordered free: the buffer may still be read by queued kernels
    if (int rc = wait_stream(s, s->stream, "shard stream (device staging regrowth)")) return rc;
    (void)hipFree(s->dstage);
  }
  s->dstage = nullptr;
  size_t nb = std::max<size_t>(bytes + bytes / 2, 1 << 20);
  if (hipMalloc(&s->dstage, nb) != hipSuccess) {
    s->dstage_bytes = 0;
    return fail(PSKV_ENOMEM, "device staging allocation failed");
  }
  s->dstage_bytes = nb;
  return PSKV_OK;
}

size_t round16(size_t x) { return (x + 15) & ~size_t(15); }

// Build the kernarg group descriptor for batches [b, e) with `chunk` elements
// per workgroup.  Returns the workgroup count.
uint32_t build_group(const std::vector<pskv_batch>& v, size_t b, size_t e, uint64_t chunk,
                     GroupArgs* ga) {
  std::memset(ga, 0, sizeof(*ga));
  ga->nb = (int)(e - b);
  uint64_t wg = 0;
  for (size_t i = b; i < e; ++i) {
    const int j = (int)(i - b);
    ga->wg_prefix[j] = (uint32_t)wg;
    ga->b[j] = DevBatch{v[i].keys, v[i].vals, v[i].n};
    wg += (v[i].n + chunk - 1) / chunk;
  }
  ga->wg_prefix[e - b] = (uint32_t)wg;
  return (uint32_t)wg;
}

uint32_t next_epoch(pskv_shard* s) {
  // Stamps are epoch<<32|index; on wrap-around the stamp arrays are reset so
  // that every old stamp still loses to the new epoch 1.
  if (s->epoch == 0xFFFFFFFFu) {
    if (s->owner) (void)hipMemsetAsync(s->owner, 0, s->range * sizeof(unsigned long long), s->stream);
    (void)hipMemsetAsync(s->flag, 0, 2 * sizeof(uint32_t), s->stream);  // both tags
    s->epoch = 0;
  }
  return ++s->epoch;
}

// Append batch b to v as consecutive pieces of at most kMaxPiece elements
// (empty batches are dropped).  A batch applied piece by piece in order is the
// same Add (last-wins / sums follow index order) and the same Get, and every
// launch group then stays below 2^32 elements (the stamp index and the
// per-launch element counts are 32 bits).
constexpr uint64_t kMaxPiece = 1ull << 31;
void push_pieces(std::vector<pskv_batch>& v, const pskv_batch& b, size_t vb) {
  for (uint64_t off = 0; off < b.n; off += kMaxPiece)
    v.push_back(pskv_batch{b.keys + off, static_cast<char*>(b.vals) + off * vb, std::min(kMaxPiece, b.n - off)});
}

// Split a batch list into launch groups: <= kMaxBatches batches and < 2^32
// elements each.  Every batch holds at most kMaxPiece elements (push_pieces),
// so every group takes at least one batch.
std::vector<std::pair<size_t, size_t>> split_groups(const std::vector<pskv_batch>& v) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t b = 0;
  while (b < v.size()) {
    size_t e = b;
    uint64_t el = 0;
    while (e < v.size() && e - b < (size_t)kMaxBatches && el + v[e].n < (1ull << 32)) {
      el += v[e].n;
      ++e;
    }
    out.emplace_back(b, e);
    b = e;
  }
  return out;
}

// Grow a device scratch buffer (stream-ordered: queued kernels may still use
// the old one, so synchronise before freeing it).
int ensure_scratch(pskv_shard* s, void** p, size_t* have, size_t need) {
  if (*have >= need) return PSKV_OK;
  if (*p) {
    if (int rc = wait_stream(s, s->stream, "shard stream (scratch regrowth)")) return rc;
    (void)hipFree(*p);
  }
  *p = nullptr;
  const size_t nb = std::max<size_t>(need + need / 4, 1 << 16);
  if (hipMalloc(p, nb) != hipSuccess) {
    *p = nullptr;
    *have = 0;
    return fail(PSKV_ENOMEM, "scratch allocation failed");
  }
  *have = nb;
  return PSKV_OK;
}

// K5: radix-bucket general Add (no random global atomics), one launch pair
// per <= kRbMaxSc super-chunks; a longer group is cut into consecutive pieces
// (a batch may be split), which run in stream order, so call order holds.
int radix_launch(pskv_shard* s, const std::vector<pskv_batch>& v, size_t b, size_t e) {
  GroupArgs ga;
  const uint32_t nsc = build_group(v, b, e, rb_superchunk(s->vb, s->tune_rb_bin_block), &ga);
  uint64_t elems = 0;
  for (size_t i = b; i < e; ++i) elems += v[i].n;
  // bucket = key offset >> bshift (more buckets: longer loff rows, shorter
  // runs).  Per mode: assign takes one bucket per 2 Ki pushed keys, at most
  // 2^11 bucket bits; accumulate, whose resolve also reads the parameters, one
  // per 4 Ki, at most 2^10.  The sweep behind the rule (tools/zipf_probe.py,
  // 4/8/16 x 1M Zipf keys) and its timings: DESIGN.md §7 "K5 bucket count",
  // logs in profiles/r01_probes/probe_tb*.log and probe_new_*.log.
  // The resolve workgroup uses a 2^13-slot LDS table while buckets average
  // <= 2 Ki pushed keys, else 2^14.
  uint32_t bits = 0;
  while (bits < 32 && ((s->range - 1) >> bits) != 0) ++bits;
  const uint32_t per = s->mode == PSKV_ASSIGN ? 11 : 12, tmax = s->mode == PSKV_ASSIGN ? 11 : 10;
  uint32_t tb = 6;
  while (tb < tmax && (elems >> (per + tb)) != 0) ++tb;
  if (s->tune_rb_tb) tb = s->tune_rb_tb;
  const uint32_t bshift = bits > tb ? bits - tb : 0;
  uint32_t nbd = (uint32_t)(((s->range - 1) >> bshift) + 1);
  if (s->tune_rb_nbd) nbd = s->tune_rb_nbd;
  const uint32_t nbk = nbd + 1;
  // The buckets own windows of 2^wbits keys dealt round-robin (window w ->
  // bucket w % nbd); wbits = bshift is one contiguous window per bucket.
  RbMap bm;
  bm.wbits = std::min<uint32_t>(bshift, s->tune_rb_wbits ? s->tune_rb_wbits : 11u);
  bm.nbd = nbd;
  bm.nlog = -1;
  for (int l = 0; l < 12; ++l)
    if (nbd == (1u << l)) bm.nlog = l;
  bm.magic = nbd > 1 ? (uint32_t)(((1ull << 32) + nbd - 1) / nbd) : 0u;  // nbd = 1 takes the shift path
  const uint64_t nwin = ((s->range - 1) >> bm.wbits) + 1;  // < 2^21: wbits = 11, or wbits = bshift and nwin = nbd
  bm.span = (uint32_t)std::min<uint64_t>(((nwin + nbd - 1) / nbd) << bm.wbits, 0xFFFFFFFFull);
  int apply_log2 = elems / nbd <= 2048 ? 13 : 14;
  if (s->tune_rb_apply_log2) apply_log2 = s->tune_rb_apply_log2;
  if (nbk > (uint32_t)kRbMaxBuckets) return fail(PSKV_EINVAL, "radix path: too many buckets");
  if (nsc > kRbMaxSc) return fail(PSKV_EINVAL, "radix path: launch piece too large");
  const size_t eb = rb_entry_bytes(s->vb);
  int rc = ensure_scratch(s, reinterpret_cast<void**>(&s->rb_loff), &s->rb_loff_bytes,
                          (size_t)nsc * (nbk + 1) * sizeof(uint16_t));
  if (!rc)
    rc = ensure_scratch(s, &s->rb_ent, &s->rb_ent_bytes,
                        (size_t)nsc * rb_superchunk(s->vb, s->tune_rb_bin_block) * eb + kRbTmpPad);
  if (rc) return rc;
  LaunchTimer t(s, PSKV_K_RADIX, elems);
  PSKV_HIP(launch_rb_add(s->dtype, s->mode, ga, nsc, s->dview(), s->ovf, bm, apply_log2,
                         s->tune_rb_bin_block, s->rb_loff, s->rb_ent, s->stream));
  t.done();
  s->n_general += 2;
  return PSKV_OK;
}

int radix_add(pskv_shard* s, const std::vector<pskv_batch>& v, size_t b, size_t e) {
  const uint64_t sc = rb_superchunk(s->vb, s->tune_rb_bin_block);
  uint64_t nsc = 0;
  for (size_t i = b; i < e; ++i) nsc += (v[i].n + sc - 1) / sc;
  const uint64_t max_sc = kRbMaxSc;
  if (nsc <= max_sc) return radix_launch(s, v, b, e);
  // pieces of whole super-chunks, each <= max_sc of them
  std::vector<pskv_batch> piece;
  uint64_t used = 0;  // super-chunks in `piece`
  auto flush = [&]() -> int {
    if (piece.empty()) return PSKV_OK;
    const int rc = radix_launch(s, piece, 0, piece.size());
    piece.clear();
    used = 0;
    return rc;
  };
  for (size_t i = b; i < e; ++i) {
    uint64_t off = 0;
    while (off < v[i].n) {
      if (used == max_sc || piece.size() == (size_t)kMaxBatches) {
        if (int rc = flush()) return rc;
      }
      const uint64_t room = (max_sc - used) * sc;
      const uint64_t n = std::min<uint64_t>(v[i].n - off, room);
      piece.push_back(pskv_batch{v[i].keys + off,
                                 static_cast<char*>(v[i].vals) + off * (uint64_t)s->vb, n});
      used += (n + sc - 1) / sc;
      off += n;
    }
  }
  return flush();
}

// The general (any order) Add over one launch group.  `cond` non-null makes
// it a repair that runs only when the sorted path tagged `epoch` (K4, whose
// idle launches are cheap); unconditional general Adds take K5.
int general_add(pskv_shard* s, const std::vector<pskv_batch>& v, size_t b, size_t e,
                uint32_t epoch, const uint32_t* cond, bool radix = true) {
  if (!cond && ((radix && s->general_path == 1) || s->general_path == 2)) return radix_add(s, v, b, e);
  if (s->mode == PSKV_ASSIGN && !s->owner) {
    // The stamp array is only needed once the general path can run: allocate it
    // on first use (8 B per owned key).
    const size_t bytes = s->range * sizeof(unsigned long long);
    if (hipMalloc(&s->owner, bytes) != hipSuccess) {
      s->owner = nullptr;
      return fail(PSKV_ENOMEM, "stamp array allocation failed");
    }
    PSKV_HIP(hipMemsetAsync(s->owner, 0, bytes, s->stream));
  }
  GroupArgs ga;
  const uint32_t nwg = build_group(v, b, e, kGeneralChunk, &ga);
  uint64_t elems = 0;
  for (size_t i = b; i < e; ++i) elems += v[i].n;
  {
    LaunchTimer t(s, PSKV_K_GENERAL_MARK, elems);
    PSKV_HIP(launch_general_mark(s->dtype, s->mode, ga, nwg, s->dview(), s->flag + 1, s->owner, cond,
                                 epoch, s->stream));
    t.done();
  }
  s->n_general++;
  if (s->mode == PSKV_ASSIGN) {
    LaunchTimer t(s, PSKV_K_GENERAL_COMMIT, elems);
    PSKV_HIP(launch_general_commit(s->vb, ga, nwg, s->dview(), s->owner, cond, epoch, s->stream));
    t.done();
    s->n_general++;
  }
  // the group's out-of-range keys, which K4a only tagged (flag[1]): one
  // workgroup applies them in call order, growing the table as it goes
  {
    LaunchTimer t(s, PSKV_K_REPLAY, elems);
    PSKV_HIP(launch_replay(s->dtype, s->mode, ga, s->dview(), s->ovf, s->flag + 1, epoch, s->stream,
                           /*oor_only=*/true));
    t.done();
    s->n_general++;
  }
  return PSKV_OK;
}

// A held replay (see replay) launched as K4r, its own launch.
int flush_replay(pskv_shard* s) {
  if (!s->pend_replay) return PSKV_OK;
  GroupArgs ga;
  ga.nb = s->pend_rg.nb;
  for (int i = 0; i < ga.nb; ++i) ga.b[i] = s->pend_rg.b[i];
  LaunchTimer t(s, PSKV_K_REPLAY, s->pend_elems);
  PSKV_HIP(launch_replay(s->dtype, s->mode, ga, s->dview(), s->ovf, s->flag, s->pend_epoch, s->stream));
  s->pend_replay = false;  // (held until its launch is queued)
  t.done();
  s->n_general++;
  return PSKV_OK;
}

// The safety net behind a verifying sorted-path launch group: K4r replays the
// group in call order iff the verification tagged s->flag with `epoch` (one
// single-workgroup launch that exits at once otherwise).
// Inside pskv_add_get_grouped (s->defer_replay) the replay of an assign group
// with 4-byte values is held instead (pend_*): the Get's first K1 launch takes
// it (K1r), or flush_replay launches it as K4r before anything else is queued.
int replay(pskv_shard* s, const std::vector<pskv_batch>& v, size_t b, size_t e, uint32_t epoch) {
  GroupArgs ga;
  (void)build_group(v, b, e, kGeneralChunk, &ga);
  uint64_t elems = 0;
  for (size_t i = b; i < e; ++i) elems += v[i].n;
  if (s->defer_replay && s->mode == PSKV_ASSIGN && s->vb == 4) {
    if (int rc = flush_replay(s)) return rc;  // (add_impl flushed it already: the order holds either way)
    s->pend_rg.nb = ga.nb;
    for (int i = 0; i < ga.nb; ++i) s->pend_rg.b[i] = ga.b[i];
    s->pend_epoch = epoch;
    s->pend_elems = elems;
    s->pend_replay = true;
    return PSKV_OK;
  }
  LaunchTimer t(s, PSKV_K_REPLAY, elems);
  PSKV_HIP(launch_replay(s->dtype, s->mode, ga, s->dview(), s->ovf, s->flag, epoch, s->stream));
  t.done();
  s->n_general++;
  return PSKV_OK;
}

// Sorted path over one launch group of device-resident batches (verifying);
// `repair` adds the conditional replay launch behind it; `maybe_windows` false
// (a host group proven sorted but not all windows) keeps K2g out of early mode.
int sorted_add(pskv_shard* s, const std::vector<pskv_batch>& v, size_t b, size_t e, bool vec,
               uint32_t epoch, bool repair, bool maybe_windows) {
  uint64_t elems = 0;
  for (size_t i = b; i < e; ++i) elems += v[i].n;
  if (e - b == 1) {
    LaunchTimer t(s, PSKV_K_ASSIGN_SORTED, elems);
    PSKV_HIP(launch_assign_sorted(s->vb, vec, v[b].keys, v[b].vals, v[b].n, s->dview(), s->flag,
                                  epoch, s->stream));
    t.done();
  } else {
    GroupArgs ga;
    const uint32_t nchunks = build_group(v, b, e, stream_chunk(s->tune_unroll), &ga);
    // Tile (tile mode): enough tiles for several workgroups per CU, 4 Ki..64 Ki keys.
    uint32_t shift = 16;
    while (shift > 12 && (elems >> shift) < 2048) --shift;
    if (s->tune_tile_shift) shift = s->tune_tile_shift;
    const uint64_t ntiles = (s->range + (1ull << shift) - 1) >> shift;
    // grid: one workgroup per dense-mode chunk (the common case: every batch a
    // window), at least 1024 for the tile mode's grid-stride over the tiles;
    // a workgroup beyond the chunks only runs the prologue (two dependent key
    // loads per batch) and leaves
    const uint32_t grid = (uint32_t)std::min<uint64_t>(
        std::max<uint64_t>(std::min<uint64_t>(ntiles, 1024), nchunks), s->tune_tile_grid);
    // Early mode (K2g's whole-chunk loads issued before its prologue, its
    // chunks storing their own elements): for launches whose windows are
    // unlikely to overlap — the pushed keys cover under a quarter of the
    // shard's range, e.g. a rank's share of cfg 4 — since it cannot skip the
    // values of a chunk a later window covers.  Results are the same either way.
    // A host group the CPU found sorted but not all windows goes to the tile
    // mode, where early loads would only be read again (maybe_windows false).
    const bool early = s->tune_early == 1 || (s->tune_early == 2 && maybe_windows && elems * 4 < s->range);
    LaunchTimer t(s, PSKV_K_ASSIGN_TILES, elems);
    PSKV_HIP(launch_assign_group(s->vb, vec, s->tune_unroll, s->tune_nt, s->tune_ntp, early, ga, s->dview(),
                                 shift, ntiles, grid, s->flag, epoch, s->stream));
    t.done();
  }
  s->n_sorted++;
  if (repair) return replay(s, v, b, e, epoch);
  return PSKV_OK;
}

// Accumulate over dense windows (K7), one launch group.  `verify`: device
// inputs under PSKV_SORTED_HINT are first proven dense by K6; if not, K7 skips
// and the conditional K4a accumulate takes the group.  Host inputs come
// proven by the CPU check (verify = false).
int dense_accumulate(pskv_shard* s, const std::vector<pskv_batch>& v, size_t b, size_t e,
                     uint32_t epoch, bool verify) {
  uint64_t elems = 0;
  for (size_t i = b; i < e; ++i) elems += v[i].n;
  GroupArgs ga;
  const uint32_t nchunks = build_group(v, b, e, stream_chunk(8), &ga);
  if (verify) {
    LaunchTimer t(s, PSKV_K_DENSE_CHECK, elems);
    PSKV_HIP(launch_dense_check(ga, nchunks, s->dview(), s->flag, epoch, s->stream));
    t.done();
  }
  {
    const uint32_t grid = std::min<uint32_t>(nchunks, s->tune_tile_grid);
    LaunchTimer t(s, PSKV_K_ACC_DENSE, elems);
    PSKV_HIP(launch_acc_dense(s->dtype, ga, grid, s->dview(), s->flag, epoch, s->stream));
    t.done();
  }
  s->n_sorted++;
  if (verify) return replay(s, v, b, e, epoch);
  return PSKV_OK;
}

// One contiguous piece of a host->pinned (or pinned->host) copy.
struct Piece {
  const char* src;
  char* dst;
  size_t bytes;
  int key_batch;  // >= 0: keys of that batch (checked while copied), -1: values
  // results of the key check
  bool sorted;
  bool dense;  // every key is its predecessor + 1
  uint32_t first, last;
  uint64_t outside;
};

// The key check, written so the compiler vectorises it (no loop-carried
// state but the or / sum reductions): 2-4x the rate of the sequential form.
void check_keys(Piece& p, const uint32_t* k, size_t n, uint32_t key_begin, uint64_t range) {
  p.sorted = p.dense = true;
  p.first = p.last = 0;
  p.outside = 0;
  if (!n) return;
  const uint32_t rmax = range ? (uint32_t)(range - 1) : 0u;  // in range: (x - key_begin) <= rmax
  uint32_t unsorted = 0, gap = 0, out = (uint32_t)(k[0] - key_begin) > rmax;
  for (size_t i = 1; i < n; ++i) {
    const uint32_t a = k[i - 1], x = k[i];
    unsorted |= (uint32_t)(a > x);
    gap |= (uint32_t)(x != a + 1u);
    out += (uint32_t)((uint32_t)(x - key_begin) > rmax);
  }
  p.sorted = unsorted == 0;
  p.dense = gap == 0;
  p.first = k[0];
  p.last = k[n - 1];
  p.outside = range ? out : n;  // pieces hold < 2^32 keys
}

void copy_piece(Piece& p, uint32_t key_begin, uint64_t range) {
  if (p.key_batch < 0) {
    std::memcpy(p.dst, p.src, p.bytes);
    return;
  }
  if (p.dst) std::memcpy(p.dst, p.src, p.bytes);  // else a page-locked caller buffer: check only
  check_keys(p, reinterpret_cast<const uint32_t*>(p.src), p.bytes / 4, key_begin, range);
}

// Cut [src, src+bytes) into pieces appended to `out`; check-only pieces
// (dst null) are smaller, so a pool spreads a medium batch's check wider.
void add_pieces(std::vector<Piece>& out, const void* src, char* dst, size_t bytes, int key_batch) {
  const char* s = static_cast<const char*>(src);
  const size_t piece = dst ? kPieceBytes : kCheckPieceBytes;
  for (size_t off = 0; off < bytes; off += piece) {
    Piece p{};
    p.src = s + off;
    p.dst = dst ? dst + off : nullptr;
    p.bytes = std::min(piece, bytes - off);
    p.key_batch = key_batch;
    p.sorted = true;
    p.dense = true;
    out.push_back(p);
  }
}

// Combine the per-piece key checks: every piece sorted, and each piece's first
// key not below the previous piece's last key within the same batch.
void combine_checks(const std::vector<Piece>& pieces, bool* all_sorted_in_range,
                    uint64_t* n_outside, bool* all_dense_in_range) {
  bool ok = true, dense = true;
  uint64_t outside = 0;
  int prev_batch = -1;
  uint32_t prev_last = 0;
  for (const auto& p : pieces) {
    if (p.key_batch < 0) continue;
    outside += p.outside;
    ok &= p.sorted;
    dense &= p.dense;
    if (p.key_batch == prev_batch) {
      ok &= prev_last <= p.first;
      dense &= p.first == prev_last + 1u;
    }
    prev_batch = p.key_batch;
    prev_last = p.last;
  }
  *all_sorted_in_range = ok && outside == 0;
  if (all_dense_in_range) *all_dense_in_range = dense && outside == 0;
  *n_outside = outside;
}

// Copy pieces window by window (pool in parallel) and DMA each window to the
// device as soon as it is staged, so the copy of window w+1 overlaps the H2D
// of window w.  Pieces must be in increasing staging order.
int pipelined_h2d(pskv_shard* s, std::vector<Piece>& pieces, char* h, char* d) {
  size_t i = 0;
  while (i < pieces.size()) {
    size_t j = i, win = 0;
    while (j < pieces.size() && (win < kWindowBytes || j == i)) win += pieces[j++].bytes;
    run_pieces(pieces, i, j, [&](Piece& p) { copy_piece(p, s->key_begin, s->range); });
    char* lo = pieces[i].dst;
    char* hi = pieces[j - 1].dst + pieces[j - 1].bytes;
    const hipError_t e = hipMemcpyAsync(d + (lo - h), lo, (size_t)(hi - lo), hipMemcpyHostToDevice, s->stream);
    if (e != hipSuccess) {
      if (i) hold_hstage(s);  // the windows queued before still read the staging
      PSKV_HIP(e);
    }
    i = j;
  }
  return PSKV_OK;
}

// Page-locked (hipHostMalloc'd / registered) host memory: the DMA engine can
// read or write it directly, so no staging copy is needed.
bool is_pinned(const void* p, void** dev = nullptr) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (dev) *dev = a.devicePointer;
  return a.type == hipMemoryTypeHost && (!dev || a.devicePointer);
}

// Device view of [p, p + bytes) when the whole range lies in ONE page-locked
// allocation (hipHostMalloc'd or registered), else null: a kernel reads and
// writes through the view, so a range that runs past its registration (a
// sub-range registration, a slice across two) must take the DMA path instead.
void* pinned_range_view(const void* p, size_t bytes) {
  void* dev = nullptr;
  if (!is_pinned(p, &dev)) return nullptr;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(dev)) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  const uintptr_t b = reinterpret_cast<uintptr_t>(base), d = reinterpret_cast<uintptr_t>(dev);
  if (d < b || d + bytes > b + size) return nullptr;
  // in place only through the unified address (valid on every device; see
  // pskv_frames.cpp): a device-specific view would tie the buffer to the
  // device that was current when the attributes were read
  if (dev != p) return nullptr;
  return dev;
}

// Device views of page-locked host batches (frames or any other pinned
// memory), or false.
bool pinned_views(const std::vector<pskv_batch>& in, size_t vb, std::vector<pskv_batch>* out) {
  out->clear();
  for (const auto& b : in) {
    pskv_batch d = b;
    void* k = pinned_range_view(b.keys, b.n * 4);
    void* v = pinned_range_view(b.vals, b.n * vb);
    if (!k || !v) return false;
    d.keys = static_cast<const uint32_t*>(k);
    d.vals = v;
    out->push_back(d);
  }
  return true;
}

// Stage host batches into one device buffer (keys then values per batch,
// 16-byte aligned) through pinned memory, checking on the way whether every
// batch is sorted and inside the dense range.  Returns device batch views.
int stage_host_batches(pskv_shard* s, const std::vector<pskv_batch>& in,
                       std::vector<pskv_batch>* out, bool* all_sorted_in_range,
                       uint64_t* n_outside, bool* all_dense_in_range = nullptr) {
  size_t bytes = 0;
  for (auto& b : in) bytes += round16(b.n * 4) + round16(b.n * (size_t)s->vb);
  bool locked = true;
  for (const auto& b : in) locked = locked && is_pinned(b.keys) && is_pinned(b.vals);
  // page-locked buffers: DMA'd directly from tune_dma_min_bytes_pinned on
  // (below it the copy, which returns before the DMA, is ahead); pageable
  // buffers only when large (the runtime's pageable copy has a high fixed cost
  // and blocks until done).  Smaller ones are copied into pinned staging and
  // DMA'd asynchronously (the call returns after the host copy).
  locked = locked && bytes >= s->tune_dma_min_bytes_pinned;
  const bool pinned = locked || (s->tune_pageable_dma && bytes >= s->tune_dma_min_bytes);
  int rc = pinned ? PSKV_OK : ensure_hstage(s, bytes);
  if (rc) return rc;
  rc = ensure_dstage(s, bytes);
  if (rc) return rc;
  char* h = static_cast<char*>(s->hstage);
  char* d = static_cast<char*>(s->dstage);
  std::vector<Piece> pieces;
  size_t off = 0;
  out->clear();
  std::vector<std::pair<char*, const pskv_batch*>> dma;  // direct DMA: (device dst, batch)
  for (size_t j = 0; j < in.size(); ++j) {
    const auto& b = in[j];
    pskv_batch db;
    if (pinned) {
      // DMA straight from the caller's buffers; the CPU only checks
      dma.emplace_back(d + off, &b);
      add_pieces(pieces, b.keys, nullptr, b.n * 4, (int)j);
    } else {
      add_pieces(pieces, b.keys, h + off, b.n * 4, (int)j);
    }
    db.keys = reinterpret_cast<const uint32_t*>(d + off);
    off += round16(b.n * 4);
    if (!pinned) add_pieces(pieces, b.vals, h + off, b.n * (size_t)s->vb, -1);
    db.vals = d + off;
    db.n = b.n;
    off += round16(b.n * (size_t)s->vb);
    out->push_back(db);
  }
  if (pinned) {
    auto issue = [&]() -> hipError_t {
      for (const auto& x : dma) {
        const pskv_batch& b = *x.second;
        hipError_t e = hipMemcpyAsync(x.first, b.keys, b.n * 4, hipMemcpyHostToDevice, s->stream);
        if (e == hipSuccess)
          e = hipMemcpyAsync(x.first + round16(b.n * 4), b.vals, b.n * (size_t)s->vb,
                             hipMemcpyHostToDevice, s->stream);
        if (e != hipSuccess) return e;
      }
      return hipEventRecord(s->h2d_done, s->stream);
    };
    auto check = [&]() {
      HostPool::get().run(pieces.size(),
                          [&](size_t t) { copy_piece(pieces[t], s->key_begin, s->range); });
    };
    hipError_t e = hipSuccess;
    if (locked) {  // page-locked: the copies are queued at once
      e = issue();
      check();
    } else {
      // pageable (PSKV_PAGEABLE_DMA): the runtime's copies block the issuing
      // thread, so they are issued from a helper while the pool checks
      std::thread t;
      try {
        t = std::thread([&]() {
          (void)hipSetDevice(s->device);
          e = issue();
        });
      } catch (...) {  // no helper thread: issue, then check
      }
      if (!t.joinable()) e = issue();
      check();
      if (t.joinable()) t.join();
    }
    if (e != hipSuccess) {
      // copies queued before the failure may still read the caller's buffers
      (void)wait_stream(s, s->stream, "shard stream (failed host copy)");
      PSKV_HIP(e);
    }
    // the caller may reuse its buffers once this returns
    if (int rc2 = wait_event(s, s->h2d_done, "host-buffer DMA completion event", s->h2d_done)) return rc2;
  } else {
    rc = pipelined_h2d(s, pieces, h, d);
    if (rc) return rc;
    PSKV_HIP(hipEventRecord(s->hstage_free, s->stream));
    s->hstage_pending = true;
  }
  combine_checks(pieces, all_sorted_in_range, n_outside, all_dense_in_range);
  return PSKV_OK;
}

// Device views of host batches that lie in pskv_host_alloc frames (every
// keys and values range inside one live frame), or false.
bool frame_views(const std::vector<pskv_batch>& in, size_t vb, std::vector<pskv_batch>* out) {
  out->clear();
  for (const auto& b : in) {
    pskv_batch d = b;
    d.keys = static_cast<const uint32_t*>(frames::device_view(b.keys, b.n * 4));
    d.vals = frames::device_view(b.vals, b.n * vb);
    if (!d.keys || !d.vals) return false;
    out->push_back(d);
  }
  return true;
}

// Host Add batches in borrowed frames (PSKV_HOST_FRAME): the CPU checks the
// keys (sorted / dense / in range, as for staged inputs) without copying
// anything; the kernels then read the frames in place across PCIe when the
// call is at most tune_frame_zc_max_bytes, otherwise the frames are DMA'd
// into device staging.  Either way nothing waits: the frames stay unmodified
// until freed, and pskv_host_free holds them until this call's work has run
// (note_frame_uses).
int frame_batches(pskv_shard* s, const std::vector<pskv_batch>& in,
                  const std::vector<pskv_batch>& views, std::vector<pskv_batch>* out,
                  bool* all_sorted_in_range, uint64_t* n_outside, bool* all_dense_in_range) {
  size_t bytes = 0;
  for (auto& b : in) bytes += round16(b.n * 4) + round16(b.n * (size_t)s->vb);
  std::vector<Piece> pieces;
  for (size_t j = 0; j < in.size(); ++j) add_pieces(pieces, in[j].keys, nullptr, in[j].n * 4, (int)j);
  if (bytes <= s->tune_frame_zc_max_bytes) {
    *out = views;
  } else {
    int rc = ensure_dstage(s, bytes);
    if (rc) return rc;
    char* d = static_cast<char*>(s->dstage);
    size_t off = 0;
    out->clear();
    for (const auto& b : in) {
      pskv_batch db;
      PSKV_HIP(hipMemcpyAsync(d + off, b.keys, b.n * 4, hipMemcpyHostToDevice, s->stream));
      db.keys = reinterpret_cast<const uint32_t*>(d + off);
      off += round16(b.n * 4);
      PSKV_HIP(hipMemcpyAsync(d + off, b.vals, b.n * (size_t)s->vb, hipMemcpyHostToDevice, s->stream));
      db.vals = d + off;
      off += round16(b.n * (size_t)s->vb);
      db.n = b.n;
      out->push_back(db);
    }
  }
  run_pieces(pieces, 0, pieces.size(), [&](Piece& p) { copy_piece(p, s->key_begin, s->range); });
  combine_checks(pieces, all_sorted_in_range, n_outside, all_dense_in_range);
  return PSKV_OK;
}

// The work queued so far reads the frames of `v` (host pointers).
int note_frame_uses(pskv_shard* s, const std::vector<pskv_batch>& v) {
  std::string err;
  for (const auto& b : v) {
    int rc = frames::note_use(b.keys, s->device, s->stream, &err);
    if (!rc && b.vals != static_cast<const void*>(b.keys))
      rc = frames::note_use(b.vals, s->device, s->stream, &err);
    if (rc) return fail(rc, err);
  }
  return PSKV_OK;
}

// K8: a host Add of at most kInlineMax keys per launch (the reference's
// per-sample messages), up to tune_inline_chunks launches per call.  The
// grouped form equals the concatenation of its batches in order (last-wins /
// sums follow index order across batches), and so does a sequence of launches
// over consecutive pieces of it, so the batches are packed into kernel-argument
// messages of kInlineMax keys; the caller's buffers are free once the launches
// are enqueued (the runtime copies the arguments).
int inline_add(pskv_shard* s, const std::vector<pskv_batch>& v) {
  // (out-of-range keys need no host step: K8 / K9 reserve room in the
  // overflow table on the device, ovf_reserve)
  const bool serve = serve_on(s);
  if (int rc = serve ? srv_ensure(s) : srv_stop(s)) return rc;
  InlineAdd a;
  a.n = 0;
  auto flush = [&]() -> int {
    if (a.n == 0) return PSKV_OK;
    if (serve) {  // K9: one ring slot instead of a launch
      SrvSlot* sl = nullptr;
      if (int rc = srv_slot(s, &sl)) return rc;
      sl->kind = kSrvAdd;
      sl->n = a.n;
      std::memcpy(sl->keys, a.keys, a.n * sizeof(uint32_t));
      std::memcpy(sl->vals, a.vals, a.n * sizeof(unsigned long long));
      srv_publish(s);
      a.n = 0;
      return PSKV_OK;
    }
    LaunchTimer t(s, PSKV_K_INLINE_ADD, a.n);
    PSKV_HIP(launch_inline_add(s->dtype, s->mode, a, s->dview(), s->ovf, s->stream));
    t.done();
    a.n = 0;
    return PSKV_OK;
  };
  for (const auto& b : v) {
    for (uint64_t e = 0; e < b.n; ++e) {
      const uint32_t i = a.n++;
      a.keys[i] = b.keys[e];
      if (s->vb == 8) {
        std::memcpy(&a.vals[i], static_cast<const char*>(b.vals) + e * 8, 8);
      } else {
        uint32_t w;
        std::memcpy(&w, static_cast<const char*>(b.vals) + e * 4, 4);
        a.vals[i] = w;
      }
      if (a.n == (uint32_t)kInlineMax)
        if (int rc = flush()) return rc;
    }
  }
  return flush();
}

// K8 Get: keys in the kernel arguments (kInlineGetMax per launch), the reply
// written by the kernels into a page-locked buffer, copied out to the caller
// once the LAST launch has published (stream order: the earlier ones are done).
int inline_get(pskv_shard* s, const std::vector<pskv_batch>& v, uint64_t total) {
  const size_t cap = (size_t)kInlineGetMax * kInlineMaxChunks * 8;
  if (int rc = ensure_ireply(s, cap)) return rc;
  if (serve_on(s)) {  // K9: ring slots of kInlineGetMax keys, then wait for the last
    if (int rc = srv_ensure(s)) return rc;
    uint64_t off = 0;
    SrvSlot* sl = nullptr;
    for (const auto& b : v) {
      for (uint64_t e = 0; e < b.n; ++e) {
        if (!sl) {
          if (int rc = srv_slot(s, &sl)) return rc;
          sl->kind = kSrvGet;
          sl->n = 0;
          sl->reply_off = (uint32_t)off;
        }
        sl->keys[sl->n++] = b.keys[e];
        ++off;
        if (sl->n == (uint32_t)kInlineGetMax) {
          srv_publish(s);
          sl = nullptr;
        }
      }
    }
    if (sl) srv_publish(s);
    if (int rc = srv_wait(s, s->srv_posted)) return rc;
    const char* r = static_cast<const char*>(s->ireply);
    for (const auto& b : v) {
      std::memcpy(b.vals, r, b.n * (size_t)s->vb);
      r += b.n * (size_t)s->vb;
    }
    return PSKV_OK;
  }
  if (int rc = srv_stop(s)) return rc;  // the K8 launches run on the shard's stream
  unsigned int* done = reinterpret_cast<unsigned int*>(static_cast<char*>(s->ireply) + cap);
  const unsigned int seq = ++s->ireply_seq;
  InlineGet a;
  a.n = 0;
  uint64_t issued = 0;  // values requested by earlier launches
  bool spin = false;
  auto flush = [&](bool last) -> int {
    if (a.n == 0) return PSKV_OK;
    LaunchTimer t(s, PSKV_K_INLINE_GET, a.n);
    // spin-wait reply (coherent host buffer, no timing events to drain): the
    // last kernel publishes a sequence number after the values; the host polls it
    spin = last && s->tune_ispin && !t.a;
    PSKV_HIP(launch_inline_get(s->vb, a, s->dview(), s->ovf,
                               static_cast<char*>(s->ireply) + issued * (size_t)s->vb,
                               spin ? done : nullptr, seq, s->stream));
    t.done();
    issued += a.n;
    a.n = 0;
    return PSKV_OK;
  };
  uint64_t seen = 0;
  for (const auto& b : v) {
    for (uint64_t e = 0; e < b.n; ++e) {
      a.keys[a.n++] = b.keys[e];
      ++seen;
      if (a.n == (uint32_t)kInlineGetMax)
        if (int rc = flush(seen == total)) return rc;
    }
  }
  if (int rc = flush(true)) return rc;
  if (spin) {
    // poll the sequence word; every 1024 polls ask the stream whether it
    // finished (or failed) without publishing, so a fault cannot hang the host
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t it = 1;; ++it) {
      if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == seq) break;
      if ((it & 1023u) == 0) {
        const hipError_t e = hipStreamQuery(s->stream);
        if (e == hipSuccess) {
          if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == seq) break;
          return fail(PSKV_EHIP, "inline get: kernel finished without publishing its reply");
        }
        if (e != hipErrorNotReady) PSKV_HIP(e);
        // bounded like every other host wait (PSKV_SYNC_TIMEOUT_MS)
        const double ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (s->tune_sync_timeout_ms && ms > (double)s->tune_sync_timeout_ms)
          return fail(PSKV_ESTATE, wait_report(s, "shard stream (inline Get reply)", s->stream, ms));
        if (ms > 50.0) std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
    }
  } else {
    if (int rc = wait_stream(s, s->stream, "shard stream (inline Get)")) return rc;
  }
  const char* r = static_cast<const char*>(s->ireply);
  for (const auto& b : v) {
    std::memcpy(b.vals, r, b.n * (size_t)s->vb);
    r += b.n * (size_t)s->vb;
  }
  return PSKV_OK;
}

int add_impl(pskv_shard* s, const std::vector<pskv_batch>& in, int flags) {
  std::vector<pskv_batch> v;
  for (auto& b : in) {
    if (b.n == 0) continue;
    if (!b.keys || !b.vals) return fail(PSKV_EINVAL, "pskv_add: null keys/vals with n > 0");
    push_pieces(v, b, (size_t)s->vb);
  }
  s->n_add++;
  if (v.empty()) return PSKV_OK;
  int rc = use_device(s);
  if (rc) return rc;
  const bool device = (flags & PSKV_DEVICE) != 0;
  if (!device && s->tune_inline) {
    uint64_t total = 0;
    for (const auto& b : v) total += b.n;
    if (total <= (uint64_t)kInlineMax * s->tune_inline_add_chunks) return inline_add(s, v);
  }
  rc = srv_stop(s);
  if (rc) return rc;
  bool host_verified = false, host_dense = false;
  std::vector<pskv_batch> framed;  // the host batches, when they are borrowed frames
  // Every exit records the frames' queued uses (pskv_host_free holds a frame
  // until they have run): a failure after some work was queued must not let
  // the frame be reused while that work still reads it.
  auto run = [&]() -> int {
    int rc = PSKV_OK;
    if (!device) {
      std::vector<pskv_batch> staged, views;
      uint64_t outside = 0;
      if ((flags & PSKV_HOST_FRAME) && frame_views(v, (size_t)s->vb, &views)) {
        framed = v;
        rc = frame_batches(s, v, views, &staged, &host_verified, &outside, &host_dense);
      } else {
        rc = stage_host_batches(s, v, &staged, &host_verified, &outside, &host_dense);
      }
      if (rc) return rc;
      // (out-of-range keys need no host step: the single workgroup that
      // inserts them reserves room on the device, ovf_reserve)
      (void)outside;
      v.swap(staged);
    }
    bool vec = true;
    for (auto& b : v) vec &= aligned16(b.keys) & aligned16(b.vals);
    for (auto& g : split_groups(v)) {
      // a replay held by the previous group goes before this group's launches
      if ((rc = flush_replay(s))) return rc;
      const uint32_t epoch = next_epoch(s);
      if (s->mode == PSKV_ACCUMULATE) {
        if (!device && host_dense) {
          // the CPU proved every batch a dense in-range window while staging it
          rc = dense_accumulate(s, v, g.first, g.second, epoch, /*verify=*/false);
        } else if (device && (flags & PSKV_SORTED_HINT)) {
          rc = dense_accumulate(s, v, g.first, g.second, epoch, /*verify=*/true);
        } else {
          // K5 (no global atomics) measured faster than K4a (LDS sums + one
          // atomic add per distinct key per chunk) on cfg 3: 322 vs 380 us per
          // 8M Zipf keys; PSKV_GENERAL=stamps selects K4a
          rc = general_add(s, v, g.first, g.second, epoch, nullptr);
        }
      } else if (!device && host_verified) {
        // the CPU proved the batches sorted and in range while staging them.
        // Sorted is not dense: a sorted batch that repeats a key and misses
        // another spans exactly n - 1 keys like a window (keys 5, 6, 6, 8), so
        // K2g's dense mode takes it and its per-element check tags it; the
        // replay then applies the group in order.  Only batches the CPU proved
        // strictly contiguous cannot trip that check and skip the replay.
        rc = sorted_add(s, v, g.first, g.second, vec, epoch, /*repair=*/!host_dense, host_dense);
      } else if (device && (flags & PSKV_SORTED_HINT)) {
        rc = sorted_add(s, v, g.first, g.second, vec, epoch, /*repair=*/true, /*maybe_windows=*/true);
      } else {
        rc = general_add(s, v, g.first, g.second, epoch, nullptr);
      }
      if (rc) return rc;
    }
    return PSKV_OK;
  };
  rc = run();
  if (!framed.empty()) {
    std::string err = rc ? g_last_error : std::string();
    const int rn = note_frame_uses(s, framed);
    if (rc) {
      g_last_error = err;  // report the first failure
      return rc;
    }
    return rn;
  }
  return rc;
}

// Zero-copy host Get of a medium batch: the keys are copied into pinned staging
// by the calling thread, K1 reads them from there and writes the values into
// pinned staging over PCIe (no DMA engine on either side), and the calling
// thread copies the values out.  The staging is default (non-coherent) pinned
// memory: the kernel's writes are visible once the stream is synchronised.
// Frames (PSKV_HOST_FRAME) skip both copies: K1 reads the keys from and
// writes the values into the caller's frames.
int zero_copy_get_views(pskv_shard* s, const std::vector<pskv_batch>& hv) {
  bool vec = true;
  for (auto& b : hv) vec &= aligned16(b.keys) & aligned16(b.vals);
  for (auto& g : split_groups(hv)) {
    GroupArgs ga;
    uint64_t elems = 0;
    for (size_t i = g.first; i < g.second; ++i) elems += hv[i].n;
    const int gu = gather_unroll(s, elems);
    const uint32_t nwg = build_group(hv, g.first, g.second, stream_chunk(gu), &ga);
    LaunchTimer t(s, PSKV_K_GATHER, elems);
    PSKV_HIP(launch_gather(s->vb, vec, gu, s->tune_nt, ga, nwg, s->dview(), s->ovf, s->stream));
    t.done();
  }
  if (int rc = wait_stream(s, s->stream, "shard stream (Get into page-locked memory)")) return rc;
  return PSKV_OK;
}

int zero_copy_get(pskv_shard* s, const std::vector<pskv_batch>& v, bool vec) {
  size_t kbytes = 0, obytes = 0;
  for (const auto& b : v) {
    kbytes += round16(b.n * 4);
    obytes += round16(b.n * (size_t)s->vb);
  }
  int rc = ensure_hstage(s, kbytes + obytes);
  if (rc) return rc;
  char* h = static_cast<char*>(s->hstage);
  std::vector<pskv_batch> hv = v;
  size_t ko = 0, oo = kbytes;
  for (size_t i = 0; i < v.size(); ++i) {
    std::memcpy(h + ko, v[i].keys, v[i].n * 4);
    hv[i].keys = reinterpret_cast<const uint32_t*>(h + ko);
    hv[i].vals = h + oo;
    ko += round16(v[i].n * 4);
    oo += round16(v[i].n * (size_t)s->vb);
  }
  for (auto& g : split_groups(hv)) {
    GroupArgs ga;
    uint64_t elems = 0;
    for (size_t i = g.first; i < g.second; ++i) elems += hv[i].n;
    const int gu = gather_unroll(s, elems);
    const uint32_t nwg = build_group(hv, g.first, g.second, stream_chunk(gu), &ga);
    LaunchTimer t(s, PSKV_K_GATHER, elems);
    const hipError_t e = launch_gather(s->vb, vec, gu, s->tune_nt, ga, nwg, s->dview(), s->ovf, s->stream);
    if (e != hipSuccess) {
      hold_hstage(s);  // earlier groups' K1 still read / write the staging
      PSKV_HIP(e);
    }
    t.done();
  }
  if (int rc = wait_stream(s, s->stream, "shard stream (zero-copy Get)")) {
    hold_hstage(s);  // its K1 may still write into the staging
    return rc;
  }
  for (size_t i = 0; i < v.size(); ++i) std::memcpy(v[i].vals, hv[i].vals, v[i].n * (size_t)s->vb);
  return PSKV_OK;
}

// Get from page-locked caller buffers by DMA: the batches go in windows of
// about kWindowBytes of keys; per window the keys are DMA'd in and K1 runs on
// the shard's stream, and the window's values are DMA'd out on a second
// stream once its K1 is done, so the values of window w travel to the host
// while the keys of window w+1 travel to the device (PCIe is full duplex; the
// two directions use different DMA engines).  The call returns when every
// value has arrived.
int pinned_get(pskv_shard* s, const std::vector<pskv_batch>& v) {
  size_t bytes = 0;
  for (auto& b : v) bytes += round16(b.n * 4) + round16(b.n * (size_t)s->vb);
  int rc = ensure_dstage(s, bytes);
  if (rc) return rc;
  if (!s->out_stream) {
    PSKV_HIP(hipStreamCreateWithFlags(&s->out_stream, hipStreamNonBlocking));
    g_queues.add_stream(s->device, 1);
  }
  std::vector<pskv_batch> dv = v;
  char* d = static_cast<char*>(s->dstage);
  size_t off = 0;
  bool vec = true;
  for (size_t i = 0; i < v.size(); ++i) {
    dv[i].keys = reinterpret_cast<const uint32_t*>(d + off);
    off += round16(v[i].n * 4);
    dv[i].vals = d + off;
    off += round16(v[i].n * (size_t)s->vb);
    vec &= aligned16(dv[i].keys) & aligned16(dv[i].vals);
  }
  // windows [first batch, end batch): >= kWindowBytes of keys, <= kMaxBatches
  // batches, < 2^32 elements (split_groups' limits for one launch)
  std::vector<std::pair<size_t, size_t>> wins;
  for (size_t i = 0; i < v.size();) {
    size_t j = i, kb = 0;
    uint64_t elems = 0;
    while (j < v.size() && (j == i || (kb < kWindowBytes && j - i < (size_t)kMaxBatches &&
                                       elems + v[j].n < (1ull << 32)))) {
      kb += v[j].n * 4;
      elems += v[j].n;
      ++j;
    }
    wins.emplace_back(i, j);
    i = j;
  }
  while (s->out_events.size() < wins.size()) {
    hipEvent_t e = nullptr;
    PSKV_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    s->out_events.push_back(e);
  }
  for (size_t w = 0; w < wins.size(); ++w) {
    const size_t b = wins[w].first, e = wins[w].second;
    for (size_t i = b; i < e; ++i)
      PSKV_HIP(hipMemcpyAsync(const_cast<uint32_t*>(dv[i].keys), v[i].keys, v[i].n * 4, hipMemcpyHostToDevice,
                              s->stream));
    GroupArgs ga;
    uint64_t elems = 0;
    for (size_t i = b; i < e; ++i) elems += dv[i].n;
    const int gu = gather_unroll(s, elems);
    const uint32_t nwg = build_group(dv, b, e, stream_chunk(gu), &ga);
    LaunchTimer t(s, PSKV_K_GATHER, elems);
    PSKV_HIP(launch_gather(s->vb, vec, gu, s->tune_nt, ga, nwg, s->dview(),
                           s->ovf, s->stream));
    t.done();
    PSKV_HIP(hipEventRecord(s->out_events[w], s->stream));
    PSKV_HIP(hipStreamWaitEvent(s->out_stream, s->out_events[w], 0));
    for (size_t i = b; i < e; ++i)
      PSKV_HIP(hipMemcpyAsync(v[i].vals, dv[i].vals, v[i].n * (size_t)s->vb, hipMemcpyDeviceToHost,
                              s->out_stream));
  }
  // the stage is free again once the out stream is done; both streams drained
  if (int rc = wait_stream(s, s->out_stream, "D2H output stream (page-locked Get)")) return rc;
  if (int rc = wait_stream(s, s->stream, "shard stream (page-locked Get)")) return rc;
  return PSKV_OK;
}

int get_impl(pskv_shard* s, const std::vector<pskv_batch>& in, int flags) {
  std::vector<pskv_batch> v;
  for (auto& b : in) {
    if (b.n == 0) continue;
    if (!b.keys || !b.vals) return fail(PSKV_EINVAL, "pskv_get: null keys/out with n > 0");
    push_pieces(v, b, (size_t)s->vb);
  }
  s->n_get++;
  if (v.empty()) return PSKV_OK;
  int rc = use_device(s);
  if (rc) return rc;
  const bool device = (flags & PSKV_DEVICE) != 0;
  if (!device && s->tune_inline) {
    uint64_t total = 0;
    for (const auto& b : v) total += b.n;
    if (total <= (uint64_t)kInlineGetMax * s->tune_inline_get_chunks) return inline_get(s, v, total);
  }
  rc = srv_stop(s);
  if (rc) return rc;
  if (!device) {  // page-locked keys and outputs (frames or not): zero copy in place
    size_t bytes = 0;
    for (auto& b : v) bytes += round16(b.n * 4) + round16(b.n * (size_t)s->vb);
    std::vector<pskv_batch> views;
    if (bytes <= s->tune_frame_zc_max_bytes &&
        (((flags & PSKV_HOST_FRAME) && frame_views(v, (size_t)s->vb, &views)) ||
         pinned_views(v, (size_t)s->vb, &views)))
      return zero_copy_get_views(s, views);
  }
  std::vector<pskv_batch> dv = v;
  size_t out_off = 0;
  bool pinned = !device;
  for (const auto& b : v) pinned = pinned && is_pinned(b.keys) && is_pinned(b.vals);
  if (!device && !pinned && s->tune_zc_max_bytes) {  // medium pageable Get: zero copy
    size_t bytes = 0;
    for (auto& b : v) bytes += round16(b.n * 4) + round16(b.n * (size_t)s->vb);
    if (bytes <= s->tune_zc_max_bytes) return zero_copy_get(s, v, true);
  }
  if (!device && !pinned && s->tune_pageable_dma) {  // pageable: direct DMA only when large
    size_t bytes = 0;
    for (auto& b : v) bytes += round16(b.n * 4) + round16(b.n * (size_t)s->vb);
    pinned = bytes >= s->tune_dma_min_bytes_get;
  }
  if (pinned) return pinned_get(s, v);
  if (!device) {
    // keys -> pinned -> device (pipelined); outputs land after the keys in the stage
    size_t kbytes = 0, obytes = 0;
    for (auto& b : v) {
      kbytes += round16(b.n * 4);
      obytes += round16(b.n * (size_t)s->vb);
    }
    rc = ensure_hstage(s, kbytes + obytes);
    if (rc) return rc;
    rc = ensure_dstage(s, kbytes + obytes);
    if (rc) return rc;
    char* h = static_cast<char*>(s->hstage);
    char* d = static_cast<char*>(s->dstage);
    std::vector<Piece> pieces;
    size_t off = 0;
    for (size_t i = 0; i < v.size(); ++i) {
      add_pieces(pieces, v[i].keys, h + off, v[i].n * 4, -1);
      dv[i].keys = reinterpret_cast<const uint32_t*>(d + off);
      off += round16(v[i].n * 4);
    }
    rc = pipelined_h2d(s, pieces, h, d);
    if (rc) return rc;
    out_off = off;
    for (size_t i = 0; i < v.size(); ++i) {
      dv[i].vals = d + off;
      off += round16(v[i].n * (size_t)s->vb);
    }
  }
  bool vec = true;
  for (auto& b : dv) vec &= aligned16(b.keys) & aligned16(b.vals);
  for (auto& g : split_groups(dv)) {
    GroupArgs ga;
    uint64_t elems = 0;
    for (size_t i = g.first; i < g.second; ++i) elems += dv[i].n;
    const int gu = gather_unroll(s, elems);
    const uint32_t nwg = build_group(dv, g.first, g.second, stream_chunk(gu), &ga);
    LaunchTimer t(s, PSKV_K_GATHER, elems);
    hipError_t e;
    if (s->pend_replay && nwg > 0) {
      // the Add's held replay rides on this first K1 (pskv_add_get_grouped);
      // it stays held (for add_get_impl's trailing K4r) unless this launch is queued
      e = launch_gather_replay(s->vb, vec, gu, s->tune_nt, ga, nwg, s->dview(), s->ovf, s->pend_rg,
                               s->flag, s->pend_epoch, s->flag + 16, s->stream);
      if (e == hipSuccess) s->pend_replay = false;
    } else {
      e = launch_gather(s->vb, vec, gu, s->tune_nt, ga, nwg, s->dview(), s->ovf, s->stream);
    }
    if (e != hipSuccess) {
      if (!device) hold_hstage(s);  // the keys' H2D from the staging is queued
      PSKV_HIP(e);
    }
    t.done();
  }
  if (!device) {
    // D2H window by window; the pool copies window w out to the caller while
    // window w+1 is still in flight
    char* h = static_cast<char*>(s->hstage);
    char* d = static_cast<char*>(s->dstage);
    std::vector<Piece> pieces;  // pinned -> caller
    size_t off = out_off;
    for (auto& b : v) {
      Piece p{};
      const size_t nb = b.n * (size_t)s->vb;
      for (size_t o = 0; o < nb; o += kPieceBytes) {
        p.src = h + off + o;
        p.dst = static_cast<char*>(b.vals) + o;
        p.bytes = std::min(kPieceBytes, nb - o);
        p.key_batch = -1;
        pieces.push_back(p);
      }
      off += round16(nb);
    }
    std::vector<std::pair<size_t, size_t>> wins;  // [first piece, end piece)
    for (size_t i = 0; i < pieces.size();) {
      size_t j = i, win = 0;
      while (j < pieces.size() && (win < kWindowBytes || j == i)) win += pieces[j++].bytes;
      wins.emplace_back(i, j);
      i = j;
    }
    while (s->win_events.size() < wins.size()) {
      hipEvent_t e = nullptr;
      PSKV_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      s->win_events.push_back(e);
    }
    for (size_t w = 0; w < wins.size(); ++w) {
      const char* lo = pieces[wins[w].first].src;
      const char* hi = pieces[wins[w].second - 1].src + pieces[wins[w].second - 1].bytes;
      hipError_t e = hipMemcpyAsync(const_cast<char*>(lo), d + (lo - h), (size_t)(hi - lo),
                                    hipMemcpyDeviceToHost, s->stream);
      if (e == hipSuccess) e = hipEventRecord(s->win_events[w], s->stream);
      if (e != hipSuccess) {
        hold_hstage(s);  // earlier windows' D2H still write into the staging
        PSKV_HIP(e);
      }
    }
    for (size_t w = 0; w < wins.size(); ++w) {
      if (int rc = wait_event(s, s->win_events[w], "D2H window event (Get to host)", s->win_events[w])) {
        hold_hstage(s);  // the queued D2H copies still write into the staging
        return rc;
      }
      run_pieces(pieces, wins[w].first, wins[w].second,
                 [&](Piece& p) { copy_piece(p, s->key_begin, s->range); });
    }
  }
  return PSKV_OK;
}

// ------------------------------------------------------------ Add then Get
// pskv_add_get_grouped: pskv_add_grouped(adds) followed by
// pskv_get_grouped(gets) in one call -- BSPModel::Clock's flush of the
// deferred Adds followed by the Gets it releases (server/consistency/
// bsp_model.cpp:14-31), or one producer round's push then pull.  Round 4
// built this as ONE fused launch (K10: the Add's and the Get's chunks as work
// units of one co-resident grid, pull keys the same call pushes answered
// from the pushed values) and measured it slower than the two launches at
// every size (headline 5.56 against 6.03 TB/s, the emulated N = 8 ranks
// 44.0-49.5 against 34.7-41.6 us; profiles/r04_probes/fused/): one register
// allocation for both halves costs the Get half of its waves, and a rank's
// fixed cost sits inside each kernel's ramp, not between the launches.  The
// kernel was removed; the call stays, as the two paths.
int add_get_impl(pskv_shard* s, const std::vector<pskv_batch>& adds, const std::vector<pskv_batch>& gets,
                 int flags) {
  // Device batches, assign, 4-byte values: the Add's last conditional replay
  // is held and rides on the Get's first K1 launch (K1r) -- one launch fewer
  // per call.  The Get's device path queues nothing before that K1; whatever
  // is still held after it (an empty Get, a failure) is launched as K4r here,
  // with nothing queued in between, so stream order is the sequential one.
  s->defer_replay = s->tune_fold_replay && (flags & PSKV_DEVICE) && s->mode == PSKV_ASSIGN && s->vb == 4;
  int rc = add_impl(s, adds, flags);
  s->defer_replay = false;
  if (!rc) rc = get_impl(s, gets, flags & ~PSKV_SORTED_HINT);
  const int rf = flush_replay(s);
  return rc ? rc : rf;
}

// ------------------------------------------------------------- options
// Every tuning knob and path selector of a shard, by name: pskv_set_option /
// pskv_get_option, and the environment variable PSKV_<NAME> as the creation
// default (the earlier interface; tests and tools now set options per shard).
// Each entry validates its value; DESIGN.md §5 says what each path is for.
struct Option {
  const char* name;
  int64_t lo, hi;  // accepted range
  int64_t (*get)(const pskv_shard*);
  void (*set)(pskv_shard*, int64_t);
};

#define PSKV_OPT(NAME, LO, HI, FIELD, T)                                           \
  Option {                                                                         \
    NAME, LO, HI, [](const pskv_shard* s) -> int64_t { return (int64_t)s->FIELD; }, \
        [](pskv_shard* s, int64_t v) { s->FIELD = (T)v; }                          \
  }

const Option kOptions[] = {
    // general (any order) Add: 0 = K4 stamps, 1 = auto (K5), 2 = K5 always;
    // the environment form also takes "stamps" / "auto" / "radix"
    PSKV_OPT("GENERAL", 0, 2, general_path, int),
    PSKV_OPT("UNROLL", 4, 8, tune_unroll, int),              // 4 or 8 (others: 8)
    PSKV_OPT("GET_UNROLL", 0, 8, tune_get_unroll, int),      // 0 (by size), 4 or 8
    PSKV_OPT("FOLD_REPLAY", 0, 1, tune_fold_replay, int),   // add_get: K4r folded into K1 (K1r)
    PSKV_OPT("NT", 0, 1, tune_nt, bool),
    PSKV_OPT("NTP", 0, 1, tune_ntp, bool),
    PSKV_OPT("EARLY", 0, 2, tune_early, int),
    PSKV_OPT("PAGEABLE_DMA", 0, 1, tune_pageable_dma, bool),
    PSKV_OPT("DMA_MIN_BYTES", 0, INT64_MAX, tune_dma_min_bytes, size_t),
    PSKV_OPT("DMA_MIN_BYTES_GET", 0, INT64_MAX, tune_dma_min_bytes_get, size_t),
    PSKV_OPT("DMA_MIN_BYTES_PINNED", 0, INT64_MAX, tune_dma_min_bytes_pinned, size_t),
    PSKV_OPT("ZC_MAX_BYTES", 0, INT64_MAX, tune_zc_max_bytes, size_t),
    PSKV_OPT("FRAME_ZC_MAX_BYTES", 0, INT64_MAX, tune_frame_zc_max_bytes, size_t),
    PSKV_OPT("INLINE", 0, 1, tune_inline, bool),
    PSKV_OPT("INLINE_ADD_CHUNKS", 1, kInlineMaxChunks, tune_inline_add_chunks, int),
    PSKV_OPT("INLINE_GET_CHUNKS", 1, kInlineMaxChunks, tune_inline_get_chunks, int),
    PSKV_OPT("ISPIN", 0, 1, tune_ispin, bool),
    PSKV_OPT("SERVE", 0, 1, tune_serve, bool),
    PSKV_OPT("SERVE_IDLE_US", 1, 10000000, tune_serve_idle_us, uint32_t),
    PSKV_OPT("TILE_SHIFT", 0, 20, tune_tile_shift, uint32_t),  // 0 = by size, else 10..20
    PSKV_OPT("TILE_GRID", 1, 65536, tune_tile_grid, uint32_t),
    PSKV_OPT("RB_WBITS", 0, 31, tune_rb_wbits, uint32_t),
    PSKV_OPT("RB_NBD", 0, kRbMaxBuckets - 1, tune_rb_nbd, uint32_t),
    PSKV_OPT("RB_TB", 0, 11, tune_rb_tb, uint32_t),
    PSKV_OPT("RB_APPLY_LOG2", 0, 14, tune_rb_apply_log2, int),  // 0 = by size, 13 or 14
    PSKV_OPT("RB_BIN_BLOCK", 512, 1024, tune_rb_bin_block, int),  // 512 or 1024
    PSKV_OPT("SYNC_TIMEOUT_MS", 0, 0x7FFFFFFF, tune_sync_timeout_ms, uint32_t),  // 0 = unbounded waits
};
#undef PSKV_OPT

const Option* find_option(const char* name) {
  for (const auto& o : kOptions)
    if (std::strcmp(o.name, name) == 0) return &o;
  return nullptr;
}

int set_option(pskv_shard* s, const Option& o, int64_t v) {
  if (v < o.lo || v > o.hi) return fail(PSKV_EINVAL, std::string("option ") + o.name + ": value out of range");
  if (std::strcmp(o.name, "UNROLL") == 0 && v != 4 && v != 8) return fail(PSKV_EINVAL, "option UNROLL: 4 or 8");
  if (std::strcmp(o.name, "GET_UNROLL") == 0 && v != 0 && v != 4 && v != 8)
    return fail(PSKV_EINVAL, "option GET_UNROLL: 0, 4 or 8");
  if (std::strcmp(o.name, "TILE_SHIFT") == 0 && v != 0 && v < 10) return fail(PSKV_EINVAL, "option TILE_SHIFT: 0 or 10..20");
  if (std::strcmp(o.name, "RB_APPLY_LOG2") == 0 && v != 0 && v != 13 && v != 14)
    return fail(PSKV_EINVAL, "option RB_APPLY_LOG2: 0, 13 or 14");
  if (std::strcmp(o.name, "RB_BIN_BLOCK") == 0 && v != 512 && v != 1024)
    return fail(PSKV_EINVAL, "option RB_BIN_BLOCK: 512 or 1024");
  o.set(s, v);
  if (std::strcmp(o.name, "SYNC_TIMEOUT_MS") == 0) refresh_grow_wait(s);
  if (std::strcmp(o.name, "INLINE_ADD_CHUNKS") == 0) s->add_chunks_set = true;
  // a ring slot costs the host ~0.2 us where a K8 launch costs 3-7: with the
  // server, Adds of up to 2 slots (512 keys) take it unless the chunk count
  // was chosen.  Measured (tools/micro/small_latency.cpp, Add then Get): 512
  // keys 17-18 us against 23-27 through the copy; from 1 Ki keys the server's
  // per-slot work (~6 us per 256-key slot) is behind the copy (1 Ki: 31-34
  // against 28)
  if (std::strcmp(o.name, "SERVE") == 0 && !s->add_chunks_set) s->tune_inline_add_chunks = v ? 2 : 1;
  return PSKV_OK;
}

// The environment only sets creation defaults: a value that does not parse or
// that pskv_set_option would reject is reported on stderr (once per variable
// and process) and ignored -- the option keeps its built-in default, and the
// shard is created as without the variable.  pskv_set_option itself stays
// strict (PSKV_EINVAL).
int apply_env_options(pskv_shard* s) {
  static std::mutex warn_mu;
  static std::vector<std::string> warned;
  // options removed after measurement: a script that still sets
  // one would otherwise measure the default path without a word
  static const char* const kRetired[] = {"RB_INSERT", "GET_DEDUP", "GET_NTP", "FUSE"};
  for (const char* name : kRetired) {
    const std::string var = std::string("PSKV_") + name;
    const char* e = std::getenv(var.c_str());
    if (!e || !*e) continue;
    std::lock_guard<std::mutex> g(warn_mu);
    if (std::find(warned.begin(), warned.end(), var) == warned.end()) {
      warned.push_back(var);
      std::fprintf(stderr, "pskv: ignoring environment %s=%s (a retired option: that path was removed)\n",
                   var.c_str(), e);
    }
  }
  for (const auto& o : kOptions) {
    const std::string var = std::string("PSKV_") + o.name;
    const char* e = std::getenv(var.c_str());
    if (!e || !*e) continue;
    int64_t v = 0;
    bool ok = true;
    if (std::strcmp(o.name, "GENERAL") == 0 && std::isalpha((unsigned char)e[0]) != 0) {
      if (std::strcmp(e, "stamps") == 0)
        v = 0;
      else if (std::strcmp(e, "auto") == 0)
        v = 1;
      else if (std::strcmp(e, "radix") == 0)
        v = 2;
      else
        ok = false;
    } else {
      char* end = nullptr;
      errno = 0;
      v = std::strtoll(e, &end, 10);
      ok = end != e && *end == '\0' && errno == 0;
    }
    const std::string saved = g_last_error;
    if (ok && set_option(s, o, v) == PSKV_OK) continue;
    const std::string why = ok ? g_last_error : std::string("not a valid value");
    g_last_error = saved;
    std::lock_guard<std::mutex> g(warn_mu);
    if (std::find(warned.begin(), warned.end(), var) == warned.end()) {
      warned.push_back(var);
      std::fprintf(stderr, "pskv: ignoring environment %s=%s (%s); the option keeps its default\n", var.c_str(), e,
                   why.c_str());
    }
  }
  return PSKV_OK;
}

}  // namespace

extern "C" {

int pskv_abi_version(void) { return PSKV_ABI_VERSION; }

const char* pskv_last_error(void) { return g_last_error.c_str(); }

int pskv_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int pskv_shard_create_ex(int device, uint32_t key_begin, uint64_t key_end, int dtype, int mode,
                         uint64_t overflow_slots, pskv_shard** out) {
  if (!out) return fail(PSKV_EINVAL, "pskv_shard_create: out is null");
  *out = nullptr;
  const int vb = value_bytes(dtype);
  if (!vb) return fail(PSKV_EINVAL, "pskv_shard_create: bad dtype");
  if (mode != PSKV_ASSIGN && mode != PSKV_ACCUMULATE)
    return fail(PSKV_EINVAL, "pskv_shard_create: bad mode");
  if (key_end <= (uint64_t)key_begin || key_end > (1ull << 32))
    return fail(PSKV_EINVAL, "pskv_shard_create: need key_begin < key_end <= 2^32");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(PSKV_EINVAL, "pskv_shard_create: no such HIP device");
  pskv_shard* s = new pskv_shard();
  s->device = device;
  s->dtype = dtype;
  s->mode = mode;
  s->vb = vb;
  s->key_begin = key_begin;
  s->range = key_end - key_begin;
  // tuning / path options: creation defaults from the environment (PSKV_<NAME>),
  // changeable later through pskv_set_option (kOptions below)
  if (int rc = apply_env_options(s)) {
    delete s;
    return rc;
  }
  auto bail = [&](int rc) {
    pskv_shard_destroy(s);
    return rc;
  };
  int rc = use_device(s);
  if (rc) return bail(rc);
  // A blocking stream: it orders against the legacy default stream, on which
  // frameworks (torch) stage device inputs and read device outputs.
  if (hipStreamCreateWithFlags(&s->own_stream, hipStreamDefault) != hipSuccess)
    return bail(fail(PSKV_EHIP, "hipStreamCreate failed"));
  s->stream = s->own_stream;
  if (hipEventCreateWithFlags(&s->hstage_free, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&s->h2d_done, hipEventDisableTiming | hipEventDisableSystemFence) !=
          hipSuccess)
    return bail(fail(PSKV_EHIP, "hipEventCreate failed"));
  if (hipMalloc(&s->dense, s->range * (size_t)vb) != hipSuccess)
    return bail(fail(PSKV_ENOMEM, "dense parameter allocation failed"));
  if (hipMemsetAsync(s->dense, 0, s->range * (size_t)vb, s->stream) != hipSuccess)
    return bail(fail(PSKV_EHIP, "hipMemsetAsync failed"));
  // flag[0]: the sorted path's verification tag
  // the verification tag (16 bytes), then K1r's replay table (add_get's folded replay)
  if (hipMalloc(&s->flag, 64 + kK1rTableWords * sizeof(uint32_t)) != hipSuccess)
    return bail(fail(PSKV_ENOMEM, "flag allocation failed"));
  if (hipMemsetAsync(s->flag, 0, 16, s->stream) != hipSuccess)
    return bail(fail(PSKV_EHIP, "hipMemsetAsync failed"));
  // the overflow table: control block, growth mailbox, first array set
  s->ocap = next_pow2(std::max<uint64_t>(overflow_slots ? overflow_slots : kDefaultOverflowSlots, 64));
  OvfCtl* ctl = nullptr;
  if (hipMalloc(&ctl, sizeof(OvfCtl)) != hipSuccess) return bail(fail(PSKV_ENOMEM, "overflow control block allocation failed"));
  s->ovf.c = ctl;
  {
    void* p = nullptr;
    if (hipHostMalloc(&p, sizeof(OvfMbox), hipHostMallocCoherent) != hipSuccess)
      return bail(fail(PSKV_ENOMEM, "overflow growth mailbox allocation failed"));
    std::memset(p, 0, sizeof(OvfMbox));
    s->mbox = static_cast<OvfMbox*>(p);
  }
  if (hipDeviceGetAttribute(&s->wall_khz, hipDeviceAttributeWallClockRate, device) != hipSuccess) s->wall_khz = 100000;
  refresh_grow_wait(s);
  rc = alloc_tab(s, s->ocap, &s->cur);
  if (rc) return bail(rc);
  OvfCtl init{};
  init.t = s->cur;
  init.mbox = s->mbox;
  if (hipMemcpyAsync(ctl, &init, sizeof(init), hipMemcpyHostToDevice, s->stream) != hipSuccess)
    return bail(fail(PSKV_EHIP, "hipMemcpyAsync failed"));
  if (int wrc = wait_stream(s, s->stream, "shard stream (creation)")) return bail(wrc);
  s->counted = g_queues.add_shard(device, 1);
  GrowService::get().add(s);
  *out = s;
  return PSKV_OK;
}

int pskv_shard_create(int device, uint32_t key_begin, uint64_t key_end, int dtype, int mode,
                      pskv_shard** out) {
  return pskv_shard_create_ex(device, key_begin, key_end, dtype, mode, 0, out);
}

int pskv_shard_destroy(pskv_shard* s) {
  if (!s) return PSKV_OK;
  (void)hipSetDevice(s->device);
  // (the grow service keeps answering while the streams drain: a growing
  // workgroup may be waiting for it)
  // every wait is bounded (PSKV_SYNC_TIMEOUT_MS): work that never completes
  // keeps its device memory, streams and shard object (leaked, never freed
  // under a running kernel), and the call reports what it waited for
  std::string stuck;
  auto drain = [&](hipStream_t st, const char* what) {
    if (wait_stream(s, st, what) != PSKV_OK) stuck += (stuck.empty() ? "" : "; ") + g_last_error;
  };
  if (s->srv) {
    (void)srv_stop(s);
    if (s->srv_running) {  // srv_stop failed: make the kernel leave anyway
      __atomic_store_n(&s->srv->stop, 1u, __ATOMIC_RELEASE);
      drain(s->srv_stream, "request-server stream (destroy)");
    }
  }
  if (s->out_stream) drain(s->out_stream, "D2H output stream (destroy)");
  if (s->own_stream) drain(s->own_stream, "shard stream (destroy)");
  if (s->stream && s->stream != s->own_stream) drain(s->stream, "caller stream (destroy)");
  if (!stuck.empty()) {
    // the leaked streams keep their hardware queues: they stay counted in
    // g_queues (pskv_queues.h), so later shards on this device do not plan
    // with queues that are still held.  The shard object itself is leaked
    // too: the grow service keeps answering its mailbox (stuck work may be a
    // workgroup waiting for it) and the service holds the pointer.
    std::fprintf(stderr, "pskv: shard destroy: %s; its device memory and streams are not freed\n", stuck.c_str());
    return fail(PSKV_ESTATE, "pskv_shard_destroy: " + stuck);
  }
  GrowService::get().remove(s);
  if (s->counted) g_queues.add_shard(s->device, -1);
  if (s->out_stream) g_queues.add_stream(s->device, -1);
  if (s->srv) (void)hipHostFree(s->srv);
  if (s->srv_stream) (void)hipStreamDestroy(s->srv_stream);
  if (s->srv_dep) (void)hipEventDestroy(s->srv_dep);
  if (s->out_stream) (void)hipStreamDestroy(s->out_stream);
  for (auto e : s->out_events) (void)hipEventDestroy(e);
  for (auto& t : s->pending) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  for (auto e : s->event_pool) (void)hipEventDestroy(e);
  if (s->sync_ev) (void)hipEventDestroy(s->sync_ev);
  if (s->dense) (void)hipFree(s->dense);
  if (s->owner) (void)hipFree(s->owner);
  if (s->flag) (void)hipFree(s->flag);
  for (const auto& t : s->tables) {  // (the service no longer touches the list)
    (void)hipFree(t.keys);
    (void)hipFree(t.vals);
  }
  if (s->ovf.c) (void)hipFree(s->ovf.c);
  if (s->mbox) (void)hipHostFree(s->mbox);
  if (s->dstage) (void)hipFree(s->dstage);
  if (s->rb_loff) (void)hipFree(s->rb_loff);
  if (s->rb_ent) (void)hipFree(s->rb_ent);
  if (s->hstage) (void)hipHostFree(s->hstage);
  if (s->ireply) (void)hipHostFree(s->ireply);
  if (s->stat_host) (void)hipHostFree(s->stat_host);
  if (s->hstage_free) (void)hipEventDestroy(s->hstage_free);
  if (s->h2d_done) (void)hipEventDestroy(s->h2d_done);
  for (auto e : s->win_events) (void)hipEventDestroy(e);
  if (s->own_stream) (void)hipStreamDestroy(s->own_stream);
  delete s;
  return PSKV_OK;
}

// Flag bits a call accepts (pskv.h): a mistyped or foreign flag fails the call
// instead of silently selecting the host path.
static bool bad_flags(int flags) {
  return (flags & ~(PSKV_DEVICE | PSKV_SORTED_HINT | PSKV_HOST_FRAME)) != 0 ||
         ((flags & PSKV_DEVICE) && (flags & PSKV_HOST_FRAME));
}

int pskv_add(pskv_shard* s, const uint32_t* keys, const void* vals, uint64_t n, int flags) {
  if (!s) return fail(PSKV_EINVAL, "pskv_add: null shard");
  if (bad_flags(flags)) return fail(PSKV_EINVAL, "pskv_add: unknown flags");
  pskv_batch b{keys, const_cast<void*>(vals), n};
  return add_impl(s, std::vector<pskv_batch>{b}, flags);
}

int pskv_get(pskv_shard* s, const uint32_t* keys, uint64_t n, void* out, int flags) {
  if (!s) return fail(PSKV_EINVAL, "pskv_get: null shard");
  if (bad_flags(flags)) return fail(PSKV_EINVAL, "pskv_get: unknown flags");
  pskv_batch b{keys, out, n};
  return get_impl(s, std::vector<pskv_batch>{b}, flags);
}

int pskv_add_grouped(pskv_shard* s, const pskv_batch* batches, uint64_t nb, int flags) {
  if (!s) return fail(PSKV_EINVAL, "pskv_add_grouped: null shard");
  if (nb && !batches) return fail(PSKV_EINVAL, "pskv_add_grouped: null batches");
  if (bad_flags(flags)) return fail(PSKV_EINVAL, "pskv_add_grouped: unknown flags");
  return add_impl(s, std::vector<pskv_batch>(batches, batches + nb), flags);
}

int pskv_add_get_grouped(pskv_shard* s, const pskv_batch* adds, uint64_t na, const pskv_batch* gets, uint64_t ng,
                         int flags) {
  if (!s) return fail(PSKV_EINVAL, "pskv_add_get_grouped: null shard");
  if ((na && !adds) || (ng && !gets)) return fail(PSKV_EINVAL, "pskv_add_get_grouped: null batches");
  if (bad_flags(flags)) return fail(PSKV_EINVAL, "pskv_add_get_grouped: unknown flags");
  return add_get_impl(s, std::vector<pskv_batch>(adds, adds + na), std::vector<pskv_batch>(gets, gets + ng), flags);
}

int pskv_get_grouped(pskv_shard* s, const pskv_batch* batches, uint64_t nb, int flags) {
  if (!s) return fail(PSKV_EINVAL, "pskv_get_grouped: null shard");
  if (nb && !batches) return fail(PSKV_EINVAL, "pskv_get_grouped: null batches");
  if (bad_flags(flags)) return fail(PSKV_EINVAL, "pskv_get_grouped: unknown flags");
  return get_impl(s, std::vector<pskv_batch>(batches, batches + nb), flags);
}

int pskv_sync(pskv_shard* s) {
  if (!s) return fail(PSKV_EINVAL, "pskv_sync: null shard");
  int rc = use_device(s);
  if (rc) return rc;
  uint32_t cnt = 0, err = 0;
  rc = read_overflow_stat(s, &cnt, &err);
  if (rc) return rc;
  rc = drain_timing(s);
  if (rc) return rc;
  if (err & kErrOverflowFull)
    return fail(PSKV_ESTATE,
                "overflow table exhausted: out-of-range keys were dropped (the device-side growth "
                "request was not answered within SYNC_TIMEOUT_MS, or its allocation failed)");
  if (2 * (uint64_t)cnt > s->ocap) return grow_overflow(s, cnt);
  return PSKV_OK;
}

int pskv_clear(pskv_shard* s) {
  if (!s) return fail(PSKV_EINVAL, "pskv_clear: null shard");
  int rc = use_device(s);
  if (rc) return rc;
  uint32_t cnt = 0, err = 0;
  rc = read_overflow_stat(s, &cnt, &err);  // (adopts the current table; stops the server)
  if (rc) return rc;
  PSKV_HIP(hipMemsetAsync(s->dense, 0, s->range * (size_t)s->vb, s->stream));
  PSKV_HIP(hipMemsetAsync(s->cur.keys, 0xFF, s->ocap * sizeof(unsigned long long), s->stream));
  PSKV_HIP(hipMemsetAsync(s->cur.vals, 0, s->ocap * (size_t)s->vb, s->stream));
  PSKV_HIP(hipMemsetAsync(s->ovf.c->stat, 0, 2 * sizeof(uint32_t), s->stream));
  s->ocount_known = 0;
  if (int rc2 = wait_stream(s, s->stream, "shard stream (clear)")) return rc2;
  return PSKV_OK;
}

int pskv_set_stream(pskv_shard* s, void* hip_stream) {
  if (!s) return fail(PSKV_EINVAL, "pskv_set_stream: null shard");
  int rc = use_device(s);
  if (rc) return rc;
  rc = srv_stop(s);
  if (rc) return rc;
  // order the switch: everything queued so far completes before the new stream's work
  if (int rc2 = wait_stream(s, s->stream, "shard stream (stream switch)")) return rc2;
  s->stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : s->own_stream;
  return PSKV_OK;
}

void* pskv_get_stream(pskv_shard* s) { return s ? static_cast<void*>(s->stream) : nullptr; }

void* pskv_dense_ptr(pskv_shard* s) { return s ? s->dense : nullptr; }

int pskv_shard_info(pskv_shard* s, pskv_info* info) {
  if (!s || !info) return fail(PSKV_EINVAL, "pskv_shard_info: null argument");
  info->device = s->device;
  info->dtype = s->dtype;
  info->mode = s->mode;
  info->value_bytes = s->vb;
  info->key_begin = s->key_begin;
  info->key_end = (uint64_t)s->key_begin + s->range;
  info->dense_bytes = s->range * (uint64_t)s->vb;
  info->overflow_capacity = s->ocap;
  info->overflow_count = s->ocount_known;
  info->n_add_calls = s->n_add;
  info->n_get_calls = s->n_get;
  info->n_sorted_launches = s->n_sorted;
  info->n_general_launches = s->n_general;
  return PSKV_OK;
}

int pskv_set_timing(pskv_shard* s, int enable) {
  if (!s) return fail(PSKV_EINVAL, "pskv_set_timing: null shard");
  s->timing_mask = enable ? (1u << PSKV_K_COUNT) - 1 : 0u;
  return PSKV_OK;
}

int pskv_set_timing_mask(pskv_shard* s, uint32_t kernel_mask) {
  if (!s) return fail(PSKV_EINVAL, "pskv_set_timing_mask: null shard");
  s->timing_mask = kernel_mask & ((1u << PSKV_K_COUNT) - 1);
  return PSKV_OK;
}

int pskv_kernel_time(pskv_shard* s, int kernel, uint64_t* launches, double* total_ms,
                     uint64_t* elements) {
  if (!s || kernel < 0 || kernel >= PSKV_K_COUNT)
    return fail(PSKV_EINVAL, "pskv_kernel_time: bad argument");
  int rc = use_device(s);
  if (rc) return rc;
  rc = drain_timing(s);
  if (rc) return rc;
  if (launches) *launches = s->t_launches[kernel];
  if (total_ms) *total_ms = s->t_ms[kernel];
  if (elements) *elements = s->t_elems[kernel];
  return PSKV_OK;
}

int pskv_reset_timing(pskv_shard* s) {
  if (!s) return fail(PSKV_EINVAL, "pskv_reset_timing: null shard");
  int rc = use_device(s);
  if (rc) return rc;
  rc = drain_timing(s);
  if (rc) return rc;
  for (int k = 0; k < PSKV_K_COUNT; ++k) {
    s->t_launches[k] = 0;
    s->t_ms[k] = 0;
    s->t_elems[k] = 0;
  }
  return PSKV_OK;
}

int pskv_set_option(pskv_shard* s, const char* name, int64_t value) {
  if (!s || !name) return fail(PSKV_EINVAL, "pskv_set_option: null argument");
  const Option* o = find_option(name);
  if (!o) return fail(PSKV_EINVAL, std::string("pskv_set_option: unknown option ") + name);
  int rc = use_device(s);
  if (rc) return rc;
  // the request server runs with the options it was launched with: drain and
  // stop it first (it restarts on the next small message if still enabled)
  rc = srv_stop(s);
  if (rc) return rc;
  return set_option(s, *o, value);
}

int pskv_get_option(pskv_shard* s, const char* name, int64_t* value) {
  if (!s || !name || !value) return fail(PSKV_EINVAL, "pskv_get_option: null argument");
  const Option* o = find_option(name);
  if (!o) return fail(PSKV_EINVAL, std::string("pskv_get_option: unknown option ") + name);
  *value = o->get(s);
  return PSKV_OK;
}

int pskv_range_slice(const uint64_t* range_begin, const uint64_t* range_end, int nranges,
                     const uint32_t* keys, uint64_t n, int32_t* slice_range,
                     uint64_t* slice_start, uint64_t* slice_len) {
  // Restates RangePartitionManager::Slice (base/range_partition_manager.hpp:19-46):
  // the range pointer only moves forward; a key stays with the current range if
  // it lies in it or the current range is the last one.
  if (n == 0) return 0;
  if (nranges <= 0 || !range_begin || !range_end || !keys || !slice_range || !slice_start ||
      !slice_len)
    return fail(PSKV_EINVAL, "pskv_range_slice: bad argument");
  int r = 0, cur = -1, ns = 0;
  for (uint64_t i = 0; i < n;) {
    const uint64_t k = keys[i];
    if ((k >= range_begin[r] && k < range_end[r]) || r + 1 >= nranges) {
      if (cur < r) {
        cur = r;
        slice_range[ns] = r;
        slice_start[ns] = i;
        slice_len[ns] = 0;
        ++ns;
      }
      slice_len[ns - 1]++;
      ++i;
    } else {
      ++r;
    }
  }
  return ns;
}

int pskv_jump_hash(const uint32_t* keys, uint64_t n, int32_t nbuckets, int32_t* out_bucket) {
  // Jump consistent hash (Lamping & Veach, "A Fast, Minimal Memory, Consistent
  // Hash Algorithm", 2014), the bucket function of the reference's default
  // partitioner ConsistentHashingPartitionManager::JumpConsistentHash
  // (base/consistent_hashing_partition_manager.hpp:81-89): a 64-bit LCG step
  // per jump, the next candidate bucket (b + 1) * 2^31 / ((state >> 33) + 1)
  // in double precision; the key enters zero-extended to 64 bits.
  if (n == 0) return PSKV_OK;
  if (nbuckets <= 0 || !keys || !out_bucket) return fail(PSKV_EINVAL, "pskv_jump_hash: bad argument");
  auto hash_range = [&](uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      uint64_t key = keys[i];
      int64_t bk = -1, j = 0;
      while (j < nbuckets) {
        bk = j;
        key = key * 2862933555777941757ULL + 1;
        j = (int64_t)((double)(bk + 1) * (double(1LL << 31) / double((key >> 33) + 1)));
      }
      out_bucket[i] = (int32_t)bk;
    }
  };
  constexpr uint64_t kPiece = 1 << 18;
  if (n <= kPiece) {
    hash_range(0, n);
  } else {
    HostPool::get().run((size_t)((n + kPiece - 1) / kPiece), [&](size_t t) {
      hash_range(t * kPiece, std::min<uint64_t>(n, (t + 1) * kPiece));
    });
  }
  return PSKV_OK;
}

int pskv_host_alloc(uint64_t bytes, void** out) {
  std::string err;
  const int rc = frames::alloc((size_t)bytes, out, &err);
  return rc ? fail(rc, err) : PSKV_OK;
}

int pskv_host_free(void* p) {
  std::string err;
  const int rc = frames::release(p, &err);
  return rc ? fail(rc, err) : PSKV_OK;
}

int pskv_host_pool_stats(uint64_t* live_bytes, uint64_t* cached_bytes, uint64_t* held_bytes) {
  frames::stats(live_bytes, cached_bytes, held_bytes);
  return PSKV_OK;
}

int pskv_host_pool_trim(void) {
  std::string err;
  const int rc = frames::trim(&err);
  return rc ? fail(rc, err) : PSKV_OK;
}

}  // extern "C"
