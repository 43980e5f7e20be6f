// pskv_queues.h — per-device hardware-queue accounting of the request server
// (K9).  Host-only, no HIP types: pskv_shard.cpp uses one process-wide
// instance, tests/cpp/queue_accounting_test.cpp (a CPU test) its own.
//
// A resident K9 server holds the hardware queue its stream maps to; work of any
// other stream of the process on that queue waits behind it until it idles
// out.  HIP gives a process GPU_MAX_HW_QUEUES queues PER DEVICE (default 4) and
// deals that device's streams to them round-robin.  On a device, every shard
// holds one stream (its own, or the caller's), a served shard a second (the
// server's), a shard that ran a page-locked Get one more (its D2H stream), and
// the null stream takes one: the server engages on a device only while
//   2 * shards(device) + 1 + extra_streams(device) <= GPU_MAX_HW_QUEUES,
// so it then holds a queue of its own.  Shards on OTHER devices do not count:
// each device has its own queues (driver/engine.hpp:98-110 puts server thread i
// on device i % ndev through include/ps/storage_factory.hpp).
#pragma once
#include <atomic>
#include <cstdlib>

namespace pskv {

constexpr int kMaxDevices = 64;

// GPU_MAX_HW_QUEUES as HIP reads it: the runtime accepts 1..32 and treats
// anything else (unset, empty, non-numeric, < 1 or > 32) as its default 4.
inline int hw_queues_from_env(const char* v) {
  if (!v || !*v) return 4;
  char* end = nullptr;
  const long q = std::strtol(v, &end, 10);
  if (end == v || *end != '\0' || q < 1 || q > 32) return 4;
  return static_cast<int>(q);
}

class DeviceQueues {
 public:
  // a shard was created / destroyed on `device` (false: device out of range)
  bool add_shard(int device, int delta) {
    if (device < 0 || device >= kMaxDevices) return false;
    shards_[device].fetch_add(delta, std::memory_order_relaxed);
    return true;
  }
  // a shard on `device` created / destroyed an extra stream (page-locked Get output)
  bool add_stream(int device, int delta) {
    if (device < 0 || device >= kMaxDevices) return false;
    extra_[device].fetch_add(delta, std::memory_order_relaxed);
    return true;
  }
  int shards(int device) const {
    return device < 0 || device >= kMaxDevices ? 0 : shards_[device].load(std::memory_order_relaxed);
  }
  int streams(int device) const {
    return device < 0 || device >= kMaxDevices ? 0 : extra_[device].load(std::memory_order_relaxed);
  }
  // may a shard on `device` run the resident request server?
  bool serve_fits(int device, int hw_queues) const {
    if (device < 0 || device >= kMaxDevices) return false;
    return 2 * shards(device) + 1 + streams(device) <= hw_queues;
  }

 private:
  std::atomic<int> shards_[kMaxDevices] = {};
  std::atomic<int> extra_[kMaxDevices] = {};
};

}  // namespace pskv
