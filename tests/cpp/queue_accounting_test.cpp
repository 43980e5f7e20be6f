// CPU unit test of the request server's per-device hardware-queue accounting
// (parameter_server_amd/csrc/pskv_queues.h).  The reference runs
// N server threads per node, each with its own storage
// (driver/simple_id_mapper.cpp:28-31, driver/engine.hpp:98-110); CreateTable
// puts server i on device i % ndev (include/ps/storage_factory.hpp).  Each
// device has its own GPU_MAX_HW_QUEUES queues, so the server may engage on one
// device while it cannot on another.  Host-only: no HIP, no GPU.
#include <cstdio>
#include <initializer_list>

#include "pskv_queues.h"

static int failed = 0, passed = 0;
#define EXPECT(c)                                                      \
  do {                                                                 \
    if (c) {                                                           \
      ++passed;                                                        \
    } else {                                                           \
      ++failed;                                                        \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);          \
    }                                                                  \
  } while (0)

int main() {
  using pskv::DeviceQueues;
  using pskv::hw_queues_from_env;
  // GPU_MAX_HW_QUEUES parsing (HIP's default 4)
  EXPECT(hw_queues_from_env(nullptr) == 4);
  EXPECT(hw_queues_from_env("") == 4);
  EXPECT(hw_queues_from_env("abc") == 4);
  EXPECT(hw_queues_from_env("0") == 4);
  EXPECT(hw_queues_from_env("-3") == 4);
  EXPECT(hw_queues_from_env("8x") == 4);
  EXPECT(hw_queues_from_env("8") == 8);
  EXPECT(hw_queues_from_env("32") == 32);
  // beyond the runtime's range (1..32) HIP keeps its default, and so do we
  EXPECT(hw_queues_from_env("33") == 4);
  EXPECT(hw_queues_from_env("64") == 4);
  EXPECT(hw_queues_from_env("1024") == 4);
  EXPECT(hw_queues_from_env("1") == 1);
  {
    // one shard on a device, default 4 queues: 2*1 + 1 = 3 <= 4 -> serves
    DeviceQueues q;
    EXPECT(q.add_shard(0, 1));
    EXPECT(q.serve_fits(0, 4));
    // a second shard on the same device: 2*2 + 1 = 5 > 4 -> K8 launches instead
    EXPECT(q.add_shard(0, 1));
    EXPECT(!q.serve_fits(0, 4));
    EXPECT(q.serve_fits(0, 5));  // GPU_MAX_HW_QUEUES=5 makes room
    // a page-locked Get's D2H stream counts against its device
    EXPECT(q.add_stream(0, 1));
    EXPECT(!q.serve_fits(0, 5));
    EXPECT(q.serve_fits(0, 6));
    // destroying a shard and its stream gives the queues back
    EXPECT(q.add_shard(0, -1));
    EXPECT(q.add_stream(0, -1));
    EXPECT(q.serve_fits(0, 4));
  }
  {
    // 8 server threads per node, CreateTable's device binding i % ndev
    for (int ndev : {1, 2, 4, 8}) {
      DeviceQueues q;
      for (int i = 0; i < 8; ++i) EXPECT(q.add_shard(i % ndev, 1));
      const int per = 8 / ndev;
      for (int d = 0; d < ndev; ++d) {
        EXPECT(q.shards(d) == per);
        // per device 2 * per + 1 <= 4 only with one shard per device
        EXPECT(q.serve_fits(d, 4) == (per == 1));
        EXPECT(q.serve_fits(d, 2 * per + 1));
        EXPECT(!q.serve_fits(d, 2 * per));
      }
      // devices without shards are untouched by the others' counts
      for (int d = ndev; d < 8; ++d) EXPECT(q.shards(d) == 0 && q.serve_fits(d, 4));
    }
  }
  {
    // extra streams on one device never affect another
    DeviceQueues q;
    q.add_shard(3, 1);
    q.add_shard(5, 1);
    q.add_stream(3, 2);
    EXPECT(!q.serve_fits(3, 4));
    EXPECT(q.serve_fits(5, 4));
  }
  {
    // out-of-range device ids are refused, never indexed
    DeviceQueues q;
    EXPECT(!q.add_shard(-1, 1));
    EXPECT(!q.add_shard(pskv::kMaxDevices, 1));
    EXPECT(!q.add_stream(pskv::kMaxDevices + 7, 1));
    EXPECT(!q.serve_fits(pskv::kMaxDevices, 1024));
    EXPECT(q.shards(-5) == 0 && q.streams(pskv::kMaxDevices) == 0);
  }
  std::printf("queue_accounting_test: %d passed, %d failed\n", passed, failed);
  return failed ? 1 : 0;
}
