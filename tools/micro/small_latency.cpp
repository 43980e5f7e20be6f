// small_latency.cpp — per-call latency of small host messages through the C ABI
// (the reference's live traffic: one LR sample's keys per message,
// app/logistic_regression.cpp:411,490).  Compares the K8 inline path (keys and
// values in the kernel arguments, reply written to page-locked memory and
// published by a polled sequence word) with the same path waiting on the stream
// (PSKV_ISPIN=0) and with the staged path (PSKV_INLINE=0: H2D / D2H DMAs).
// The last two variants take the message from page-locked pool frames
// (pskv_host_alloc): "pinned" passes them as plain host memory (direct DMA),
// "frames" under PSKV_HOST_FRAME (read and written in place).
// "serve": the defaults with the K9 request server (PSKV_SERVE=1) in place of
// the K8 launches.
//   g++ -O2 -std=c++11 -I include tools/micro/small_latency.cpp \
//       -L parameter_server_amd -lpskv -Wl,-rpath,$PWD/parameter_server_amd -o /tmp/small_latency
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "pskv.h"

static double now_us() {
  using namespace std::chrono;
  return duration<double, std::micro>(steady_clock::now().time_since_epoch()).count();
}

static void die(int rc, const char* what) {
  if (rc) {
    std::fprintf(stderr, "%s: %d %s\n", what, rc, pskv_last_error());
    std::exit(1);
  }
}

int main() {
  const int sizes[] = {1, 16, 64, 256, 512, 1024, 2048, 4096, 16384, 65536, 262144, 1048576, 4194304};
  const int reps = 600;
  std::mt19937 rng(7);
  {  // the CPU side of a frame: the mailbox's receive copy into one, and reads of it
    const size_t nb = 1 << 20;
    std::vector<char> a(nb, 1), b(nb, 2);
    void* f = nullptr;
    die(pskv_host_alloc(nb, &f), "host_alloc");
    char* fp = static_cast<char*>(f);
    std::memset(fp, 3, nb);
    auto rate = [&](char* dst, const char* src) {
      std::vector<double> t;
      for (int r = 0; r < 50; ++r) {
        const double t0 = now_us();
        std::memcpy(dst, src, nb);
        t.push_back(now_us() - t0);
      }
      std::nth_element(t.begin(), t.begin() + t.size() / 2, t.end());
      return t[t.size() / 2];
    };
    const double hh = rate(b.data(), a.data()), hf = rate(fp, a.data()), fh = rate(b.data(), fp);
    std::printf("memcpy 1 MiB: heap->heap %.1f us, heap->frame %.1f us, frame->heap %.1f us\n", hh, hf, fh);
    die(pskv_host_free(f), "host_free");
  }
  std::printf("%-10s %6s %10s %10s %12s %12s\n", "path", "keys", "add_us", "get_us", "add+get_us",
              "get_only_us");
  // variants: the defaults (inline small messages, pinned staging copy for
  // medium ones, direct DMA of pageable buffers from PSKV_DMA_MIN_BYTES on);
  // inline Gets waiting on the stream (PSKV_ISPIN=0); no inline path with
  // every pageable buffer DMA'd directly; no inline path with every pageable
  // buffer copied into pinned staging
  // and the defaults with medium Gets zero-copy (PSKV_ZC_MAX_BYTES = 4 MiB)
  const char* names[] = {"default", "inline-sync", "dma-always", "copy-always", "zero-copy", "pinned", "frames",
                         "serve"};
  constexpr int kVariants = 8;
  for (int pass = 0; pass < 2; ++pass)  // pass 0 warms the runtime up (its pageable-copy paths); pass 1 prints
  for (int var = 0; var < kVariants; ++var) {
    // SL_VARIANTS="0,6": only those variants (quicker A/B runs)
    if (const char* only = std::getenv("SL_VARIANTS")) {
      const std::string list = std::string(",") + only + ",";
      if (list.find("," + std::to_string(var) + ",") == std::string::npos) continue;
    }
    const bool framed = var == 5 || var == 6;
    setenv("PSKV_SERVE", var == 7 ? "1" : "0", 1);  // K9: the resident request server
    const int flags = var == 6 ? PSKV_HOST | PSKV_HOST_FRAME : PSKV_HOST;
    if (var == 4)
      setenv("PSKV_ZC_MAX_BYTES", "4194304", 1);
    else
      unsetenv("PSKV_ZC_MAX_BYTES");
    setenv("PSKV_INLINE", (var < 2 || var >= 4) ? "1" : "0", 1);
    setenv("PSKV_ISPIN", var != 1 ? "1" : "0", 1);
    const char* th = var == 2 ? "0" : var == 3 ? "1000000000000" : nullptr;  // nullptr: library defaults
    if (th) {
      setenv("PSKV_DMA_MIN_BYTES", th, 1);
      setenv("PSKV_DMA_MIN_BYTES_GET", th, 1);
    } else {
      unsetenv("PSKV_DMA_MIN_BYTES");
      unsetenv("PSKV_DMA_MIN_BYTES_GET");
    }
    pskv_shard* s = nullptr;
    die(pskv_shard_create(0, 0, 1000000, PSKV_F64, PSKV_ASSIGN, &s), "create");
    for (int n : sizes) {
      std::vector<uint32_t> kv(framed ? 0 : n);
      std::vector<double> vv(framed ? 0 : n), ov(framed ? 0 : n);
      uint32_t* k = kv.data();
      double *v = vv.data(), *out = ov.data();
      void *fk = nullptr, *fv = nullptr, *fo = nullptr;
      if (framed) {
        die(pskv_host_alloc(n * 4ull, &fk), "host_alloc");
        die(pskv_host_alloc(n * 8ull, &fv), "host_alloc");
        die(pskv_host_alloc(n * 8ull, &fo), "host_alloc");
        k = static_cast<uint32_t*>(fk);
        v = static_cast<double*>(fv);
        out = static_cast<double*>(fo);
      }
      std::vector<double> ta, tg, tb, to;
      const int nrep = std::max(20, std::min(reps, (int)((1 << 22) / n)));
      for (int r = 0; r < nrep + 10; ++r) {
        for (int i = 0; i < n; ++i) {
          k[i] = rng() % 1000000;
          v[i] = (double)r + i;
        }
        std::sort(k, k + n);  // LR pushes [0] + sorted feature ids
        const double t0 = now_us();
        die(pskv_add(s, k, v, n, flags), "add");
        const double t1 = now_us();
        die(pskv_get(s, k, n, out, flags), "get");  // also: the Add has run before k, v are rewritten
        const double t2 = now_us();
        die(pskv_get(s, k, n, out, flags), "get");  // nothing queued before it
        const double t3 = now_us();
        if (r >= 10) {
          ta.push_back(t1 - t0);
          tg.push_back(t2 - t1);
          tb.push_back(t2 - t0);
          to.push_back(t3 - t2);
        }
        for (int i = 0; i < n; ++i)  // read-your-writes (last duplicate wins)
          if (i + 1 == n || k[i] != k[i + 1])
            if (out[i] != v[i]) {
              std::fprintf(stderr, "mismatch at %d\n", i);
              return 1;
            }
      }
      auto med = [](std::vector<double>& x) {
        std::nth_element(x.begin(), x.begin() + x.size() / 2, x.end());
        return x[x.size() / 2];
      };
      if (pass == 1)
        std::printf("%-10s %6d %10.2f %10.2f %12.2f %12.2f\n", names[var], n, med(ta), med(tg), med(tb),
                    med(to));
      if (framed) {
        die(pskv_host_free(fk), "host_free");
        die(pskv_host_free(fv), "host_free");
        die(pskv_host_free(fo), "host_free");
      }
    }
    die(pskv_shard_destroy(s), "destroy");
  }
  return 0;
}
