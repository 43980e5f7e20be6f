// k5_phases.cpp — where K5's time goes on cfg-3-shaped pushes: the shader-clock
// stamps a diagnostic build of the library records at every phase boundary of
// K5a (k_rb_bin) and K5b (k_rb_resolve), averaged over workgroups and passes.
// Keys: 8 x 1M Zipf(0.99) ranks (inverse CDF) mapped through a seeded
// permutation of [0, 1e8), as workload.zipf_batches draws them (not the same
// stream: std::mt19937_64, so statistics match, values do not).
// A second argument picks the key distribution, to tell what the hot keys of
// Zipf cost the insert phase:
//   zipf     (default) as above
//   uniform  uniform over the 1e8 keys (no hot keys, ~every key distinct)
//   matched  uniform over a pool sized so a super-chunk of 8 Ki keys holds as
//            many distinct keys as a Zipf super-chunk does (same duplicate
//            count, spread evenly: no key hotter than another)
//   bash tools/micro/build_k5_phases.sh && tools/micro/k5_phases [mode] [dist]
#include <cstring>
#include <unordered_set>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#include "pskv.h"

extern "C" int pskv_diag_k5_stamps(unsigned long long* out);

static void die(int rc, const char* what) {
  if (rc < 0) {
    std::fprintf(stderr, "%s: %d %s\n", what, rc, pskv_last_error());
    std::exit(1);
  }
}

int main(int argc, char** argv) {
  const uint64_t space = 100000000ull;
  const int J = 8, B = 1000000, reps = 6;
  const int mode = argc > 1 ? std::atoi(argv[1]) : PSKV_ASSIGN;
  const char* dist = argc > 2 ? argv[2] : "zipf";
  std::vector<double> cdf(space);
  double acc = 0;
  for (uint64_t r = 0; r < space; ++r) cdf[r] = (acc += std::pow((double)(r + 1), -0.99));
  for (auto& c : cdf) c /= acc;
  std::vector<uint32_t> perm(space);
  std::iota(perm.begin(), perm.end(), 0u);
  std::mt19937_64 rng(7);
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<std::vector<uint32_t>> keys(J, std::vector<uint32_t>(B));
  std::vector<std::vector<float>> vals(J, std::vector<float>(B));
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  for (int j = 0; j < J; ++j)
    for (int i = 0; i < B; ++i) {
      const uint64_t rank = std::min<uint64_t>(std::lower_bound(cdf.begin(), cdf.end(), u01(rng)) - cdf.begin(), space - 1);
      keys[j][i] = perm[rank];
      vals[j][i] = (float)u01(rng);
    }
  // distinct keys per 8 Ki-key super-chunk (K5a's unit for 4-byte values)
  auto distinct_per_sc = [&]() {
    double tot = 0;
    int n = 0;
    for (int j = 0; j < J; ++j)
      for (int b = 0; b + 8192 <= B; b += 8192) {
        std::unordered_set<uint32_t> u(keys[j].begin() + b, keys[j].begin() + b + 8192);
        tot += (double)u.size();
        ++n;
      }
    return tot / n;
  };
  const double zipf_distinct = distinct_per_sc();
  if (std::strcmp(dist, "uniform") == 0 || std::strcmp(dist, "matched") == 0) {
    uint64_t pool = space;
    if (dist[0] == 'm') {
      // pool S with S * (1 - exp(-8192 / S)) = the Zipf super-chunk's distinct count
      double lo = zipf_distinct, hi = 1e9;
      for (int it = 0; it < 200; ++it) {
        const double mid = 0.5 * (lo + hi);
        (mid * (1.0 - std::exp(-8192.0 / mid)) < zipf_distinct ? lo : hi) = mid;
      }
      pool = (uint64_t)std::llround(lo);
    }
    std::uniform_int_distribution<uint64_t> pick(0, pool - 1);
    for (int j = 0; j < J; ++j)
      for (int i = 0; i < B; ++i) keys[j][i] = perm[pick(rng)];
    std::printf("keys: %s (pool %llu)\n", dist, (unsigned long long)pool);
  } else if (std::strcmp(dist, "zipf") != 0) {
    std::fprintf(stderr, "dist: zipf, uniform or matched\n");
    return 2;
  }
  std::printf("distinct keys per 8 Ki-key super-chunk: %.0f (Zipf: %.0f)\n", distinct_per_sc(), zipf_distinct);
  cdf.clear();
  cdf.shrink_to_fit();
  pskv_shard* s = nullptr;
  die(pskv_shard_create(0, 0, space, PSKV_F32, mode, &s), "create");
  std::vector<pskv_batch> bs(J);
  for (int j = 0; j < J; ++j) bs[j] = pskv_batch{keys[j].data(), vals[j].data(), (uint64_t)B};
  const size_t n = 2 * 512 * 8 * 8;
  std::vector<unsigned long long> st(n), sum_a(8 * 8, 0), sum_b(8 * 8, 0);
  std::vector<unsigned long long> cnt_a(8 * 8, 0), cnt_b(8 * 8, 0);
  die(pskv_diag_k5_stamps(st.data()), "stamps");  // clear
  for (int r = 0; r < reps; ++r) {
    die(pskv_add_grouped(s, bs.data(), J, PSKV_HOST), "add");
    die(pskv_sync(s), "sync");
    die(pskv_diag_k5_stamps(st.data()), "stamps");
    if (r == 0) continue;  // warm-up
    for (int k = 0; k < 2; ++k)
      for (int wg = 0; wg < 512; ++wg)
        for (int p = 0; p < 8; ++p) {
          const unsigned long long* t = &st[((size_t)k * 512 + wg) * 64 + (size_t)p * 8];
          const unsigned long long* tn = p + 1 < 8 ? t + 8 : nullptr;
          const int nph = k == 0 ? 6 : 3;
          for (int ph = 0; ph < nph; ++ph) {
            // phase ph lasts from stamp ph to stamp ph+1 (the last one: to the
            // next pass's first stamp)
            const unsigned long long a = t[ph];
            const unsigned long long b = ph + 1 < nph ? t[ph + 1] : (tn ? tn[0] : 0ull);
            if (!a || !b || b < a) continue;
            (k == 0 ? sum_a : sum_b)[p * 8 + ph] += b - a;
            (k == 0 ? cnt_a : cnt_b)[p * 8 + ph] += 1;
          }
        }
  }
  const char* na[] = {"insert (CAS + max/add)", "keep check + bucket count", "bucket scan",
                      "row + staging", "copy-out + clear", "next pass"};
  const char* nb[] = {"run wait + totals", "direct passes", "stores + next loads"};
  std::printf("mode %s, 8 x 1M %s keys over 1e8, %d timed Adds; shader-clock cycles per phase\n",
              mode == PSKV_ASSIGN ? "assign" : "accumulate", dist, reps - 1);
  for (int k = 0; k < 2; ++k) {
    std::printf("%s\n", k == 0 ? "K5a k_rb_bin (per super-chunk pass)" : "K5b k_rb_resolve (per bucket)");
    const int nph = k == 0 ? 5 : 3;
    for (int ph = 0; ph < nph; ++ph) {
      unsigned long long tot = 0, c = 0;
      for (int p = 0; p < 8; ++p) {
        tot += (k == 0 ? sum_a : sum_b)[p * 8 + ph];
        c += (k == 0 ? cnt_a : cnt_b)[p * 8 + ph];
      }
      std::printf("  %-28s %10.0f cycles  (n=%llu)\n", k == 0 ? na[ph] : nb[ph], c ? (double)tot / c : 0.0, c);
    }
  }
  die(pskv_shard_destroy(s), "destroy");
  pskv_host_pool_trim();
  return 0;
}
