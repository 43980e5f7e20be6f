"""Estimated N-GPU aggregate from ranks emulated one at a time on one GPU.

Each emulated rank (bench.py under PSKV_BENCH_EMULATE=r/N) runs rank r's share
of the N-GPU cfg-4 workload alone and reports its own step time and bytes.
The N ranks run independently (no collective on the data path), so the N-GPU
step takes the slowest rank's time, and the aggregate is all ranks' bytes over
it — the same formula bench.py applies to a real N-GPU run (max over ranks of
the timed region, sum of the bytes).  Compared with the N = 1 value of the same
head (a bench.py JSON line).

  python tools/emu_summary.py N1.json emu_rank0.json ... emu_rank{N-1}.json
"""
import json
import sys


def main():
    n1 = json.load(open(sys.argv[1]))
    ranks = [json.load(open(p)) for p in sys.argv[2:]]
    ms = [r["ms_per_step"] for r in ranks]
    bytes_ = [r["config"]["bytes_per_step_per_gpu"] for r in ranks]
    agg = sum(bytes_) / (max(ms) * 1e-3) / 1e9
    out = {
        "n_ranks": len(ranks),
        "rank_ms_per_step": ms,
        "rank_GB/s": [b / (m * 1e-3) / 1e9 for b, m in zip(bytes_, ms)],
        "rank_bytes_per_step": bytes_,
        "slowest_rank": ms.index(max(ms)),
        "estimated_aggregate_GB/s": agg,
        "n1_value_GB/s": n1["value"],
        "estimated_speedup_vs_n1": agg / n1["value"],
        "imbalance_max_over_mean_bytes": max(bytes_) / (sum(bytes_) / len(bytes_)),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
