"""Per-kernel duration summary from a rocprofv3 SQLite output (rocpd tables):
  python tools/kstats.py gpurun_out/x/run_results.db [name-regex]"""
import collections
import re
import sqlite3
import statistics
import sys


def _short(name):
    """'void pskv::(anon)::k_rb_apply<float, float, 1>(...)' -> 'k_rb_apply<float, float, 1>'."""
    m = re.search(r"(k_[a-z_0-9]+(<[^()]*>)?)", name)
    if m:
        return m.group(1)[:90]
    return re.sub(r"\(.*", "", name)[:90]


def main():
    c = sqlite3.connect(sys.argv[1])
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    rows = c.execute("select s.kernel_name, d.end - d.start, d.grid_size_x, d.workgroup_size_x, "
                     "s.arch_vgpr_count, s.sgpr_count, d.group_segment_size "
                     "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    by = collections.defaultdict(list)
    meta = {}
    for name, dur, gx, wx, vg, sg, lds in rows:
        short = _short(name)
        if pat and not pat.search(name):
            continue
        by[short].append(dur / 1e3)
        meta[short] = (gx // max(wx, 1), wx, vg, sg, lds)
    tot = sum(sum(v) for v in by.values())
    print(f"{'kernel':90s} {'calls':>6s} {'avg_us':>9s} {'med_us':>9s} {'pct':>6s}  grid/wg/vgpr/sgpr/lds")
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:90s} {len(v):6d} {statistics.mean(v):9.2f} {statistics.median(v):9.2f} "
              f"{100 * sum(v) / tot:6.1f}  {meta[k]}")


if __name__ == "__main__":
    main()
