"""Median duration of every template instance of the K5 / K1 kernels in a
rocprofv3 SQLite output (run_results.db), e.g. to split K5a / K5b by mode:
  python tools/ktrace_split.py gpurun_out/x/run_results.db [name-regex]"""
import re
import sqlite3
import statistics
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_rb_bin|k_rb_resolve|k_gather")
    rows = c.execute("select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    by = {}
    for n, dur in rows:
        m = re.search(r"(k_\w+?)I(\w+?)EEEv", n)
        if not m or not pat.search(m.group(1)):
            continue
        by.setdefault(f"{m.group(1)}<{m.group(2)}>", []).append(dur / 1e3)
    for k, ds in sorted(by.items()):
        print(f"{k[:48]:48s} n={len(ds):3d} median {statistics.median(ds):8.1f} us  min {min(ds):8.1f}")


if __name__ == "__main__":
    main()
