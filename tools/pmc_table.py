"""Median per-dispatch PMC values per kernel from rocprofv3 --pmc CSV files:
  python tools/pmc_table.py DIR/*_counter_collection.csv [--match k_rb]"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    pat = None
    if "--match" in sys.argv:
        pat = re.compile(sys.argv[sys.argv.index("--match") + 1])
        args = [a for a in args if a != sys.argv[sys.argv.index("--match") + 1]]
    vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for path in args:
        with open(path) as f:
            for r in csv.DictReader(f):
                m = re.search(r"(k_[a-z_0-9]+(<[^()]*>)?)", r["Kernel_Name"])
                name = m.group(1) if m else r["Kernel_Name"][:60]
                if pat and not pat.search(name):
                    continue
                vals[name][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, cs in sorted(vals.items()):
        print(k)
        for c, d in sorted(cs.items()):
            print(f"    {c:28s} {statistics.median(d.values()):16.1f}  (n={len(d)})")


if __name__ == "__main__":
    main()
