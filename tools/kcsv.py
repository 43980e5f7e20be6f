"""Print pskv kernel rows of a rocprofv3 --stats kernel_stats.csv: name, calls, avg/min us.
  python tools/kcsv.py gpurun_out/x/zt_kernel_stats.csv"""
import csv
import re
import sys

for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_[a-z_0-9]+<[^()]*>)", r["Name"])
    if m and "pskv" in r["Name"]:
        print(f"{m.group(1):55s} {r['Calls']:>5} {float(r['AverageNs']) / 1e3:9.2f} {float(r['MinNs']) / 1e3:9.2f}")
