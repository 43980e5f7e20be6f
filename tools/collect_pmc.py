"""Summarise rocprofv3 PMC passes into profiles/pmc_latest.json.

Usage (on the GPU box, two SEPARATE counter runs, as MI355X_MICROARCH.md's
HBM section prescribes):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d D -o fetch -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d D -o write -- python3 bench.py ...
  python tools/collect_pmc.py D/fetch_counter_collection.csv D/write_counter_collection.csv OUT.json

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half
the bytes of a wide (16 B/lane) coalesced stream, so it is doubled; WRITE_SIZE
is exact for 16-B-per-lane stores.  Both counters are in KiB.  Infinity-Cache
hits are counted as fetches, so with a working set above 256 MiB (bench.py's)
the figure approximates HBM traffic.
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def per_dispatch(path, counter):
    vals = defaultdict(dict)  # kernel -> dispatch -> value
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            vals[r["Kernel_Name"]][r["Dispatch_Id"]] = vals[r["Kernel_Name"]].get(r["Dispatch_Id"], 0.0) + \
                float(r["Counter_Value"])
    return vals


def short(name):
    for k in ("k_gather", "k_assign_group", "k_assign_sorted", "k_general_mark",
              "k_general_commit", "k_replay", "k_rb_bin", "k_rb_resolve"):
        if k in name:
            return k + name[name.index(k) + len(k):].split("(")[0]
    return None


def main():
    fetch_csv, write_csv, out = sys.argv[1:4]
    # the bench configuration profiled (bench.py uses the traffic only for the same one)
    config = json.loads(sys.argv[4]) if len(sys.argv) > 4 else {"n_gpus": 1, "batches": 64, "batch_keys": 1000000,
                                                                "sets": 16, "form": "pull-free-slots"}
    fe = per_dispatch(fetch_csv, "FETCH_SIZE")
    wr = per_dispatch(write_csv, "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of bench.py; "
                     "traffic = (2*FETCH_SIZE + WRITE_SIZE) KiB per dispatch, median over dispatches",
           "config": config, "kernels": {}}
    for name in set(fe) | set(wr):
        s = short(name)
        if not s:
            continue
        f = statistics.median(fe.get(name, {}).values()) if fe.get(name) else None
        w = statistics.median(wr.get(name, {}).values()) if wr.get(name) else None
        rec = {"fetch_kib_raw": f, "write_kib": w, "dispatches": len(fe.get(name, {}))}
        if f is not None and w is not None:
            rec["hbm_bytes_per_dispatch"] = (2 * f + w) * 1024
        key = s
        res["kernels"][key] = rec
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
