"""HBM traffic per launch of the dominant kernel from rocprofv3 --pmc runs.

    python tools/traffic_from_pmc.py <pmc_dir_root> <kernel-substring> \
        <population> <d> <out.json>

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of
16-B-per-lane streaming reads (the x3 kernel's fragment loads are 16 B per
lane), so it is doubled; WRITE_SIZE is taken as is.  Memory-side counters
include Infinity-Cache hits, so this is an upper bound on HBM bytes.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root, pat, pop, d, out = sys.argv[1:6]
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"),
                       recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"] and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
    write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
    res = {"kernel": pat, "population": int(pop), "candidates": int(pop),
           "d": int(d), "fetch_size_kib": fetch, "write_size_kib": write,
           "fetch_correction": 2.0,
           "traffic_bytes": 2.0 * fetch * 1024 + write * 1024,
           "dispatches": len(vals["FETCH_SIZE"]),
           "note": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate "
                   "runs of `bench.py --steps 3 --warmup 1`; FETCH doubled "
                   "(gfx950 16 B/lane streaming-read correction); includes "
                   "Infinity-Cache hits"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
