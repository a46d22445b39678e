"""HBM traffic per launch of the dominant kernel from rocprofv3 --pmc runs.

    python tools/traffic_from_pmc.py <pmc_dir_root> <kernel-substring> \
        <population> <d> <out.json>

The substring must select ONE instantiation (rocprofv3 reports this kernel
by its mangled name: "mvn_x3_kernelILi3ELi8ELb0E" is the main c3 launch,
"mvn_x3_kernelILi3ELi8ELb1E" the small unhinted rescue pass, ~1% of the
bytes): dispatches are grouped by their full kernel name and
the tool refuses a substring that matches more than one name, so launches of
different shapes are never averaged together.  Only dispatches at least 10%
of the largest matching one's FETCH_SIZE are kept (the same instantiation
also runs small rescue subsets).

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


def collect(root, pat):
    by_name = defaultdict(lambda: defaultdict(dict))   # name -> counter -> dispatch -> v
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"),
                       recursive=True):
        for r in csv.DictReader(open(f)):
            c = r["Counter_Name"]
            if pat in r["Kernel_Name"] and c in ("FETCH_SIZE", "WRITE_SIZE"):
                key = (f, r.get("Dispatch_Id") or r.get("Correlation_Id"))
                by_name[r["Kernel_Name"]][c][key] = (
                    by_name[r["Kernel_Name"]][c].get(key, 0.0) + float(r["Counter_Value"]))
    return by_name


def main():
    root, pat, pop, d, out = sys.argv[1:6]
    by_name = collect(root, pat)
    if len(by_name) != 1:
        sys.exit(f"substring {pat!r} matches {len(by_name)} kernel names: "
                 + "; ".join(n[:120] for n in by_name))
    name, vals = next(iter(by_name.items()))
    res = {"kernel": pat, "kernel_name": name[:200], "population": int(pop),
           "candidates": int(pop), "d": int(d), "fetch_correction": 2.0}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        v = list(vals[c].values())
        big = [x for x in v if x >= 0.1 * max(v)]
        res[c.lower() + "_kib"] = sum(big) / len(big)
        res[c.lower() + "_dispatches"] = len(big)
        res[c.lower() + "_dispatches_dropped"] = len(v) - len(big)
    res["traffic_bytes"] = 2.0 * res["fetch_size_kib"] * 1024 + res["write_size_kib"] * 1024
    res["note"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate runs; "
                   "one kernel instantiation; FETCH doubled (gfx950 16 B/lane "
                   "streaming-read correction); includes Infinity-Cache hits")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
