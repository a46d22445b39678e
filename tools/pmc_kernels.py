"""Per-kernel HBM counters + durations from separate rocprofv3 passes.

    rocprofv3 --kernel-trace --output-format csv -d D/trace -o run -- CMD
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d D/fetch -o run -- CMD
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d D/write -o run -- CMD
    python tools/pmc_kernels.py D [--match SUBSTR ...] [--fetch-scale 2] > out.json

Per kernel name (one instantiation each): dispatches, mean duration (us, from
the kernel trace), mean FETCH_SIZE / WRITE_SIZE per dispatch in bytes and
the fetch bytes times --fetch-scale (gfx950 reports half the bytes of
coalesced streaming reads: MI355X_MICROARCH.md, HBM section; calibrate with
a kernel whose bytes are known, e.g. colsum_kernel reading the matrix once),
and the resulting GB/s.  Memory-side counters include Infinity-Cache hits.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def rows(root, pattern):
    out = []
    for f in glob.glob(os.path.join(root, "**", pattern), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--match", nargs="*", default=None)
    ap.add_argument("--fetch-scale", type=float, default=2.0)
    a = ap.parse_args()
    dur = defaultdict(list)
    for r in rows(os.path.join(a.root, "trace"), "*kernel_trace.csv"):
        dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for sub in ("fetch", "write"):
        for r in rows(os.path.join(a.root, sub), "*counter_collection.csv"):
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            ctr[r["Kernel_Name"]][r["Counter_Name"]][key] += float(r["Counter_Value"])
    out = []
    for name in sorted(set(dur) | set(ctr)):
        if a.match and not any(m in name for m in a.match):
            continue
        d = dur.get(name, [])
        rec = {"kernel": name[:160], "dispatches": len(d),
               "mean_us": round(sum(d) / len(d) / 1e3, 3) if d else None}
        for c, scale in (("FETCH_SIZE", a.fetch_scale), ("WRITE_SIZE", 1.0)):
            v = ctr[name].get(c)
            if v:
                kib = sum(v.values()) / len(v)
                rec[c.lower() + "_bytes_raw"] = round(kib * 1024)
                rec[c.lower().split("_")[0] + "_bytes"] = round(kib * 1024 * scale)
        if rec["mean_us"] and "fetch_bytes" in rec:
            tot = rec["fetch_bytes"] + rec.get("write_bytes", 0)
            rec["GBps"] = round(tot / (rec["mean_us"] * 1e3), 1)
        out.append(rec)
    print(json.dumps({"fetch_scale": a.fetch_scale, "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
