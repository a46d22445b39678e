"""Host gaps of one generation from a rocprofv3 kernel + HIP API trace.

    rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d D -o run \
        -- python3 bench.py --pop 100000 --steps 3 --warmup 2 --no-cpu-baseline
    python tools/host_gaps.py D [--gen -1] [--min-us 20]

Generations are delimited by the hinted x3 density launches (one per
generation, mvn_x3_kernel<..., false>); --gen picks one (default: the last
complete window).  Every idle stretch of the GPU longer than --min-us
between two kernels of that window is listed with the HIP calls the host
made inside it: a blocking call (hipMemcpy*/hipStreamSynchronize/...)
names a host sync; a stretch with only launches or no call at all is Python
time between launches.  The launch-to-start delay of the kernel after the
gap tells whether the GPU waited for the host (the launch came after the
previous kernel ended).
"""
import argparse
import csv
import glob
import os
from collections import defaultdict

SYNC = ("hipMemcpy", "hipStreamSynchronize", "hipDeviceSynchronize",
        "hipEventSynchronize", "hipMemcpyDtoH", "hipStreamWaitEvent",
        "hipHostMalloc", "hipMalloc", "hipFree")


def load(root, pattern):
    fs = glob.glob(os.path.join(root, "**", pattern), recursive=True)
    rows = []
    for f in fs:
        rows += list(csv.DictReader(open(f)))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--gen", type=int, default=-1)
    ap.add_argument("--min-us", type=float, default=20.0)
    ap.add_argument("--anchor", default="mvn_x3_kernel")
    a = ap.parse_args()
    ks = load(a.root, "*kernel_trace.csv")
    api = load(a.root, "*hip_api_trace.csv")
    for r in ks:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ks.sort(key=lambda r: r["s"])
    for r in api:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    api.sort(key=lambda r: r["s"])
    launch = {r["Correlation_Id"]: r for r in api}
    anch = [i for i, r in enumerate(ks)
            if a.anchor in r["Kernel_Name"] and "Lb0E" in r["Kernel_Name"]]
    if len(anch) < 2:
        anch = [i for i, r in enumerate(ks) if a.anchor in r["Kernel_Name"]]
    wins = list(zip(anch[:-1], anch[1:]))
    i0, i1 = wins[a.gen]
    win = ks[i0:i1]
    t0, t1 = win[0]["s"], win[-1]["s"]
    busy = sum(r["e"] - r["s"] for r in win)
    print(f"window: kernels {len(win)} (from the x3 launch to the next), "
          f"wall {(t1 - t0) / 1e6:.3f} ms, kernel busy {busy / 1e6:.3f} ms")
    gaps = []
    prev_end = win[0]["e"]
    for r in win[1:]:
        g = r["s"] - max(prev_end, 0)
        if g > a.min_us * 1e3:
            calls = [c for c in api if prev_end <= c["s"] < r["s"]]
            names = defaultdict(lambda: [0, 0])
            for c in calls:
                names[c["Function"]][0] += 1
                names[c["Function"]][1] += c["e"] - c["s"]
            lc = launch.get(r["Correlation_Id"])
            late = (lc["s"] - prev_end) / 1e3 if lc else float("nan")
            syncs = [n for n in names if n.startswith(SYNC)]
            gaps.append((g, r["Kernel_Name"][:70], late, syncs, dict(names)))
        prev_end = max(prev_end, r["e"])
    tot = sum(g for g, *_ in gaps)
    print(f"gaps > {a.min_us} us: {len(gaps)}, total {tot / 1e3:.1f} us")
    for g, name, late, syncs, names in gaps:
        kind = ("host sync: " + ", ".join(syncs)) if syncs else "python between launches"
        top = sorted(names.items(), key=lambda kv: -kv[1][1])[:4]
        print(f"  {g / 1e3:8.1f} us before {name}")
        print(f"           launch issued {late:.1f} us after the previous kernel ended; {kind}")
        if top:
            print("           calls: " + "; ".join(f"{n} x{c} {d / 1e3:.1f} us"
                                             for n, (c, d) in top))
    agg = defaultdict(lambda: [0, 0])
    for r in win:
        agg[r["Kernel_Name"][:60]][0] += 1
        agg[r["Kernel_Name"][:60]][1] += r["e"] - r["s"]
    print("kernels of the window by time:")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"  {v[0]:4d} {v[1] / 1e3:9.1f} us  {k}")


if __name__ == "__main__":
    main()
