"""Per-generation GPU timeline from a rocprofv3 kernel trace.

    python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv [anchor]

Windows are delimited by the anchor kernel (default mvn_x3_kernel): for each
window, wall time, kernel count, busy time; then the kernel mix and the
largest idle gaps of the last window.
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "mvn_x3_kernel"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for a, b in zip(idx[:-1], idx[1:]):
        seg = rows[a + 1:b]
        t0, t1 = int(rows[a]["End_Timestamp"]), int(rows[b]["Start_Timestamp"])
        busy = sum(dur(r) for r in seg)
        print(f"window {(t1 - t0) / 1e6:.3f} ms, kernels {len(seg)}, "
              f"busy {busy / 1e6:.3f} ms, anchor {dur(rows[b]) / 1e6:.3f} ms")
    a, b = idx[-2], idx[-1]
    agg = defaultdict(lambda: [0, 0])
    prev = int(rows[a]["End_Timestamp"])
    gaps = []
    for r in rows[a + 1:b]:
        gaps.append((int(r["Start_Timestamp"]) - prev, r["Kernel_Name"][:50]))
        prev = int(r["End_Timestamp"])
        k = r["Kernel_Name"][:60]
        agg[k][0] += 1
        agg[k][1] += dur(r)
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{v[0]:4d} {v[1] / 1e3:9.1f} us  {k}")
    gaps.sort(reverse=True)
    print("sum gaps %.1f us; largest:" % (sum(g for g, _ in gaps) / 1e3),
          [(round(g / 1e3, 1), n) for g, n in gaps[:12]])


if __name__ == "__main__":
    main()
