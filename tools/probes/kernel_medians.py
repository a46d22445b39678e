"""Median duration per (kernel, grid) from a rocprofv3 --kernel-trace csv
directory (probe helper):  python tools/probes/kernel_medians.py DIR [substr ...]"""
import collections
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    keys = sys.argv[2:]
    path = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if keys and not any(k in name for k in keys):
            continue
        per[(name[:90], r["Grid_Size_X"])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(per.items()):
        v = sorted(v)
        print(f"  {k[0]:90s} grid {k[1]:>8s}: median {v[len(v) // 2]:8.2f} us  "
              f"p10 {v[len(v) // 10]:8.2f}  n {len(v)}")
    # gaps between consecutive kernels of the listed names (launch gaps)
    ts = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:30])
                for r in rows if not keys or any(k in r["Kernel_Name"] for k in keys))
    gaps = [(ts[i + 1][0] - ts[i][1]) / 1e3 for i in range(len(ts) - 1)]
    if gaps:
        g = sorted(gaps)
        print(f"  gaps between listed kernels: median {g[len(g) // 2]:.2f} us, p10 {g[len(g) // 10]:.2f}")


if __name__ == "__main__":
    main()
