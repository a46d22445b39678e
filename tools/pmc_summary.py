"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch).

    python tools/pmc_summary.py gpurun_out/pmc [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"),
                              recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if pat and pat not in k:
                continue
            vals[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:34s} {sum(v) / len(v):16.4g}   (n={len(v)})")


if __name__ == "__main__":
    main()
