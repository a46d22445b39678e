"""Per-dispatch PMC averages of one kernel from rocprofv3 csv passes
(counter_collection.csv + kernel_trace.csv under DIR/p*/), with the held
clock GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md, DVFS give-back).

    python tools/pmc_clock_summary.py KERNEL_SUBSTRING DIR
"""
import collections
import csv
import glob
import os
import sys


def main():
    kern, root = sys.argv[1], sys.argv[2]
    tot = collections.defaultdict(float)
    cnt = collections.defaultdict(set)
    durs = []
    names = set()
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            if kern not in row["Kernel_Name"]:
                continue
            names.add(row["Kernel_Name"][:90])
            c = row["Counter_Name"]
            tot[(f, c)] += float(row["Counter_Value"])
            cnt[(f, c)].add(row["Dispatch_Id"])
    for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            if kern in row["Kernel_Name"]:
                durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    per = {}
    for (f, c), v in tot.items():
        per.setdefault(c, []).append(v / len(cnt[(f, c)]))
    print("kernels:", sorted(names))
    avg = {c: sum(v) / len(v) for c, v in per.items()}
    for c in sorted(avg):
        print(f"{c:28s} per dispatch {avg[c]:.4e}")
    if durs:
        d = sum(durs) / len(durs)
        print(f"duration (kernel trace, {len(durs)} dispatches) {d / 1e6:.3f} ms")
        if "GRBM_GUI_ACTIVE" in avg:
            print(f"held clock GRBM_GUI_ACTIVE / 8 / duration = {avg['GRBM_GUI_ACTIVE'] / 8 / d:.3f} GHz")


if __name__ == "__main__":
    main()
