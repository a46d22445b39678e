"""Per-kernel PMC totals from rocprofv3 rocpd databases (one per --pmc pass),
normalised per dispatch and per work item.

    python tools/pmc_summary.py KERNEL_SUBSTRING DB [DB ...] [--per N]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--per", type=float, default=None,
                    help="work items per dispatch (e.g. candidates) to normalise by")
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    meta = {}
    for db in a.dbs:
        con = sqlite3.connect(db)
        for name, cname, val, did, vg, avg, sg, lds, dur in con.execute(
                "select kernel_name, counter_name, value, dispatch_id, vgpr_count, "
                "accum_vgpr_count, sgpr_count, lds_block_size, duration from counters_collection"):
            if a.kernel not in name:
                continue
            tot[cname] += val
            disp[cname].add((db, did))
            meta = dict(kernel=name[:120], vgpr=vg, agpr=avg, sgpr=sg, lds=lds)
    print(meta)
    for c in sorted(tot):
        n = len(disp[c])
        line = f"{c:28s} total {tot[c]:.4e}  per dispatch {tot[c] / n:.4e}"
        if a.per:
            line += f"  per item {tot[c] / n / a.per:.4g}"
        print(line)


if __name__ == "__main__":
    main()
