"""Kernel statistics from a rocprofv3 rocpd database (run_results.db):
per kernel name, calls, total / average / min / max duration (ns) and the
share of the summed kernel time, like --stats' kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/prof1/run_results.db [--csv out.csv]
"""
import argparse
import csv
import sqlite3
import sys


def table(con, prefix):
    for (name,) in con.execute("select name from sqlite_master where type='table'"):
        if name.startswith(prefix):
            return name
    raise KeyError(prefix)


def stats(db):
    con = sqlite3.connect(db)
    kd = table(con, "rocpd_kernel_dispatch")
    ks = table(con, "rocpd_info_kernel_symbol")
    cols = [r[1] for r in con.execute(f"pragma table_info({ks})")]
    name_col = "display_name" if "display_name" in cols else "kernel_name"
    rows = con.execute(
        f"select s.{name_col}, count(*), sum(d.end - d.start), min(d.end - d.start), "
        f"max(d.end - d.start), min(d.start), max(d.end) from {kd} d join {ks} s "
        f"on d.kernel_id = s.id group by s.{name_col} order by 3 desc").fetchall()
    span = con.execute(f"select min(start), max(end) from {kd}").fetchone()
    return rows, span


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    a = ap.parse_args()
    rows, span = stats(a.db)
    tot = sum(r[2] for r in rows)
    out = [("Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage")]
    for n, c, t, mn, mx, _, _ in rows:
        out.append((n, c, t, t / c, mn, mx, 100.0 * t / tot))
    w = csv.writer(open(a.csv, "w") if a.csv else sys.stdout)
    w.writerows(out)
    print(f"# kernel time {tot/1e9:.3f} s over a dispatch span of "
          f"{(span[1]-span[0])/1e9:.3f} s", file=sys.stderr)


if __name__ == "__main__":
    main()
