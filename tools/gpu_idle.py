"""GPU idle share of a rocprofv3 kernel trace (rocpd database): the union of
kernel execution intervals against the span from the first to the last
dispatch, overall and inside a window (e.g. the bench's timed region, from
the first candidate-round kernel of generation `--skip` on).

    python tools/gpu_idle.py gpurun_out/prof/run_results.db [--after-kernel fused_round --skip N]
    python tools/gpu_idle.py gpurun_out/prof/run_kernel_trace.csv [...]   (csv output)
"""
import argparse
import csv
import sqlite3


def table(con, prefix):
    for (name,) in con.execute("select name from sqlite_master where type='table'"):
        if name.startswith(prefix):
            return name
    raise KeyError(prefix)


def busy(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--after-kernel", default=None,
                    help="start the window at the --skip-th dispatch of this kernel")
    ap.add_argument("--skip", type=int, default=0)
    a = ap.parse_args()
    if a.db.endswith(".csv"):
        with open(a.db) as f:
            rows = sorted((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                          for r in csv.DictReader(f))
        rows.sort(key=lambda r: r[1])
    else:
        con = sqlite3.connect(a.db)
        kd, ks = table(con, "rocpd_kernel_dispatch"), table(con, "rocpd_info_kernel_symbol")
        cols = [r[1] for r in con.execute(f"pragma table_info({ks})")]
        nc = "display_name" if "display_name" in cols else "kernel_name"
        rows = con.execute(f"select s.{nc}, d.start, d.end from {kd} d join {ks} s "
                           f"on d.kernel_id = s.id order by d.start").fetchall()
    t0 = rows[0][1]
    if a.after_kernel:
        hits = [r for r in rows if a.after_kernel in r[0]]
        t0 = hits[a.skip][1]
    iv = [(s, e) for _, s, e in rows if s >= t0]
    span = max(e for _, e in iv) - t0
    b = busy(iv)
    print(f"window {span / 1e9:.3f} s, kernels busy {b / 1e9:.3f} s, "
          f"idle {100 * (1 - b / span):.2f} %  ({len(iv)} dispatches)")


if __name__ == "__main__":
    main()
