"""Per-kernel summary of a rocprofv3 results database (rocpd sqlite, the default output format of rocprofv3 7.x):
name, calls, total / average microseconds, share of the summed kernel time, optionally restricted to the last
--last dispatches (the timed steps).  Usage: python tools/kt_summary.py RESULTS.db [--last N] [--by-grid]"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--by-grid", action="store_true", help="split each kernel by grid size")
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, start from kernels order by start").fetchall()
    if args.last:
        rows = rows[-args.last:]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, dur, gx, gy, gz, _ in rows:
        key = name.split("(")[0][:60] + (f" grid={gx}x{gy}x{gz}" if args.by_grid else "")
        agg[key][0] += 1
        agg[key][1] += dur
    tot = sum(v[1] for v in agg.values())
    span = (rows[-1][5] - rows[0][5]) if rows else 0
    print(f"{len(rows)} dispatches, kernel time {tot / 1e3:.1f} us, span {span / 1e3:.1f} us")
    for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{d / tot * 100:6.2f}%  {n:5d}  {d / 1e3:10.1f} us  {d / n / 1e3:8.2f} us/call  {k}")


if __name__ == "__main__":
    main()
