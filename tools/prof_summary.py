"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite, ROCm 7 default output) per kernel and launch shape.

usage: python tools/prof_summary.py <results.db> [--like PATTERN] [--by-shape]
Prints: kernel name, grid (work-items), launches, average / min duration in microseconds, total.
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--like", default="%")
    ap.add_argument("--by-shape", action="store_true")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    key = "name, grid_x, grid_y, grid_z" if a.by_shape else "name"
    q = (f"select name, grid_x, grid_y, grid_z, count(*), avg(end-start)/1e3, min(end-start)/1e3, sum(end-start)/1e3 "
         f"from kernels where name like ? group by {key} order by sum(end-start) desc limit ?")
    rows = list(c.execute(q, (a.like, a.top)))
    total = sum(r[7] for r in rows)
    print(f"{'kernel':70s} {'grid':>18s} {'n':>6s} {'avg_us':>9s} {'min_us':>9s} {'total_us':>10s} {'pct':>6s}")
    for name, gx, gy, gz, n, avg, mn, tot in rows:
        grid = f"{gx}x{gy}x{gz}" if a.by_shape else "-"
        print(f"{name[:70]:70s} {grid:>18s} {n:6d} {avg:9.1f} {mn:9.1f} {tot:10.1f} {100 * tot / total:6.1f}")


if __name__ == "__main__":
    main()
