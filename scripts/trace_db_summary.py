#!/usr/bin/env python3
"""Per-(kernel, grid) summary of a rocprofv3 --kernel-trace SQLite output (run_results.db):
launches, average / total duration, and the average gap between consecutive dispatches.
usage: trace_db_summary.py <run_results.db> [top]"""
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = db.execute("select name, grid_x, grid_y, workgroup_x, start, end from kernels order by start").fetchall()
agg = {}
for name, gx, gy, wx, s, e in rows:
    short = re.sub(r"\(.*$", "", name)
    short = short.replace("(anonymous namespace)::", "")
    key = (short[:70], gx // max(wx, 1), gy)
    a = agg.setdefault(key, [0, 0.0])
    a[0] += 1
    a[1] += (e - s) / 1e3
busy = sum(v[1] for v in agg.values())
span = (rows[-1][5] - rows[0][4]) / 1e3 if rows else 0.0
print(f"{len(rows)} dispatches, busy {busy:.1f} us over span {span:.1f} us")
print(f"{'kernel':70s} {'wgs':>6s} {'gy':>4s} {'n':>6s} {'avg_us':>8s} {'total_us':>10s}")
for (k, g, gy), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{k:70s} {g:6d} {gy:4d} {n:6d} {t / n:8.2f} {t:10.1f}")
