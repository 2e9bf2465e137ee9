#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv: per kernel calls, total ms, average us and
share, optionally divided by a step count (per-step us).
    python scripts/kstats.py KERNEL_STATS_CSV [steps]"""
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.3f} ms over {sum(int(r['Calls']) for r in rows)} launches")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    t = float(r["TotalDurationNs"])
    line = f"{r['Name'][:70]:70s} calls {int(r['Calls']):6d} total {t / 1e6:8.3f} ms avg {float(r['AverageNs']) / 1e3:8.2f} us {100 * t / tot:5.1f} %"
    if steps:
        line += f"  per step {t / 1e3 / steps:8.1f} us"
    print(line)
