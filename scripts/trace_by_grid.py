#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace CSV split by launch grid, so launches of one
kernel instance at different shapes (the 1M x 512 and 512k x 512 K7 scans share a template
instance) are separate rows: calls, average / min / max us, total ms, share.
    python scripts/trace_by_grid.py KERNEL_TRACE_CSV [top]"""
import collections
import csv
import re
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
agg = collections.defaultdict(list)
with open(path) as f:
    for r in csv.DictReader(f):
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))[:60]
        grid = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in agg.values())
print(f"total {tot / 1e3:.3f} ms over {sum(len(v) for v in agg.values())} dispatches")
for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    g = "x".join(str(x) for x in grid)
    print(f"{name:60s} grid {g:>14s} calls {len(v):5d} avg {sum(v) / len(v):9.2f} us "
          f"min {min(v):9.2f} max {max(v):9.2f} total {sum(v) / 1e3:8.3f} ms {100 * sum(v) / tot:5.1f} %")
