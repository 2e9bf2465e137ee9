#!/usr/bin/env python3
"""Per-kernel summary from a rocprofv3 rocpd database (the default output of --kernel-trace):
kernel (short name) x grid size -> calls, total and average us, optionally per step.
    python scripts/rocpd_kernels.py RESULTS.db [steps] [top]"""
import collections
import re
import sqlite3
import sys

db = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
c = sqlite3.connect(db)
agg = collections.defaultdict(lambda: [0, 0.0])
for name, dur, gx in c.execute("select name, duration, grid_x from kernels"):
    short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))[:60]
    key = (short, gx)
    agg[key][0] += 1
    agg[key][1] += dur / 1e3
tot = sum(v[1] for v in agg.values())
print(f"total {tot / 1e3:.3f} ms, {sum(v[0] for v in agg.values())} dispatches")
for (k, gx), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    line = f"{k:60s} grid {gx:8d} calls {n:5d} avg {t / n:8.1f} us total {t / 1e3:8.3f} ms {100 * t / tot:5.1f} %"
    if steps:
        line += f" per-step {t / steps:8.1f} us"
    print(line)
