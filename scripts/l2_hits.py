#!/usr/bin/env python3
"""Per-kernel L2 (TCC) hit rate and fetched bytes from rocprofv3 --pmc passes (separate runs:
TCC_HIT_sum + TCC_MISS_sum, and FETCH_SIZE), averaged per dispatch.
    python scripts/l2_hits.py HITS_DIR FETCH_DIR [kernel substrings...]"""
import collections
import csv
import glob
import sys


def load(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


hits, fetch = load(sys.argv[1]), load(sys.argv[2])
needles = sys.argv[3:] or ["gemm"]
for k in sorted(set(hits) | set(fetch)):
    if not any(n in k for n in needles):
        continue
    h = hits.get(k, {})
    hm = sum(h.get("TCC_HIT_sum", [0])) / max(1, len(h.get("TCC_HIT_sum", [1])))
    mm = sum(h.get("TCC_MISS_sum", [0])) / max(1, len(h.get("TCC_MISS_sum", [1])))
    fs = fetch.get(k, {}).get("FETCH_SIZE", [])
    fb = 2 * 1024 * sum(fs) / len(fs) if fs else None  # gfx950: FETCH_SIZE counts half of wide streaming reads
    print(f"{k:70s} dispatches {len(h.get('TCC_HIT_sum', []))} hit_rate {hm / max(1, hm + mm):.3f} "
          f"req/dispatch {hm + mm:.3e} fetched_MB/dispatch {fb / 1e6 if fb else float('nan'):.1f}")
