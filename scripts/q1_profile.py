#!/usr/bin/env python3
"""One query per search (the reference's call pattern) over a 1M x 512 shard, for a kernel trace:
rocprofv3 --kernel-trace --output-format csv -d OUT -o q1 -- python3 scripts/q1_profile.py
then scripts/q1_profile.py --trace OUT/.../q1_kernel_trace.csv prints the per-search timeline
(each kernel's mean duration and the idle gap before it)."""
import csv
import json
import os
import sys
import time

if len(sys.argv) > 2 and sys.argv[1] == "--trace":
    rows = list(csv.DictReader(open(sys.argv[2])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last 100 searches: prep -> scan -> merge, grouped by the scan launches
    scans = [i for i, r in enumerate(rows) if "knn_scan3_kernel" in r["Kernel_Name"] and ", 0, " in r["Kernel_Name"]]
    seq = {}
    for si in scans[-100:]:
        lo = si - 1
        while lo > 0 and "prep_rows" not in rows[lo]["Kernel_Name"]:
            lo -= 1
        hi = si + 1
        while hi < len(rows) and "prep_rows" not in rows[hi]["Kernel_Name"]:
            hi += 1
        for j in range(lo, hi):
            r = rows[j]
            name = r["Kernel_Name"].split("((")[0][-60:]
            gap = int(r["Start_Timestamp"]) - int(rows[j - 1]["End_Timestamp"]) if j > lo else 0
            d = seq.setdefault((j - lo, name), [0, 0.0, 0.0])
            d[0] += 1
            d[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            d[2] += gap / 1e3
    for (pos, name), (n, dur, gap) in sorted(seq.items()):
        print(json.dumps({"pos": pos, "kernel": name, "n": n, "us": round(dur / n, 2), "gap_before_us": round(gap / n, 2)}))
    sys.exit(0)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
import torch  # noqa: E402

from app.vector_store import FlatIndex  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(7)
x = torch.randn((1 << 20, 512), generator=g, device=dev)
ix = FlatIndex(512)
ix.add(x)
del x
q = torch.randn((int(os.environ.get("NQ", "1")), 512), generator=g, device=dev)
s = torch.cuda.Stream(device=dev)
with torch.cuda.stream(s):
    for _ in range(20):
        ix.search(q, 10)
    s.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        ix.search(q, 10)
    s.synchronize()
print(json.dumps({"ms_per_search": round((time.perf_counter() - t0) / 200 * 1e3, 4)}), flush=True)
