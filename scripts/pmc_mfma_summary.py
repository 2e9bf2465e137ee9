#!/usr/bin/env python3
"""Reduce a rocprofv3 --pmc counter_collection.csv (SQ MFMA / LDS / GRBM counters) to per-kernel
utilisation figures.

    python scripts/pmc_mfma_summary.py gpurun_out/r2_pmc_sq/run_counter_collection.csv > profiles/r2_pmc_mfma.json

Per kernel (averaged over its dispatches):
* eff_clock_ghz       = GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time (MI355X_MICROARCH.md, DVFS give-back)
* mfma_busy_frac      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): share of SIMD cycles
                        the matrix pipe was busy (1.0 = MFMA-bound at the clock held)
* mfma_tflops         = SQ_INSTS_VALU_MFMA_MOPS_F16 x 512 FLOP / wall time (MOPS counts 512-FLOP units)
* lds_conflict_frac   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import collections
import csv
import json
import sys

SIMDS = 1024
XCDS = 8


def main(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    wall = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        wall[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = []
    for k, c in agg.items():
        n = len(wall[k])
        t = sum(wall[k].values()) / n
        if c.get("SQ_INSTS_MFMA", 0) == 0 and "knn" not in k:
            continue
        g = c.get("GRBM_GUI_ACTIVE", 0) / n
        row = {"kernel": k[:120], "dispatches": n, "avg_wall_ms": round(t * 1e3, 4)}
        if g and t > 0:
            row["eff_clock_ghz"] = round(g / XCDS / t / 1e9, 3)
            row["mfma_busy_frac"] = round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / n / (SIMDS * g / XCDS), 4)
        mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0) / n
        if mops and t > 0:
            row["mfma_tflops"] = round(mops * 512 / t / 1e12, 1)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
        row["counters_per_dispatch"] = {kk: round(v / n) for kk, v in sorted(c.items())}
        out.append(row)
    out.sort(key=lambda r: -r["avg_wall_ms"] * r["dispatches"])
    json.dump({"source": path, "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
