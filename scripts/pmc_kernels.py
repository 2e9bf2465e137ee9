#!/usr/bin/env python3
"""Merge rocprofv3 --pmc passes (one counter_collection.csv per pass) into per-kernel rows.

    python scripts/pmc_kernels.py OUT.json PASS_DIR [PASS_DIR ...]

Counters are averaged per dispatch within each pass (a kernel's dispatches differ between passes
only in which counters were read), then merged by kernel name. Derived, per kernel:
* eff_clock_ghz     = GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall (MI355X_MICROARCH.md, DVFS give-back)
* mfma_busy_frac    = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
* wait_any_frac     = SQ_WAIT_ANY / SQ_WAVE_CYCLES (both quad-cycles, per wave)
* wait_inst_any_frac, wait_inst_lds_frac, active_{vmem,lds,valu,sca,misc}_frac: the same over SQ_WAVE_CYCLES
* lds_busy_frac     = SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM_GUI_ACTIVE / 8)
* lds_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS, CUS, XCDS = 1024, 256, 8


def read_pass(d):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not path:
        return {}
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    wall = collections.defaultdict(dict)
    for r in csv.DictReader(open(path[0])):
        k = r["Kernel_Name"]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        wall[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k, c in agg.items():
        n = len(wall[k])
        out[k] = {"n": n, "wall": sum(wall[k].values()) / n, "c": {kk: v / n for kk, v in c.items()}}
    return out


def main(out_path, dirs):
    merged = {}
    for d in dirs:
        for k, v in read_pass(d).items():
            m = merged.setdefault(k, {"dispatches": {}, "walls": [], "c": {}})
            m["dispatches"][d] = v["n"]
            m["walls"].append(v["wall"])
            m["c"].update(v["c"])
    rows = []
    for k, m in merged.items():
        c, t = m["c"], sum(m["walls"]) / len(m["walls"])
        g = c.get("GRBM_GUI_ACTIVE")
        wc = c.get("SQ_WAVE_CYCLES")
        row = {"kernel": k[:140], "dispatches_per_pass": m["dispatches"], "avg_wall_ms": round(t * 1e3, 4)}
        if g and t > 0:
            row["eff_clock_ghz"] = round(g / XCDS / t / 1e9, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                row["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * g / XCDS), 4)
            if "SQ_LDS_IDX_ACTIVE" in c:
                row["lds_busy_frac"] = round(c["SQ_LDS_IDX_ACTIVE"] / (CUS * g / XCDS), 4)
        if wc:
            for name, key in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_any_frac"),
                              ("SQ_WAIT_INST_LDS", "wait_inst_lds_frac"), ("SQ_ACTIVE_INST_ANY", "active_any_frac"),
                              ("SQ_ACTIVE_INST_VMEM", "active_vmem_frac"), ("SQ_ACTIVE_INST_LDS", "active_lds_frac"),
                              ("SQ_ACTIVE_INST_VALU", "active_valu_frac"), ("SQ_ACTIVE_INST_SCA", "active_sca_frac"),
                              ("SQ_ACTIVE_INST_MISC", "active_misc_frac")):
                if name in c:
                    row[key] = round(c[name] / wc, 4)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
        if c.get("SQ_INSTS_VALU_MFMA_MOPS_F16") and t > 0:
            row["mfma_tflops"] = round(c["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512 / t / 1e12, 1)
        row["counters_per_dispatch"] = {kk: round(v) for kk, v in sorted(c.items())}
        rows.append(row)
    rows.sort(key=lambda r: -r["avg_wall_ms"] * max(r["dispatches_per_pass"].values()))
    with open(out_path, "w") as f:
        json.dump({"passes": dirs, "kernels": rows}, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
