#!/bin/bash
# Round 4, session 19: vector-memory path counters (TA / TD / TCP) of K3d qkv vs the isolated
# LDS-DMA stream (bench_micro/fill_rate), one --pmc pass per block group (within the per-block
# limits: <= 2 TA, <= 2 TD, <= 4 TCP, <= 2 GRBM counters).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $R/gpurun_out/r4s19_avail.txt 2>&1 || true
grep -oE "\b(TA|TD|TCP)_[A-Z0-9_]+" $R/gpurun_out/r4s19_avail.txt | sort -u > $R/gpurun_out/r4s19_names.txt
P1="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
P2="TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
P3="TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  for c in $P; do b=${c%_sum}; grep -qx "$b" $R/gpurun_out/r4s19_names.txt || [ "${b#GRBM}" != "$b" ] || { echo "counter $b not listed, skipping pass $i"; continue 2; }; done
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/r4s19_g$i -o run -- python3 $R/scripts/gemm_bench.py qkv > $R/gpurun_out/r4s19_g$i.log 2>&1 || { echo "gemm pass $i failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/r4s19_f$i -o run -- $R/bench_micro/fill_rate 1 > $R/gpurun_out/r4s19_f$i.log 2>&1 || { echo "fill pass $i failed"; exit 2; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for tag, pat in (("gemm", "gpurun_out/r4s19_g*"), ("fill", "gpurun_out/r4s19_f*")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{pat}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:50]
            if ("gemm_8p" in k) or ("fill_kernel<0, 8>" in k):
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(tag, k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
find gpurun_out/r4s19_* -name "*.csv" -size +5M -delete
