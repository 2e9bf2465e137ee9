#!/bin/bash
# Round 3, session 21: counters on this tree. K7 HBM traffic (FETCH_SIZE / WRITE_SIZE in separate
# passes + a kernel-trace pass, reduced by scripts/pmc_summary.py into profiles/knn_scan_pmc.json)
# and the four SQ passes over the whole bench (scripts/pmc_kernels.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
KNN="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-clip --no-fusion --no-call-pattern --knn-streams 1"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- $KNN > $R/gpurun_out/r3s21_fetch.log 2>&1 || exit 11
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- $KNN > $R/gpurun_out/r3s21_write.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o run -- python3 $R/bench.py --steps 20 --no-cpu-baseline --no-clip --no-fusion --no-call-pattern --knn-streams 1 > $R/gpurun_out/r3s21_stats.log 2>&1 || exit 13
cd $R
f=$(find gpurun_out/prof_fetch -name "*counter_collection.csv" | head -1); [ "$f" = gpurun_out/prof_fetch/run_counter_collection.csv ] || cp "$f" gpurun_out/prof_fetch/run_counter_collection.csv
f=$(find gpurun_out/prof_write -name "*counter_collection.csv" | head -1); [ "$f" = gpurun_out/prof_write/run_counter_collection.csv ] || cp "$f" gpurun_out/prof_write/run_counter_collection.csv
f=$(find gpurun_out/prof_stats -name "*kernel_stats.csv" | head -1); [ "$f" = gpurun_out/prof_stats/run_kernel_stats.csv ] || cp "$f" gpurun_out/prof_stats/run_kernel_stats.csv
python3 scripts/pmc_summary.py "knn_scan3_kernel<512, 0, 4>" gpurun_out/knn_scan_pmc.json 1074765824 || exit 14
find gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/prof_stats -name "*trace*.csv" -delete
cd /tmp
CMD="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --knn-streams 1"
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
P3="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_VALU"
P4="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/r3pmc_p$i -o run -- $CMD > $R/gpurun_out/r3pmc_p$i.log 2>&1 || exit $((20+i))
done
cd $R && python3 scripts/pmc_kernels.py gpurun_out/r3s2_pmc_kernels.json gpurun_out/r3pmc_p1 gpurun_out/r3pmc_p2 gpurun_out/r3pmc_p3 gpurun_out/r3pmc_p4 || exit 30
rm -rf gpurun_out/r3pmc_p1 gpurun_out/r3pmc_p2 gpurun_out/r3pmc_p3 gpurun_out/r3pmc_p4
cat gpurun_out/knn_scan_pmc.json; du -sh gpurun_out
