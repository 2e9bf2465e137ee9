#!/bin/bash
# PMC: K7 v3 vs v4 (wait / LDS / MFMA busy)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
for v in 0 1; do
MRAG_SCAN_V4=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/r2_v4pmc_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-clip --no-fusion > $R/gpurun_out/r2_v4pmc_$v.log 2>&1 || exit 1
done
