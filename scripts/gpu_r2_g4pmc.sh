#!/bin/bash
# K3e vs K3d counters on qkv / sq4k: L2 request traffic and MFMA / wait cycles
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  MRAG_GEMM_4W=$v timeout -s KILL 90 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d $R/gpurun_out/r2_g4pmc_l2_$v -o run -- python3 $R/scripts/gemm_bench.py qkv sq4k > $R/gpurun_out/r2_g4pmc_l2_$v.log 2>&1 || exit 1
  MRAG_GEMM_4W=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/r2_g4pmc_sq_$v -o run -- python3 $R/scripts/gemm_bench.py qkv sq4k > $R/gpurun_out/r2_g4pmc_sq_$v.log 2>&1 || exit 2
  MRAG_GEMM_4W=$v timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/r2_g4pmc_ta_$v -o run -- python3 $R/scripts/gemm_bench.py qkv sq4k > $R/gpurun_out/r2_g4pmc_ta_$v.log 2>&1 || exit 3
done
