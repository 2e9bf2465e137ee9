#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for v in -1 0 2; do
MRAG_GEMM_BIG=$v timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_big$v.log 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc_gemm1 -o run -- python3 $R/scripts/gemm_bench.py fc1 > $R/gpurun_out/pmc_gemm1.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmc_gemm2 -o run -- python3 $R/scripts/gemm_bench.py fc1 > $R/gpurun_out/pmc_gemm2.log 2>&1 || exit 4
