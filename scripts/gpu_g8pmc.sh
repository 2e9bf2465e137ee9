#!/bin/bash
# K3d PMC passes on the 4096^3 shape (and qkv): wave-state and LDS counters, MFMA busy, clock
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
SH=${SHAPE:-sq4k}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/gpurun_out/g8pmc1 -o run -- python3 $R/scripts/gemm_bench.py $SH > $R/gpurun_out/g8pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/g8pmc2 -o run -- python3 $R/scripts/gemm_bench.py $SH > $R/gpurun_out/g8pmc2.log 2>&1 || exit 2
