#!/bin/bash
# Round-2: MFMA peak microbenchmark, full GPU tests (new config tests + numerics table),
# PMC pass (MFMA busy / instruction counts / LDS conflicts / GRBM clock) over the bench's kNN and CLIP legs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 120 ./scripts/mfma_peak > gpurun_out/mfma_peak.json 2> gpurun_out/mfma_peak.err || exit 1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_tests2.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_tests2.log; exit 2; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/r2_pmc_sq -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fusion > $R/gpurun_out/r2_pmc_sq.log 2>&1 || exit 3
