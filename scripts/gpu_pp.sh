#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_encoders_gpu.py -x -q -m gpu > gpurun_out/pp_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/pp_tests.log; exit 1; }
for v in -1 256; do
MRAG_GEMM_BIG=$v timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_pp$v.log 2>&1 || exit 2
MRAG_GEMM_BIG=$v timeout -k 10 300 python scripts/clip_bench.py 10 > gpurun_out/clip_pp$v.log 2>&1 || exit 3
done
