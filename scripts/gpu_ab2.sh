#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_knn_gpu.py tests/test_encoders_gpu.py -x -q -m gpu > gpurun_out/ab2_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/ab2_tests.log; exit 1; }
for v in -1 2 0; do
MRAG_GEMM_BIG=$v timeout -k 10 300 python scripts/clip_bench.py 10 > gpurun_out/clip_big$v.log 2>&1 || exit 2
done
for a in 0 11; do
MRAG_SCAN_ABLATE=$a timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip > gpurun_out/bench_abl$a.log 2>&1 || exit 3
done
