#!/bin/bash
# K7 v5 (three 48-row LDS buffers): exactness under MRAG_SCAN_V5=1, then A/B against v3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
MRAG_SCAN_V5=1 timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_generic_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_v5_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_v5_tests.log; exit 1; }
for r in 1 2; do
  for v in 0 1; do
    MRAG_SCAN_V5=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-clip --no-fusion > gpurun_out/r2_v5_bench_${v}_$r.log 2>&1 || exit 2
  done
done
