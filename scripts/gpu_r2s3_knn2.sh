#!/bin/bash
# search contexts: kNN GPU suite (+ concurrent searches), then the bench with 2 searches in flight
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_generic_gpu.py tests/test_compat_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/k2_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/k2_tests.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-clip --no-fusion > gpurun_out/k2_bench.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --no-cpu-baseline --no-clip --no-fusion --knn-streams 3 > gpurun_out/k2_bench3.log 2>&1 || exit 3
