#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_knn_gpu.py tests/test_compat_gpu.py -x -q -m gpu > gpurun_out/knn_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/knn_tests.log; exit 1; }
for a in 0 12 11 14; do
MRAG_SCAN_ABLATE=$a timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip > gpurun_out/bench_abl$a.log 2>&1 || exit 2
done
MRAG_SCAN_NO_SAMPLE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip > gpurun_out/bench_v2ns.log 2>&1 || exit 3
