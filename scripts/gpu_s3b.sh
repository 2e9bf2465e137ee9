#!/bin/bash
# K7 v3 (KL3 = 6): kNN parity, then v3 / v2 A/B and v3 ablations (timing only) on one box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_compat_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/s3b_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/s3b_tests.log; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-fusion --no-clip --steps 40 > gpurun_out/s3b_v3_$i.log 2>&1 || exit 2
  MRAG_SCAN_V2=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-fusion --no-clip --steps 40 > gpurun_out/s3b_v2_$i.log 2>&1 || exit 3
done
MRAG_SCAN_ABLATE=21 timeout -k 10 200 python bench.py --no-cpu-baseline --no-fusion --no-clip --steps 40 > gpurun_out/s3b_abl21.log 2>&1 || exit 4
MRAG_SCAN_ABLATE=24 timeout -k 10 200 python bench.py --no-cpu-baseline --no-fusion --no-clip --steps 40 > gpurun_out/s3b_abl24.log 2>&1 || exit 5
