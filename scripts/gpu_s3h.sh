#!/bin/bash
# K7 v3 DMA front-loading A/B (FRONT 2 default vs 1) + kNN parity.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s3h_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-fusion --no-clip --steps 40 > gpurun_out/s3h_f2_$i.log 2>&1 || exit 2
  MRAG_SCAN_FRONT=2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-fusion --no-clip --steps 40 > gpurun_out/s3h_f1_$i.log 2>&1 || exit 3
done
