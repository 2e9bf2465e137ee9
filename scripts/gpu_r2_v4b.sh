#!/bin/bash
# K7 v4 DMA placement A/B (pieces per k-step 1/2/4) against v3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
MRAG_SCAN_V4=1 timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread -k "full_size or seeded or lane_list or clusters" > gpurun_out/r2_v4b_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_v4b_tests.log; exit 1; }
for r in 1 2; do
  MRAG_SCAN_V4=0 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-clip --no-fusion > gpurun_out/r2_v4b_v3_$r.log 2>&1 || exit 2
  for k in 1 2 4; do
    MRAG_SCAN_V4=1 MRAG_SCAN4_PPK=$k timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-clip --no-fusion > gpurun_out/r2_v4b_p${k}_$r.log 2>&1 || exit 3
  done
done
