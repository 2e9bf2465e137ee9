#!/bin/bash
# CLIP batch split over concurrent streams: identity test, then parts 1/2/4 A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 300 python -u -m pytest tests/test_encoders_gpu.py -k "split or batch_consistency" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r2_split_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_split_tests.log; exit 1; }
for r in 1 2; do
  for p in 1 2 4; do
    MRAG_CLIP_PARTS=$p timeout -k 10 200 python scripts/clip_bench.py 10 > gpurun_out/r2_split_${p}_$r.log 2>&1 || exit 2
  done
done
