#!/bin/bash
# four sample maxima per (split, query) for the v3 seed: kNN parity, then bench A/B vs pairs
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_generic_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_seed4_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_seed4_tests.log; exit 1; }
for r in 1 2; do
  for v in 0 1; do
    MRAG_SAMPLE_PAIRS=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-clip --no-fusion > gpurun_out/r2_seed4_${v}_$r.log 2>&1 || exit 2
  done
done
