#!/bin/bash
# sample pre-pass stride A/B (16 / 32 / 8) on the 1M x 512 bench, kNN tests at the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for i in 1 2; do
  for st in 16 32 8; do
    MRAG_SAMPLE_STRIDE=$st timeout -k 10 200 python bench.py --no-cpu-baseline --no-fusion --no-clip --steps 40 > gpurun_out/s3d_st${st}_$i.log 2>&1 || exit 2
  done
done
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py -x -v -m gpu -k cfg1 --timeout 300 --timeout-method thread > gpurun_out/s3d_tests.log 2>&1 || exit 3
