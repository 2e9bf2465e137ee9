#!/bin/bash
# sample pre-pass stride A/B on the kNN bench (same box)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for r in 1 2; do
  for st in 16 32 64 128; do
    MRAG_SAMPLE_STRIDE=$st timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-clip --no-fusion > gpurun_out/r2_stride_${st}_$r.log 2>&1 || exit 1
  done
done
