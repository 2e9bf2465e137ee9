#!/bin/bash
# config-5 leg: one stream vs two branches in two host threads (A/B, two rounds)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
for r in 1 2; do
  for v in 1 2; do
    MRAG_FUSION_STREAMS=$v timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/r2_fus2_${v}_$r.log 2>&1 || exit 1
  done
done
