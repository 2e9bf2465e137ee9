#!/bin/bash
# Round 3, session 29: config-5 leg with 2 / 3 steps in flight (two rounds).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for round in 1 2; do
  for f in 2 3; do
    MRAG_FUSION_INFLIGHT=$f timeout -k 10 300 python scripts/fusion_bench.py 24 > gpurun_out/r3s29_fusion.json 2>gpurun_out/r3s29_fusion.err || { echo "fusion failed"; tail -5 gpurun_out/r3s29_fusion.err; exit 2; }
    echo "inflight=$f $(grep -v amdgpu gpurun_out/r3s29_fusion.json | cut -c1-150)" >> gpurun_out/r3s29_legs.log
  done
done
cat gpurun_out/r3s29_legs.log
