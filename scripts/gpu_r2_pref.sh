#!/bin/bash
# K3d everywhere it applies vs the round heuristic: config-5 leg A/B on one box
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
for r in 1 2; do
  for t in 0 1; do
    MRAG_GEMM_PREFER_K3D=$t timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/r2_pref_fus_${t}_$r.log 2>&1 || exit 2
  done
done
