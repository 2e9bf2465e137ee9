#!/bin/bash
# GEMM selection ties -> K3 vs K3d: config-5 leg A/B on one box (serial and two-stream)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
for r in 1 2; do
  for t in 0 1; do
    MRAG_GEMM_TIE_K3D=$t timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/r2_tie_fus_${t}_$r.log 2>&1 || exit 2
  done
done
