#!/bin/bash
# K3-only (MRAG_GEMM_BIG=0, non-persistent 128 x 128, XCD-remapped) vs default K3d under work in flight
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
for v in 1 0 1 0; do
MRAG_GEMM_BIG=$v timeout -k 10 200 python scripts/clip_bench.py 30 3 > gpurun_out/k3o_clip3_$v.log 2>&1 || exit 1
MRAG_GEMM_BIG=$v timeout -k 10 200 python scripts/clip_bench.py 30 1 > gpurun_out/k3o_clip1_$v.log 2>&1 || exit 2
MRAG_GEMM_BIG=$v timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/k3o_fus_$v.log 2>&1 || exit 3
done
MRAG_GEMM_BIG=0 timeout -k 10 200 python scripts/gemm_bench.py qkv fc1 fc2 out > gpurun_out/k3o_gemm.log 2>&1 || exit 4
