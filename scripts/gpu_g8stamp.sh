#!/bin/bash
# K3d in-kernel stamps (ABL 6 diagnostic build) on the 4096^3 and qkv shapes
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
MRAG_GEMM_ABL=6 timeout -k 10 100 python scripts/gemm_bench.py sq4k qkv > gpurun_out/g8stamp.log 2>&1 || exit 1
