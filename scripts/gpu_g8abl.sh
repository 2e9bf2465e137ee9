#!/bin/bash
# K3d ablations (timing only): MRAG_GEMM_ABL on the qkv / out / 4096^3 shapes (EPI_F16)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for a in ${ABLS:-0 1 2 3 5 7}; do
MRAG_GEMM_ABL=$a timeout -k 10 100 python scripts/gemm_bench.py qkv sq4k > gpurun_out/g8abl$a.log 2>&1 || exit 1
done
