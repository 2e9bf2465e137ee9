#!/bin/bash
# K3d grid / LDS diagnostics on the 4096^3 and qkv shapes
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
: > gpurun_out/g8diag.log
for gr in 256 248 240 224 128; do
echo "grid $gr" >> gpurun_out/g8diag.log
MRAG_G8_VERBOSE=1 MRAG_G8_GRID=$gr timeout -k 10 100 python scripts/gemm_bench.py sq4k qkv >> gpurun_out/g8diag.log 2>&1 || exit 1
done
echo "ABL 8 (no LDS bias)" >> gpurun_out/g8diag.log
MRAG_GEMM_ABL=8 timeout -k 10 100 python scripts/gemm_bench.py sq4k qkv >> gpurun_out/g8diag.log 2>&1 || exit 2
