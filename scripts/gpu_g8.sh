#!/bin/bash
# GEMM A/B: K3d default vs K3 only (MRAG_GEMM_BIG=0), ablations, encoder GPU tests, CLIP bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/g8_new.log 2>&1 || exit 1
MRAG_GEMM_BIG=0 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/g8_k3.log 2>&1 || exit 2
timeout -k 10 300 python -m pytest -x -q tests/test_encoders_gpu.py tests/test_cross_encoder_gpu.py tests/test_compat_gpu.py > gpurun_out/g8_tests.log 2>&1 || exit 3
timeout -k 10 300 python scripts/clip_bench.py 10 > gpurun_out/g8_clip.log 2>&1 || exit 4
for a in ${ABLS:-}; do
MRAG_GEMM_ABL=$a timeout -k 10 100 python scripts/gemm_bench.py qkv sq4k > gpurun_out/g8abl$a.log 2>&1 || exit 5
done
