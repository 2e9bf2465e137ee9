#!/bin/bash
# K4 v3 (flash16) attention: encoder tests + A/B timing against the round-1 dispatch
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_cross_encoder_gpu.py tests/test_configs_gpu.py tests/test_compat_gpu.py tests/test_embedder_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_attn_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_attn_tests.log; exit 1; }
for v in 0 1; do
  MRAG_ATTN_LEGACY=$v timeout -k 10 200 python scripts/fusion_bench.py 10 > gpurun_out/r2_attn_fusion_$v.log 2>&1 || exit 2
  MRAG_ATTN_LEGACY=$v timeout -k 10 200 python scripts/clip_bench.py > gpurun_out/r2_attn_clip_$v.log 2>&1 || exit 3
done
