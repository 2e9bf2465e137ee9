#!/bin/bash
# attention operand prefetch: encoder parity (default = prefetch), then CLIP / config-5 A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_cross_encoder_gpu.py tests/test_embedder_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_attnpf_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_attnpf_tests.log; exit 1; }
for r in 1 2; do
  for v in 0 1; do
    MRAG_ATTN_PREFETCH=$v timeout -k 10 200 python scripts/clip_bench.py 10 > gpurun_out/r2_attnpf_clip_${v}_$r.log 2>&1 || exit 2
    MRAG_ATTN_PREFETCH=$v timeout -k 10 200 python scripts/fusion_bench.py 10 > gpurun_out/r2_attnpf_fus_${v}_$r.log 2>&1 || exit 3
  done
done
