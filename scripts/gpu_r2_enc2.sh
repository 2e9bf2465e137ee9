#!/bin/bash
# encoder parity + CLIP / config-5 timing after the LN revert and the attention load-at-top change
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py tests/test_embedder_gpu.py tests/test_cross_encoder_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_enc2_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_enc2_tests.log; exit 1; }
for r in 1 2; do
  timeout -k 10 200 python scripts/clip_bench.py 10 > gpurun_out/r2_enc2_clip_$r.log 2>&1 || exit 2
  timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/r2_enc2_fus_$r.log 2>&1 || exit 3
done
