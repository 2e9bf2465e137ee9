#!/bin/bash
# K3d CFG 1 (128 x 384 tiles for N = 768): encoder parity, GEMM A/B per shape, CLIP A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_compat_gpu.py tests/test_cross_encoder_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/s3c_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/s3c_tests.log; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python scripts/gemm_bench.py fc2 out > gpurun_out/s3c_gemm_cfg_auto_$i.log 2>&1 || exit 2
  MRAG_G8_CFG=0 timeout -k 10 200 python scripts/gemm_bench.py fc2 out > gpurun_out/s3c_gemm_cfg0_$i.log 2>&1 || exit 3
  timeout -k 10 200 python scripts/clip_bench.py 20 > gpurun_out/s3c_clip_auto_$i.log 2>&1 || exit 4
  MRAG_G8_CFG=0 timeout -k 10 200 python scripts/clip_bench.py 20 > gpurun_out/s3c_clip_cfg0_$i.log 2>&1 || exit 5
done
