#!/bin/bash
# K3d stream-K: parity (forced SK on every K3d shape + the encoder suite), then GEMM and CLIP A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_encoders_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/sk_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/sk_tests.log; exit 1; }
for v in 0 1; do
MRAG_G8_SK=$v timeout -k 10 200 python scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_fc1 t_fc2 m_fc1 > gpurun_out/sk_gemm$v.log 2>&1 || exit 2
MRAG_G8_SK=$v timeout -k 10 200 python scripts/clip_bench.py 20 > gpurun_out/sk_clip$v.log 2>&1 || exit 3
done
MRAG_G8_SK=2 timeout -k 10 200 python scripts/gemm_bench.py qkv fc1 t_qkv t_fc1 > gpurun_out/sk_gemm2.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/sk_bench.log 2>&1 || exit 5
