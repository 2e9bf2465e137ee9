#!/bin/bash
# K3 XCD-contiguous tile order: GEMM shapes on K3 and the config-5 leg, A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 300 python -u -m pytest tests/test_encoders_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/km_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/km_tests.log; exit 1; }
for v in 0 1; do
MRAG_K3_REMAP=$v timeout -k 10 200 python scripts/gemm_bench.py t_out t_fc2 m_qkv m_out m_fc2 t_qkv > gpurun_out/km_gemm$v.log 2>&1 || exit 2
MRAG_K3_REMAP=$v timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/km_fus$v.log 2>&1 || exit 3
done
MRAG_K3_REMAP=0 timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/km_fus0b.log 2>&1 || exit 4
MRAG_K3_REMAP=1 timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/km_fus1b.log 2>&1 || exit 5
