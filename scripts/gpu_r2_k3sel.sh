#!/bin/bash
# K3 vs K3d selection on the text-tower shapes (config-5 batch) and the ViT shapes
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for v in -1 0; do
  MRAG_GEMM_BIG=$v timeout -k 10 150 python scripts/gemm_bench.py t_qkv t_out t_fc1 t_fc2 m_qkv m_out m_fc1 m_fc2 qkv fc1 fc2 out > gpurun_out/r2_k3sel_$v.log 2>&1 || exit 1
done
