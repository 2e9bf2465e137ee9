#!/bin/bash
# Round 3, session 3: K7 variant A/B, K3f GEMM A/B (bit-identity digests + timing on the ViT / text
# shapes), then the counter passes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for k in 0 3 1; do
  MRAG_GEMM_K3F=$k timeout -k 10 200 python scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_fc1 t_fc2 m_fc1 > gpurun_out/r3s3_gemm_k3f$k.log 2>&1 || { echo "gemm k3f=$k failed"; tail -5 gpurun_out/r3s3_gemm_k3f$k.log; exit 1; }
done
for k in 0 3 1; do echo "== K3F=$k"; cat gpurun_out/r3s3_gemm_k3f$k.log; done
for round in 1 2; do
  for v in 0 1 2 4 8 7 15; do
    MRAG_K7_V=$v timeout -k 10 120 python scripts/knn_scan_ab.py 30 >> gpurun_out/r3s3_k7v.log 2>&1 || exit 2
  done
  MRAG_K7S_NOSAMPLE=1 timeout -k 10 120 python scripts/knn_scan_ab.py 30 >> gpurun_out/r3s3_k7v.log 2>&1 || exit 3
done
cat gpurun_out/r3s3_k7v.log
bash scripts/gpu_r3_pmc.sh || exit 4
