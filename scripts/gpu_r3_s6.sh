#!/bin/bash
# Round 3, session 6: K3f v3 (A-fragment ring, 1 / 2 staging sets) vs K3d, ablations of K3f.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for k in 0 1 2; do
  MRAG_GEMM_K3F=$k timeout -k 10 200 python scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_fc1 t_fc2 m_fc1 > gpurun_out/r3s6_gemm_k3f$k.log 2>&1 || { echo "gemm k3f=$k failed"; tail -5 gpurun_out/r3s6_gemm_k3f$k.log; exit 1; }
done
for a in 1 2 4 7; do
  MRAG_GEMM_K3F=2 MRAG_K3F_ABL=$a timeout -k 10 100 python scripts/gemm_bench.py qkv t_qkv > gpurun_out/r3s6_abl$a.log 2>&1 || { echo "abl $a failed"; tail -5 gpurun_out/r3s6_abl$a.log; exit 2; }
done
for k in 0 1 2; do echo "== K3F=$k"; grep -v amdgpu.ids gpurun_out/r3s6_gemm_k3f$k.log; done
for a in 1 2 4 7; do echo "== ABL=$a"; grep -v amdgpu.ids gpurun_out/r3s6_abl$a.log; done
