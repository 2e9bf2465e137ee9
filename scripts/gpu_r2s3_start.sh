#!/bin/bash
# Session-3 start: bench sanity on a fresh build + GEMM shapes vs the vendor library
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s3_bench.log 2>&1 || { echo "bench failed rc=$?" >> gpurun_out/s3_bench.log; exit 1; }
TORCH_REF=1 timeout -k 10 300 python scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_out t_fc1 t_fc2 m_qkv m_out m_fc1 m_fc2 > gpurun_out/s3_gemm.log 2>&1 || exit 2
