#!/bin/bash
# vendor GEMM (hipBLASLt via torch.matmul) on the ViT shapes beside ours: kernel names and times
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
TORCH_REF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_blaslt -o run -- python3 $R/scripts/gemm_bench.py qkv fc1 fc2 out sq4k > $R/gpurun_out/r2_blaslt.log 2>&1
