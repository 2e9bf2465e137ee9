#!/bin/bash
# Round 3, session 18: fc1 on K3d (quick_gelu) vs the library's swish form; kernel trace of the CLIP
# leg (one batch in flight) under the default library selection.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 200 python scripts/gemm_bench.py fc1 fc1s qkv fc2 out > gpurun_out/r3s18_gemm.log 2>&1 || { echo "gemm failed"; tail -5 gpurun_out/r3s18_gemm.log; exit 1; }
grep -v amdgpu gpurun_out/r3s18_gemm.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s18_prof -o clip -- python3 scripts/clip_bench.py 20 1 > gpurun_out/r3s18_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r3s18_prof.log; exit 2; }
f=$(find gpurun_out/r3s18_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r3s18_clip_kernel_stats.csv
find gpurun_out/r3s18_prof -name "*kernel_trace.csv" -delete
python3 scripts/kstats.py gpurun_out/r3s18_clip_kernel_stats.csv > gpurun_out/r3s18_kstats.txt
head -16 gpurun_out/r3s18_kstats.txt
