#!/bin/bash
# Session 3: parity of the new kernels (K7 v3, K8 16-lane rescoring, attention v2, LN/im2col),
# then A/B timings (v3 vs v2 scan, attention v2 vs v1) and a kernel-stats profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/s3_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/s3_tests.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fusion --steps 30 > gpurun_out/s3_bench_v3.log 2>&1 || exit 2
MRAG_SCAN_V2=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-fusion --no-clip --steps 30 > gpurun_out/s3_bench_v2.log 2>&1 || exit 3
MRAG_ATTN_V1=1 timeout -k 10 300 python scripts/clip_bench.py 20 > gpurun_out/s3_clip_attn_v1.log 2>&1 || exit 4
timeout -k 10 300 python scripts/clip_bench.py 20 > gpurun_out/s3_clip_attn_v2.log 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s3_stats -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fusion > $R/gpurun_out/s3_stats.log 2>&1 || exit 6
