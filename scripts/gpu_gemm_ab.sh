#!/bin/bash
# Encoder GEMM round: parity, then CLIP bench A/B over the GEMM variants + kernel stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_encoders_gpu.py -x -q -m gpu > gpurun_out/enc_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/enc_tests.log; exit 1; }
for v in -1 0 128; do
MRAG_GEMM_BIG=$v timeout -k 10 300 python scripts/clip_bench.py 10 > gpurun_out/clip_big$v.log 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_clip -o run -- python3 $R/scripts/clip_bench.py 10 > $R/gpurun_out/prof_clip.log 2>&1 || exit 4
