#!/bin/bash
# persistent attention v2: parity, then CLIP A/B over workgroups per CU (and one pair per wave = 3).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_compat_gpu.py tests/test_cross_encoder_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s3g_tests.log 2>&1 || exit 1
for i in 1 2; do
  for g in 1 2 3; do
    MRAG_ATTN_WG_PER_CU=$g timeout -k 10 200 python scripts/clip_bench.py 20 > gpurun_out/s3g_clip_g${g}_$i.log 2>&1 || exit 2
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s3g_stats -o run -- python3 $R/scripts/clip_bench.py 10 > $R/gpurun_out/s3g_stats.log 2>&1 || exit 3
