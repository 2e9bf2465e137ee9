#!/bin/bash
# kernel breakdowns of the config-5 leg (two-stream default and serial) and of the CLIP tower
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s3_fus -o run -- python3 $R/scripts/fusion_bench.py 10 > $R/gpurun_out/s3_fus.log 2>&1 || exit 1
MRAG_FUSION_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s3_fus1 -o run -- python3 $R/scripts/fusion_bench.py 10 > $R/gpurun_out/s3_fus1.log 2>&1 || exit 2
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s3_clip -o run -- python3 $R/scripts/clip_bench.py 10 > $R/gpurun_out/s3_clip.log 2>&1 || exit 3
