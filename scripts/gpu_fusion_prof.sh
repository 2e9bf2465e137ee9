#!/bin/bash
# config-5 leg: kernel stats
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fusion -o run -- python3 $R/scripts/fusion_bench.py 10 > $R/gpurun_out/prof_fusion.log 2>&1 || exit 1
