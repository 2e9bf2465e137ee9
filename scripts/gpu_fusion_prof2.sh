#!/bin/bash
# kernel stats of the config-5 leg alone (kNN + CLIP legs skipped via a tiny main leg).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fus_stats -o run -- python3 $R/scripts/fusion_bench.py > $R/gpurun_out/fus_stats.log 2>&1 || exit 1
