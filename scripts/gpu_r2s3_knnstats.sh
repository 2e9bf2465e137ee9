#!/bin/bash
# kernel-trace stats of the kNN leg alone (one search in flight): every knn_scan3_kernel<512,0,0,4>
# launch in the summary is a 1M x 512 scan, so its average compares with the bench line's
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s3k_stats -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip --no-fusion --knn-streams 1 > $R/gpurun_out/s3k_stats.log 2>&1 || exit 1
