#!/bin/bash
# CLIP batches in flight vs stream choice (hardware-queue mapping experiment)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
for cfg in "1 1" "2 1" "2 2" "2 3" "3 1" "4 1" "2 4"; do
set -- $cfg
MRAG_BENCH_STREAM_SKIP=$2 timeout -k 10 200 python scripts/clip_bench.py 30 $1 > gpurun_out/c3_clip_$1_$2.log 2>&1 || exit 1
done
for sk in 1 2 3; do
MRAG_BENCH_STREAM_SKIP=$sk timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/c3_fus_$sk.log 2>&1 || exit 2
done
