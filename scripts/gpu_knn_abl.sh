#!/bin/bash
# K7 v2 ablation: full / fast-filter only / no epilogue (kNN leg only).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for a in ${ABLS:-0 12 11}; do
MRAG_SCAN_ABLATE=$a timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip > gpurun_out/bench_abl$a.log 2>&1 || exit 2
done
