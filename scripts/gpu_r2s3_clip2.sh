#!/bin/bash
# CLIP batches in flight: 1 / 2 / 3 (alternating), plus the old default-stream form for reference
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
for r in 1 2; do
for v in 1 2 3; do
timeout -k 10 200 python scripts/clip_bench.py 30 $v > gpurun_out/c2_clip${v}_$r.log 2>&1 || exit 1
done
done
