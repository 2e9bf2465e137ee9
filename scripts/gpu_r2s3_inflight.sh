#!/bin/bash
# work in flight: CLIP batches 1-4, config-5 steps 1-3, kNN searches 2-4
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
for v in 1 2 3 4 3; do
timeout -k 10 200 python scripts/clip_bench.py 30 $v > gpurun_out/if_clip$v.log 2>&1 || exit 1
done
for v in 1 2 3 2 1; do
MRAG_FUSION_INFLIGHT=$v timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/if_fus$v.log 2>&1 || exit 2
done
for v in 2 3 4; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-clip --no-fusion --knn-streams $v > gpurun_out/if_knn$v.log 2>&1 || exit 3
done
