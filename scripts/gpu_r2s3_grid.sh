#!/bin/bash
# K3d persistent grid size under work in flight (MRAG_G8_GRID caps the workgroups per launch)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
for g in 0 128 192 0 128 192; do
if [ $g = 0 ]; then unset MRAG_G8_GRID; else export MRAG_G8_GRID=$g; fi
timeout -k 10 200 python scripts/clip_bench.py 30 3 > gpurun_out/gr_clip_$g.log 2>&1 || exit 1
timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/gr_fus_$g.log 2>&1 || exit 2
echo "$g $(tail -1 gpurun_out/gr_clip_$g.log | cut -c1-90) $(tail -1 gpurun_out/gr_fus_$g.log | cut -c1-110)" >> gpurun_out/gr_summary.log
done
