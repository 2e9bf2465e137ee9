#!/bin/bash
# Round 3, session 27: CLIP batches in flight 2 / 3 / 4 with the library GEMMs (two rounds).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for round in 1 2; do
  for f in 2 3 4; do
    timeout -k 10 200 python scripts/clip_bench.py 40 $f > gpurun_out/r3s27_clip.json 2>gpurun_out/r3s27_clip.err || { echo "clip failed"; tail -5 gpurun_out/r3s27_clip.err; exit 2; }
    echo "inflight=$f $(grep -v amdgpu gpurun_out/r3s27_clip.json | cut -c1-130)" >> gpurun_out/r3s27_legs.log
  done
done
cat gpurun_out/r3s27_legs.log
