#!/bin/bash
# Round 3, session 2: K7 variant A/B (MRAG_K7_V bits; two rounds, alternating), K7s with / without
# the sample pre-pass, then the counter passes (scripts/gpu_r3_pmc.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for round in 1 2; do
  for v in 0 1 2 4 8 7 15; do
    MRAG_K7_V=$v timeout -k 10 120 python scripts/knn_scan_ab.py 30 >> gpurun_out/r3s2_k7v.log 2>&1 || exit 1
  done
  MRAG_K7S_NOSAMPLE=1 timeout -k 10 120 python scripts/knn_scan_ab.py 30 >> gpurun_out/r3s2_k7v.log 2>&1 || exit 2
done
cat gpurun_out/r3s2_k7v.log
bash scripts/gpu_r3_pmc.sh || exit 3
