#!/bin/bash
# Round 6 session 5: K3w probe (time vs M per kernel) for the text-tower shapes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for s in "1536 512 0" "2048 512 1" "1152 384 0" "1536 384 2"; do
  timeout -k 10 200 python3 scripts/gemm_ws_probe.py $s >> gpurun_out/r6s5_probe.jsonl 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r6s5_probe.jsonl; exit 2; }
done
grep '^{' gpurun_out/r6s5_probe.jsonl
