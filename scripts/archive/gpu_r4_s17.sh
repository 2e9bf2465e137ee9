#!/bin/bash
# Round 4, session 17 (A/B only): ViT N = 768 GEMMs on K3 (600 tiles) vs K3d (150 tiles).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for v in 0 768 0 768; do
  for n in 3 1; do
    MRAG_EXP_K3_N=$v timeout -k 10 200 python3 -u scripts/clip_bench.py 30 $n > gpurun_out/r4s17_tmp.json 2>/dev/null || { echo "clip failed"; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r4s17_tmp.json')); print('k3_n=$v inflight=$n', d['value'])" | tee -a gpurun_out/r4s17_ab.txt
  done
done
MRAG_EXP_K3_N=768 timeout -k 10 300 python3 -u -m pytest tests/test_encoders_gpu.py -q -k "clip_image" --timeout 120 --timeout-method thread 2>&1 | tail -2
