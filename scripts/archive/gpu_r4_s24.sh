#!/bin/bash
# Round 4, session 24 (A/B only): config-5 steps in flight (MRAG_FUSION_INFLIGHT 2 = default, 3, 4).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for n in ${NS:-2 3 4 2 3 4}; do
  MRAG_FUSION_INFLIGHT=$n timeout -k 10 300 python3 -u scripts/fusion_bench.py ${STEPS:-20} > gpurun_out/r4s24_f$n.json 2>/dev/null || { echo "fusion $n failed"; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r4s24_f$n.json')); print('inflight $n', d['value'], d.get('steps_in_flight'))" | tee -a gpurun_out/r4s24_ab.txt
done
