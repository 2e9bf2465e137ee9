#!/bin/bash
# Round 5: the SQ / TCC counter passes (scripts/gpu_r5_pmc.sh), then the config-5 leg with two vs
# four steps in flight, three interleaved pairs (re-check of the round-4 choice).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
bash scripts/gpu_r5_pmc.sh || exit $?
cd $R
for v in 2 4 2 4 2 4; do
  MRAG_FUSION_INFLIGHT=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip --no-call-pattern --no-retrieve-pattern --no-ingest > gpurun_out/r5_fusion_if$v.log 2>&1 || { echo "fusion $v failed"; tail -5 gpurun_out/r5_fusion_if$v.log; exit 30; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/r5_fusion_if$v.log') if l.startswith('{\"metric\"')][-1])
f=d.get('fusion') or d.get('config5') or {}
print('inflight $v', json.dumps({k: f.get(k) for k in ('value','ms_per_step','steps_in_flight')}))" | tee -a gpurun_out/r5_fusion_inflight_ab.txt
done
