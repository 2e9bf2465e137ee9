#!/bin/bash
# Round 4, session 16: searches in flight for the kNN leg (2 = default) on one box, twice each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for n in 2 3 4 2 3 4; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-clip --no-fusion --no-call-pattern --knn-streams $n --steps 40 > gpurun_out/r4s16_s$n.log 2>&1 || { echo "streams $n failed"; tail -5 gpurun_out/r4s16_s$n.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r4s16_s$n.log') if l.startswith('{')][-1])
print($n, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config'].get('searches_in_flight'))" | tee -a gpurun_out/r4s16_streams.txt
done
