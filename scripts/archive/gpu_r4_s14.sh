#!/bin/bash
# Round 4, session 14: CLIP batches in flight (hand-written GEMMs only) and a one-batch kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for n in 3 4 5 6 3; do
  timeout -k 10 200 python3 -u $R/scripts/clip_bench.py 30 $n >> $R/gpurun_out/r4s14_inflight.log 2>/dev/null || { echo "clip $n failed"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4s14_prof -o clip -- python3 $R/scripts/clip_bench.py 10 1 > $R/gpurun_out/r4s14_prof.log 2>&1 || { echo "prof failed"; exit 2; }
cd $R
python3 -c "
import json
for l in open('gpurun_out/r4s14_inflight.log'):
    d=json.loads(l); print(d['batches_in_flight'], d['value'], d['ms_per_batch'])"
f=$(find gpurun_out/r4s14_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_by_grid.py $f 20 | tee gpurun_out/r4s14_clip_by_grid.txt
rm -f $f
