#!/bin/bash
# K7 sample pre-pass stride with two searches in flight (MRAG_SAMPLE_STRIDE; default 16)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for st in 16 12 20 24 16 12 20 24; do
MRAG_SAMPLE_STRIDE=$st timeout -k 10 300 python bench.py --no-cpu-baseline --no-clip --no-fusion > gpurun_out/st_$st.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/st_$st.log') if l.startswith('{\"metric\"')][-1]); print($st, d['value'], d['config']['one_search_in_flight']['queries_per_s'], d['roofline']['avg_launch_ms'], d['config']['uncertified_queries_last_step'])" >> gpurun_out/st_summary.log
done
