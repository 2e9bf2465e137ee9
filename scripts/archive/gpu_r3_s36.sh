#!/bin/bash
# Round 3, session 36: kernel timeline of one-query searches (the reference's call pattern).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/q1_profile.py > gpurun_out/r3s36_plain.log 2>&1 || { echo "plain failed"; tail -5 gpurun_out/r3s36_plain.log; exit 2; }
cat gpurun_out/r3s36_plain.log
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3s36_prof -o q1 -- python3 scripts/q1_profile.py > gpurun_out/r3s36_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r3s36_prof.log; exit 3; }
f=$(find gpurun_out/r3s36_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/q1_profile.py --trace "$f" > gpurun_out/r3s36_timeline.log
rm -f "$f"
cat gpurun_out/r3s36_timeline.log
