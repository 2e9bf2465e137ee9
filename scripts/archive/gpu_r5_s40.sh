#!/bin/bash
# Round 5, session 40: the device-decode stage alone, wall per group and its kernels + copies.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/decode_stage_split.py > gpurun_out/r5s40_split.json 2> gpurun_out/r5s40.err || { echo "split failed"; tail gpurun_out/r5s40.err; exit 3; }
cat gpurun_out/r5s40_split.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/r5s40_prof -o run -- python3 $R/scripts/decode_stage_split.py > $R/gpurun_out/r5s40_prof.log 2>&1 || { echo "prof failed"; tail $R/gpurun_out/r5s40_prof.log; exit 4; }
cd $R
tail -1 gpurun_out/r5s40_prof.log
for f in $(find gpurun_out/r5s40_prof -name "*_stats.csv"); do echo "== $f"; cut -d, -f1-8 "$f" | head -12; done
find gpurun_out/r5s40_prof -name "*trace.csv" -size +20M -delete
