#!/bin/bash
# kNN leg per-step kernel breakdown (rocprofv3 kernel trace of bench.py without the other legs)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r2_knnprof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip --no-fusion > $R/gpurun_out/r2_knnprof.log 2>&1
