#!/bin/bash
# config-5 leg kernel breakdown (serial branches), rocprofv3 kernel trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export MRAG_SYNTHETIC_WEIGHTS=1 MRAG_FUSION_STREAMS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_fusprof -o run -- python3 $R/scripts/fusion_bench.py 10 > $R/gpurun_out/r2_fusprof.log 2>&1
