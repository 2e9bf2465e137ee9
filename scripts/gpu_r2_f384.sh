#!/bin/bash
# K7 at DP = 384 (config-5 text shard): DMA front 2 / 3 / 4, kernel stats of the serial config-5 leg
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export MRAG_SYNTHETIC_WEIGHTS=1 MRAG_FUSION_STREAMS=1
for f in 4 2 3 4; do
  MRAG_SCAN_FRONT384=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_f384_$f -o run -- python3 $R/scripts/fusion_bench.py 10 > $R/gpurun_out/r2_f384_$f.log 2>&1 || exit 1
done
