#!/bin/bash
# attention kernel time with / without the operand prefetch (kernel stats of the CLIP bench)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export MRAG_SYNTHETIC_WEIGHTS=1
for v in 0 1; do
  MRAG_ATTN_PREFETCH=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_attnprof_$v -o run -- python3 $R/scripts/clip_bench.py 5 > $R/gpurun_out/r2_attnprof_$v.log 2>&1 || exit 1
done
