#!/bin/bash
# LayerNorm statistics A/B (kernel stats of the CLIP bench and the config-5 leg)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export MRAG_SYNTHETIC_WEIGHTS=1
for v in 0 1; do
  MRAG_LN_V=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_lnab_$v -o run -- python3 $R/scripts/clip_bench.py 5 > $R/gpurun_out/r2_lnab_$v.log 2>&1 || exit 1
  MRAG_LN_V=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_lnabf_$v -o run -- python3 $R/scripts/fusion_bench.py 5 > $R/gpurun_out/r2_lnabf_$v.log 2>&1 || exit 2
done
