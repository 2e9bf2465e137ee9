#!/bin/bash
# Round 6 session 9: the config-5 leg (bench fusion_leg, four steps in flight) per GEMM kernel
# rule, interleaved on one box: base = round-5 rules (HEAD before K3w), cur = K3w for the f16
# q|k|v GEMMs, wsall = K3w for every f16 epilogue, wsk3tie = cur + K3 on K3/K3d ties.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=$R/multimodal-rag-for-image-text-search_amd/lib
for round in 1 2; do
  for lib in libmrag_base libmrag libmrag_wsall libmrag_wsk3tie; do
    MRAG_LIB=$L/$lib.so timeout -k 10 200 python3 -c "
import json, sys
sys.path[:0] = ['$R', '$R/multimodal-rag-for-image-text-search_amd']
import bench
out = bench.fusion_leg(1, 0, 0, 40, 4)
print(json.dumps({'lib': '$lib', 'round': $round, 'value': out['value'], 'ms_per_step': out['ms_per_step']}))
" >> gpurun_out/r6s9_fusion_ab.jsonl 2>&1 || { echo "fusion failed $lib"; tail -5 gpurun_out/r6s9_fusion_ab.jsonl; exit 2; }
  done
done
grep '^{' gpurun_out/r6s9_fusion_ab.jsonl
