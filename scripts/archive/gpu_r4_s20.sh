#!/bin/bash
# Round 4, session 20 (A/B only): non-temporal f16 epilogue stores (lib/libmrag_nt.so) vs default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
P=$R/multimodal-rag-for-image-text-search_amd/lib
for v in nt def nt def; do
  L=$P/libmrag.so; [ $v = nt ] && L=$P/libmrag_nt.so
  MRAG_LIB=$L timeout -k 10 150 python3 -u scripts/gemm_bench.py qkv fc1 t_qkv t_fc1 > gpurun_out/r4s20_$v.log 2>&1 || { echo "bench $v failed"; exit 1; }
  MRAG_LIB=$L timeout -k 10 200 python3 -u scripts/clip_bench.py 30 3 > gpurun_out/r4s20_clip_$v.json 2>/dev/null || { echo "clip $v failed"; exit 1; }
  echo "$v: $(grep -h '"shape"' gpurun_out/r4s20_$v.log | python3 -c "
import sys, json
print(' '.join(f\"{d['shape']}={d['us']}/{d['digest'][:8]}\" for d in map(json.loads, sys.stdin)))") clip3=$(python3 -c "import json; print(json.load(open('gpurun_out/r4s20_clip_$v.json'))['value'])")" | tee -a gpurun_out/r4s20_ab.txt
done
