#!/bin/bash
# Round 6 session 21: LayerNorm with four rows in flight per wave (layernorm_stream4_kernel)
# against the one-row prefetch (libmrag_base = the tree before). Encoder parity tests, then the
# config-5 leg and CLIP (three / one batches in flight) interleaved, three rounds.
P=r6s21
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=$R/multimodal-rag-for-image-text-search_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${P}_tests.log; exit 3; }
tail -1 gpurun_out/${P}_tests.log
for round in 1 2 3; do
  for lib in libmrag_base libmrag; do
    MRAG_LIB=$L/$lib.so timeout -k 10 200 python3 -c "
import json, sys
sys.path[:0] = ['$R', '$R/multimodal-rag-for-image-text-search_amd']
import bench
out = bench.fusion_leg(1, 0, 0, 40, 4)
print(json.dumps({'leg': 'fusion', 'lib': '$lib', 'round': $round, 'value': out['value'], 'one': out['one_step_in_flight']['queries_per_s']}))
" 2>/dev/null | grep '^{' >> gpurun_out/${P}_ab.jsonl || { echo "fusion failed $lib"; exit 2; }
    MRAG_LIB=$L/$lib.so timeout -k 10 200 python3 scripts/clip_bench.py 30 3 2>/dev/null | grep '^{' | sed "s/^{/{\"leg\": \"clip3\", \"lib\": \"$lib\", \"round\": $round, /" >> gpurun_out/${P}_ab.jsonl || { echo "clip failed $lib"; exit 5; }
    MRAG_LIB=$L/$lib.so timeout -k 10 200 python3 scripts/clip_bench.py 30 1 2>/dev/null | grep '^{' | sed "s/^{/{\"leg\": \"clip1\", \"lib\": \"$lib\", \"round\": $round, /" >> gpurun_out/${P}_ab.jsonl || { echo "clip failed $lib"; exit 6; }
  done
done
cut -c1-160 gpurun_out/${P}_ab.jsonl
