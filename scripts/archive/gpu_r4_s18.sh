#!/bin/bash
# Round 4, session 18: K3d f16 epilogue writing 8 rows x 128 B per store (DPP lane exchange) vs the
# previous build (lib/libmrag_abl0.so = the same tree before the change), digests must match.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for v in new old new old; do
  L=$R/multimodal-rag-for-image-text-search_amd/lib/libmrag.so
  [ $v = old ] && L=$R/multimodal-rag-for-image-text-search_amd/lib/libmrag_abl0.so
  MRAG_LIB=$L timeout -k 10 150 python3 -u scripts/gemm_bench.py qkv fc1 t_qkv t_fc1 m_fc1 > gpurun_out/r4s18_$v.log 2>&1 || { echo "bench $v failed"; exit 1; }
  echo "$v: $(grep -h '"shape"' gpurun_out/r4s18_$v.log | python3 -c "
import sys, json
print(' '.join(f\"{d['shape']}={d['us']}/{d['digest'][:8]}\" for d in map(json.loads, sys.stdin)))")" | tee -a gpurun_out/r4s18_ab.txt
done
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_embedder_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r4s18_tests.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/r4s18_tests.log
timeout -k 10 300 python3 -u scripts/clip_bench.py 30 3 > gpurun_out/r4s18_clip.json 2>/dev/null && python3 -c "import json; print('clip3', json.load(open('gpurun_out/r4s18_clip.json'))['value'])"
MRAG_LIB=$R/multimodal-rag-for-image-text-search_amd/lib/libmrag_abl0.so timeout -k 10 300 python3 -u scripts/clip_bench.py 30 3 > gpurun_out/r4s18_clip_old.json 2>/dev/null && python3 -c "import json; print('clip3 old', json.load(open('gpurun_out/r4s18_clip_old.json'))['value'])"
