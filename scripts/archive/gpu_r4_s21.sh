#!/bin/bash
# Round 4, session 21: K3d with the slot's LDS-DMA issued in the MFMA segment (lib/libmrag.so) vs
# the validated build (lib/libmrag_prev.so): digests, timings, encoder parity, CLIP, config 5.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
P=$R/multimodal-rag-for-image-text-search_amd/lib
for v in new prev new prev; do
  L=$P/libmrag.so; [ $v = prev ] && L=$P/libmrag_prev.so
  MRAG_LIB=$L timeout -k 10 200 python3 -u scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_fc1 > gpurun_out/r4s21_$v.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/r4s21_$v.log; exit 1; }
  echo "$v: $(grep -h '"shape"' gpurun_out/r4s21_$v.log | python3 -c "
import sys, json
print(' '.join(f\"{d['shape']}={d['us']}/{d['digest'][:8]}/{d['deterministic']}\" for d in map(json.loads, sys.stdin)))")" | tee -a gpurun_out/r4s21_ab.txt
done
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_embedder_gpu.py tests/test_cross_encoder_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r4s21_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r4s21_tests.log
[ $rc -ne 0 ] && exit $rc
for v in new prev new; do
  L=$P/libmrag.so; [ $v = prev ] && L=$P/libmrag_prev.so
  MRAG_LIB=$L timeout -k 10 200 python3 -u scripts/clip_bench.py 30 3 > gpurun_out/r4s21_clip_$v.json 2>/dev/null || { echo "clip failed"; exit 1; }
  MRAG_LIB=$L timeout -k 10 300 python3 -u scripts/fusion_bench.py 20 > gpurun_out/r4s21_fus_$v.json 2>/dev/null || { echo "fusion failed"; exit 1; }
  python3 -c "
import json
c=json.load(open('gpurun_out/r4s21_clip_$v.json')); f=json.load(open('gpurun_out/r4s21_fus_$v.json'))
print('$v clip3', c['value'], 'fusion', f['value'])" | tee -a gpurun_out/r4s21_ab.txt
done
