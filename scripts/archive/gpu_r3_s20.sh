#!/bin/bash
# Round 3, session 20: K7 class bounds with batched per-query-block refresh loads (every 16 tiles, k <= 16) A/B (MRAG_K7_GK=0 off), stamps, kNN tests.
# disjoint row classes) A/B in one binary (MRAG_K7_GK=0 off), stamps with fire counts, kNN tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
timeout -k 10 900 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_generic_gpu.py tests/test_full_configs_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s20_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s20_tests.log; exit 1; }
tail -1 gpurun_out/r3s20_tests.log
for round in 1 2 3; do
  for g in 0 1; do
    MRAG_K7_GK=$g timeout -k 10 120 python scripts/knn_scan_ab.py 30 >> gpurun_out/r3s20_ab.log 2>&1 || { echo "ab $g failed"; tail -5 gpurun_out/r3s20_ab.log; exit 2; }
  done
done
grep -v amdgpu.ids gpurun_out/r3s20_ab.log
for g in 0 1; do
  MRAG_K7_GK=$g MRAG_LIB=$L/libmrag_k7stamp.so timeout -k 10 120 python scripts/k7_stamps.py >> gpurun_out/r3s20_stamps.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/r3s20_stamps.log; exit 3; }
done
grep -v amdgpu.ids gpurun_out/r3s20_stamps.log | grep QB4 | cut -c1-700
