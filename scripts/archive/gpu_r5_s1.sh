#!/bin/bash
# Round 5, session 1: K7 fire path with the chain-free list insert (list_insert_par).
# kNN GPU tests on the working tree, then same-box A/B of the main scan (base = HEAD before the
# change, par = working tree) and the K7 segment stamps of both.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s1_knn_tests.log 2>&1 || { echo "knn tests failed"; tail -30 gpurun_out/r5s1_knn_tests.log; exit 3; }
tail -1 gpurun_out/r5s1_knn_tests.log
for v in base par base par base par; do
  MRAG_LIB=$R/$L/libmrag_$v.so timeout -k 10 240 python3 -u scripts/knn_scan_ab.py 40 > gpurun_out/r5s1_ab_$v.json 2>/dev/null || { echo "ab $v failed"; exit 4; }
  echo "$v $(cat gpurun_out/r5s1_ab_$v.json)" | tee -a gpurun_out/r5s1_ab.txt
done
for v in base par; do
  MRAG_LIB=$R/$L/libmrag_k7stamp_$v.so timeout -k 10 240 python3 -u scripts/k7_stamps.py > gpurun_out/r5s1_stamps_$v.log 2>&1 || { echo "stamps $v failed"; exit 5; }
  echo "stamps $v"; head -1 gpurun_out/r5s1_stamps_$v.log | cut -c1-600
done
# K3x (activation operand direct to VGPRs) vs K3 / K3d on every encoder GEMM shape, digests must match
for v in par ax par ax; do
  MRAG_LIB=$R/$L/libmrag_$v.so timeout -k 10 300 python3 -u scripts/gemm_bench.py > gpurun_out/r5s1_gemm_$v.jsonl 2>&1 || { echo "gemm $v failed"; tail -5 gpurun_out/r5s1_gemm_$v.jsonl; exit 6; }
  echo "== gemm $v"; cat gpurun_out/r5s1_gemm_$v.jsonl | cut -c1-200
done
MRAG_LIB=$R/$L/libmrag_ax.so timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s1_enc_ax.log 2>&1 || { echo "encoder tests (ax) failed"; tail -30 gpurun_out/r5s1_enc_ax.log; exit 7; }
tail -1 gpurun_out/r5s1_enc_ax.log
