#!/bin/bash
# Round 3, session 40: K8 phase stamps of the merge variants (base / ins / resc / wsort / all).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
for round in 1 2; do
for v in base ins resc wsort all; do
  MRAG_LIB=$L/libmrag_k7stamp_$v.so timeout -k 10 200 python scripts/k8_stamps.py >> gpurun_out/r3s40_k8.log 2>gpurun_out/r3s40.err || { echo "$v failed"; tail -5 gpurun_out/r3s40.err; exit 2; }
done
done
cat gpurun_out/r3s40_k8.log
