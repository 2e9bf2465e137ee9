#!/bin/bash
# Round 3, session 33: K7 sample pre-pass stride for k > 16 (16 / 8 / 4), whole-search time.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for st in 16 8 4 16; do
  MRAG_K7_STRIDE_BIGK=$st KS=10,32,50,64 timeout -k 10 240 python scripts/knn_k_sweep.py >> gpurun_out/r3s33_stride.log 2>gpurun_out/r3s33.err || { echo "sweep failed"; tail -5 gpurun_out/r3s33.err; exit 2; }
done
cat gpurun_out/r3s33_stride.log
