#!/bin/bash
# Round 5, session 23: the encoder GEMMs alone — buffer rotation (HBM vs MALL-resident operands)
# and operand switching activity (random vs small vs zero activations: the clock the MFMA load
# holds), against the in-tower kernel times.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
O=gpurun_out/r5s23_gemm_ab.jsonl; : > $O
for a in "--sets 1 --operands randn" "--sets 3 --operands randn" "--sets 1 --operands small" "--sets 1 --operands zeros"; do
  timeout -k 10 200 python3 -u scripts/gemm_roofline.py $a --only vit_b32:qkv,vit_b32:fc2,clip_text:out,minilm:fc1 >> $O 2>> gpurun_out/r5s23.err || { echo "failed: $a"; exit 3; }
done
cat $O
