#!/bin/bash
# Round 4, session 3: K3d stream-K timing ablations (2: no hand-off, 3: partial stores only).
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
for abl in 0 2 3 4 5; do
  MRAG_G8_SK_ABL=$abl MRAG_GEMM_BLASLT=0 timeout -k 10 200 python -u scripts/gemm_bench.py fc1 fc2 out > gpurun_out/r4s3_gemm_abl$abl.log 2>&1; rc=$?; echo "abl=$abl rc=$rc"; fatal $rc gemm
done
grep -h shape gpurun_out/r4s3_gemm_abl*.log | cut -c1-110
