#!/bin/bash
# Round 4, session 6: CLIP hand-written data-parallel (no stream-K) vs stream-K vs library, one box.
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
for v in "-1 0" "0 0" "0 1"; do
  set -- $v
  for inf in 1 3; do
    MRAG_G8_SK_ABL=$1 MRAG_GEMM_BLASLT=$2 timeout -k 10 200 python -u scripts/clip_bench.py 30 $inf > gpurun_out/r4s6_clip_sk$1_lib$2_inf$inf.json 2>>gpurun_out/r4s6_clip.err; rc=$?; echo "clip sk=$1 lib=$2 inf=$inf rc=$rc"; fatal $rc clip
  done
done
MRAG_G8_SK_ABL=-1 MRAG_GEMM_BLASLT=0 timeout -k 10 200 python -u scripts/gemm_bench.py qkv fc1 fc2 out > gpurun_out/r4s6_gemm_dp.log 2>&1; rc=$?; echo "gemm dp rc=$rc"; fatal $rc gemm
for f in gpurun_out/r4s6_clip_*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_batch'])")"; done
grep -h shape gpurun_out/r4s6_gemm_dp.log | cut -c1-100
