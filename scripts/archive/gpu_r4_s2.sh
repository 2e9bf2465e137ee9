#!/bin/bash
# Round 4, session 2: K3d stream-K with per-quadrant partial loads: parity + timing vs the library.
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_encoders_gpu.py -q --timeout 120 --timeout-method thread -k "gemm" -rA > gpurun_out/r4s2_gemm_tests.log 2>&1; rc=$?; echo "gemm tests rc=$rc"; fatal $rc gemm_tests
for lib in 0 1; do
  MRAG_GEMM_BLASLT=$lib timeout -k 10 200 python -u scripts/gemm_bench.py qkv fc1 fc2 out > gpurun_out/r4s2_gemm_lib$lib.log 2>&1; rc=$?; echo "gemm lib=$lib rc=$rc"; fatal $rc gemm
done
for inf in 1 3; do
  MRAG_GEMM_BLASLT=0 timeout -k 10 200 python -u scripts/clip_bench.py 30 $inf > gpurun_out/r4s2_clip_lib0_inf$inf.json 2>gpurun_out/r4s2_clip.err; rc=$?; echo "clip inf=$inf rc=$rc"; fatal $rc clip
done
tail -5 gpurun_out/r4s2_gemm_tests.log
cat gpurun_out/r4s2_gemm_lib*.log gpurun_out/r4s2_clip_lib0_inf*.json
