#!/bin/bash
# Round 4, session 1: kNN collect-pass diagnosis, kNN GPU tests, K3d stream-K parity, CLIP/GEMM
# library vs hand-written A/B.
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 400 python -u scripts/knn_collect_diag.py > gpurun_out/r4s1_diag.log 2>&1; rc=$?; echo "diag rc=$rc"; fatal $rc diag
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py -q --timeout 120 --timeout-method thread -rA > gpurun_out/r4s1_knn_tests.log 2>&1; rc=$?; echo "knn tests rc=$rc"; fatal $rc knn_tests
timeout -k 10 300 python -u -m pytest tests/test_encoders_gpu.py -q --timeout 120 --timeout-method thread -k "gemm_shapes_every_epilogue" -rA > gpurun_out/r4s1_gemm_tests.log 2>&1; rc=$?; echo "gemm tests rc=$rc"; fatal $rc gemm_tests
for lib in 0 1; do
  MRAG_GEMM_BLASLT=$lib timeout -k 10 200 python -u scripts/gemm_bench.py qkv fc1 fc2 out > gpurun_out/r4s1_gemm_lib$lib.log 2>&1; rc=$?; echo "gemm lib=$lib rc=$rc"; fatal $rc gemm
  for inf in 1 3; do
    MRAG_GEMM_BLASLT=$lib timeout -k 10 200 python -u scripts/clip_bench.py 30 $inf > gpurun_out/r4s1_clip_lib${lib}_inf$inf.json 2>gpurun_out/r4s1_clip.err; rc=$?; echo "clip lib=$lib inf=$inf rc=$rc"; fatal $rc clip
  done
done
tail -c 6000 gpurun_out/r4s1_diag.log
tail -25 gpurun_out/r4s1_knn_tests.log
tail -5 gpurun_out/r4s1_gemm_tests.log
cat gpurun_out/r4s1_gemm_lib*.log gpurun_out/r4s1_clip_lib*.json
