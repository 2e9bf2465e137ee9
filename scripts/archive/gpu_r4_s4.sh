#!/bin/bash
# Round 4, session 4: batched residual epilogues (K3, K3d, SK reader): parity + timing.
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py -q --timeout 120 --timeout-method thread -rA > gpurun_out/r4s4_enc_tests.log 2>&1; rc=$?; echo "encoder tests rc=$rc"; fatal $rc enc_tests
for lib in 0 1; do
  MRAG_GEMM_BLASLT=$lib timeout -k 10 200 python -u scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_out t_fc1 t_fc2 m_qkv m_out m_fc1 m_fc2 > gpurun_out/r4s4_gemm_lib$lib.log 2>&1; rc=$?; echo "gemm lib=$lib rc=$rc"; fatal $rc gemm
done
for inf in 1 3; do
  MRAG_GEMM_BLASLT=0 timeout -k 10 200 python -u scripts/clip_bench.py 30 $inf > gpurun_out/r4s4_clip_lib0_inf$inf.json 2>gpurun_out/r4s4_clip.err; rc=$?; echo "clip inf=$inf rc=$rc"; fatal $rc clip
done
MRAG_GEMM_BLASLT=1 timeout -k 10 200 python -u scripts/clip_bench.py 30 3 > gpurun_out/r4s4_clip_lib1_inf3.json 2>>gpurun_out/r4s4_clip.err; rc=$?; echo "clip lib1 rc=$rc"; fatal $rc clip
tail -3 gpurun_out/r4s4_enc_tests.log
grep -h shape gpurun_out/r4s4_gemm_lib*.log | cut -c1-100
cat gpurun_out/r4s4_clip_lib*.json | cut -c1-200
