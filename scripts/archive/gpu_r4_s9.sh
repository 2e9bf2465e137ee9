#!/bin/bash
# Round 4, session 9: K3p (persistent four-stage K3) for M >= 1024: parity + A/B timing.
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_embedder_gpu.py tests/test_cross_encoder_gpu.py -q --timeout 120 --timeout-method thread -rA > gpurun_out/r4s9_enc_tests.log 2>&1; rc=$?; echo "encoder tests rc=$rc"; fatal $rc enc_tests
for v in 0 1; do
  MRAG_K3P=$v timeout -k 10 200 python -u scripts/gemm_bench.py t_out t_fc2 m_qkv m_out m_fc2 t_qkv m_fc1 > gpurun_out/r4s9_gemm_$v.log 2>&1; rc=$?; echo "gemm k3p=$v rc=$rc"; fatal $rc gemm
done
for v in 0 1 0 1; do
  MRAG_K3P=$v timeout -k 10 200 python -u scripts/text_tower_bench.py 20 >> gpurun_out/r4s9_text.log 2>>gpurun_out/r4s9_text.err; rc=$?; echo "text k3p=$v rc=$rc"; fatal $rc text
done
for v in 0 1; do
  MRAG_K3P=$v timeout -k 10 300 python -u scripts/fusion_bench.py 20 > gpurun_out/r4s9_fusion_$v.json 2>>gpurun_out/r4s9_text.err; rc=$?; echo "fusion k3p=$v rc=$rc"; fatal $rc fusion
done
grep -E "passed|failed" gpurun_out/r4s9_enc_tests.log | tail -2; grep FAILED gpurun_out/r4s9_enc_tests.log | head
for v in 0 1; do echo "k3p=$v"; grep -h shape gpurun_out/r4s9_gemm_$v.log | cut -c1-110; done
cat gpurun_out/r4s9_text.log
for v in 0 1; do python3 -c "import json; d=json.load(open('gpurun_out/r4s9_fusion_$v.json')); print('fusion $v', d.get('value'), d.get('one_step_in_flight'))"; done
