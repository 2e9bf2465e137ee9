#!/bin/bash
# Round 4, session 8: K3r (residual GEMM + LayerNorm fused) in the text towers: parity + A/B timing.
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_embedder_gpu.py tests/test_cross_encoder_gpu.py -q --timeout 120 --timeout-method thread -rA > gpurun_out/r4s8_enc_tests.log 2>&1; rc=$?; echo "encoder tests rc=$rc"; fatal $rc enc_tests
for v in 0 1 0 1; do
  MRAG_ROWLN=$v timeout -k 10 200 python -u scripts/text_tower_bench.py 20 >> gpurun_out/r4s8_text.log 2>>gpurun_out/r4s8_text.err; rc=$?; echo "text rowln=$v rc=$rc"; fatal $rc text
done
for v in 0 1; do
  MRAG_ROWLN=$v timeout -k 10 300 python -u scripts/fusion_bench.py 20 > gpurun_out/r4s8_fusion_$v.json 2>>gpurun_out/r4s8_text.err; rc=$?; echo "fusion rowln=$v rc=$rc"; fatal $rc fusion
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4s8_prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/text_tower_bench.py 10 > $GRAFT_REPO_ROOT/gpurun_out/r4s8_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; cd $GRAFT_REPO_ROOT
grep -E "passed|failed" gpurun_out/r4s8_enc_tests.log | tail -2; grep FAILED gpurun_out/r4s8_enc_tests.log | head
cat gpurun_out/r4s8_text.log
for v in 0 1; do python3 -c "import json; d=json.load(open('gpurun_out/r4s8_fusion_$v.json')); print('fusion $v', d.get('value'), d.get('one_step_in_flight'))"; done
f=$(find gpurun_out/r4s8_prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 scripts/kstats.py $f 10 | head -20
