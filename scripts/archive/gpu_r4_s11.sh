#!/bin/bash
# Round 4, session 11: LayerNorm folded into the GEMMs (EPI_FOLD / EPI_STATS / EPI_RESLN):
# encoder parity, then text towers, config-5 leg, CLIP image tower, and a kernel trace of a
# text-tower pass (no standalone LayerNorm expected but the last BERT one).
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 200 python -u scripts/gemm_ln_check.py > gpurun_out/r4s11_lncheck.log 2>&1 && timeout -k 10 200 python -u scripts/fold_debug.py >> gpurun_out/r4s11_lncheck.log 2>&1; rc=$?; echo "lncheck rc=$rc"; fatal $rc lncheck
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_embedder_gpu.py tests/test_cross_encoder_gpu.py -q --timeout 120 --timeout-method thread -rA > gpurun_out/r4s11_enc_tests.log 2>&1; rc=$?; echo "encoder tests rc=$rc"; fatal $rc enc_tests
grep -E "passed|failed" gpurun_out/r4s11_enc_tests.log | tail -2; grep FAILED gpurun_out/r4s11_enc_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for v in 1 2; do
  timeout -k 10 200 python -u scripts/text_tower_bench.py 20 >> gpurun_out/r4s11_text.log 2>>gpurun_out/r4s11_text.err; rc=$?; echo "text rc=$rc"; fatal $rc text
done
timeout -k 10 300 python -u scripts/fusion_bench.py 20 > gpurun_out/r4s11_fusion.json 2>>gpurun_out/r4s11_text.err; rc=$?; echo "fusion rc=$rc"; fatal $rc fusion
timeout -k 10 300 python -u scripts/clip_bench.py 20 3 > gpurun_out/r4s11_clip.json 2>>gpurun_out/r4s11_text.err; rc=$?; echo "clip rc=$rc"; fatal $rc clip
timeout -k 10 300 python -u scripts/clip_bench.py 20 1 >> gpurun_out/r4s11_clip.json 2>>gpurun_out/r4s11_text.err; rc=$?; echo "clip1 rc=$rc"; fatal $rc clip1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4s11_prof -o fus -- python3 scripts/fusion_bench.py 5 > gpurun_out/r4s11_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; fatal $rc prof
cat gpurun_out/r4s11_text.log
cat gpurun_out/r4s11_fusion.json | cut -c1-600
cat gpurun_out/r4s11_clip.json | cut -c1-400
find gpurun_out/r4s11_prof -name "*kernel_stats.csv" | head -3
