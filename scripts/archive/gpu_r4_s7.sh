#!/bin/bash
# Round 4, session 7: hand-written GEMMs only (hipBLASLt and stream-K removed): full GPU suite,
# smoke, CLIP 1 / 3 in flight, GEMM shapes.
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rA > gpurun_out/r4s7_gpu_tests.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; fatal $rc gpu_tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4s7_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; fatal $rc smoke
for inf in 1 3; do
  timeout -k 10 200 python -u scripts/clip_bench.py 30 $inf > gpurun_out/r4s7_clip_inf$inf.json 2>>gpurun_out/r4s7_clip.err; rc=$?; echo "clip inf=$inf rc=$rc"; fatal $rc clip
done
timeout -k 10 200 python -u scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_out t_fc1 t_fc2 m_qkv m_out m_fc1 m_fc2 > gpurun_out/r4s7_gemm.log 2>&1; rc=$?; echo "gemm rc=$rc"; fatal $rc gemm
grep -E "passed|failed" gpurun_out/r4s7_gpu_tests.log | tail -3
grep FAILED gpurun_out/r4s7_gpu_tests.log | head
tail -2 gpurun_out/r4s7_smoke.log
for f in gpurun_out/r4s7_clip_inf*.json; do echo "$f $(python3 -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_batch'])")"; done
grep -h shape gpurun_out/r4s7_gemm.log | cut -c1-100
