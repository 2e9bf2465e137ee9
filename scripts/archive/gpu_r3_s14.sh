#!/bin/bash
# Round 3, session 14: plain encoder GEMMs (bias / residual / f32) on hipBLASLt (MRAG_GEMM_BLASLT=1,
# M >= 4096) vs K3 / K3d: per-shape timings + determinism, CLIP one and three batches in flight,
# config-5 leg, encoder parity tests under hipBLASLt.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for b in 0 1; do
  MRAG_GEMM_BLASLT=$b timeout -k 10 200 python scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_out t_fc1 t_fc2 m_qkv m_out m_fc1 m_fc2 >> gpurun_out/r3s14_gemm.log 2>&1 || { echo "gemm $b failed"; tail -5 gpurun_out/r3s14_gemm.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r3s14_gemm.log | cut -c1-260
for round in 1 2; do
  for b in 0 1; do
    for f in 1 3; do
      MRAG_GEMM_BLASLT=$b timeout -k 10 200 python scripts/clip_bench.py 30 $f > gpurun_out/r3s14_clip_$b_$f.json 2>gpurun_out/r3s14_clip.err || { echo "clip $b $f failed"; tail -5 gpurun_out/r3s14_clip.err; exit 2; }
      echo "blaslt=$b inflight=$f $(grep -v amdgpu gpurun_out/r3s14_clip_$b_$f.json | cut -c1-200)"
    done
  done
done
for b in 0 1; do
  MRAG_GEMM_BLASLT=$b timeout -k 10 300 python scripts/fusion_bench.py 20 > gpurun_out/r3s14_fusion_$b.json 2>gpurun_out/r3s14_fusion.err || { echo "fusion $b failed"; tail -5 gpurun_out/r3s14_fusion.err; exit 3; }
  echo "blaslt=$b $(grep -v amdgpu gpurun_out/r3s14_fusion_$b.json | cut -c1-300)"
done
MRAG_GEMM_BLASLT=1 timeout -k 10 900 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py tests/test_compat_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s14_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s14_tests.log; exit 4; }
tail -2 gpurun_out/r3s14_tests.log
