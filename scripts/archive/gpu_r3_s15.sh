#!/bin/bash
# Round 3, session 15: hipBLASLt for the plain and quick_gelu (swish slope 1.702) encoder GEMMs at
# K >= 768, M >= 4096 (MRAG_GEMM_BLASLT=1, the new default) vs hand-written only (0) vs every
# eligible call (2): per-shape timings, errors vs a torch fp32 reference, determinism; CLIP one /
# three batches in flight; config-5 leg; encoder / config / compat parity tests at the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for b in 0 1 2; do
  MRAG_GEMM_BLASLT=$b timeout -k 10 200 python scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_out t_fc1 t_fc2 m_qkv m_out m_fc1 m_fc2 >> gpurun_out/r3s15_gemm.log 2>&1 || { echo "gemm $b failed"; tail -5 gpurun_out/r3s15_gemm.log; exit 1; }
done
for round in 1 2; do
  for b in 0 1 2; do
    for f in 1 3; do
      MRAG_GEMM_BLASLT=$b timeout -k 10 200 python scripts/clip_bench.py 30 $f > gpurun_out/r3s15_clip.json 2>gpurun_out/r3s15_clip.err || { echo "clip $b $f failed"; tail -5 gpurun_out/r3s15_clip.err; exit 2; }
      echo "clip blaslt=$b inflight=$f $(grep -v amdgpu gpurun_out/r3s15_clip.json | cut -c1-140)" >> gpurun_out/r3s15_legs.log
    done
    MRAG_GEMM_BLASLT=$b timeout -k 10 300 python scripts/fusion_bench.py 20 > gpurun_out/r3s15_fusion.json 2>gpurun_out/r3s15_fusion.err || { echo "fusion $b failed"; tail -5 gpurun_out/r3s15_fusion.err; exit 3; }
    echo "fusion blaslt=$b $(grep -v amdgpu gpurun_out/r3s15_fusion.json | cut -c1-140)" >> gpurun_out/r3s15_legs.log
  done
done
cat gpurun_out/r3s15_legs.log
timeout -k 10 900 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py tests/test_compat_gpu.py tests/test_embedder_gpu.py tests/test_cross_encoder_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s15_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s15_tests.log; exit 4; }
tail -2 gpurun_out/r3s15_tests.log
