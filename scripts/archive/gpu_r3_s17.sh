#!/bin/bash
# Round 3, session 17: image-tower fc1 as the library's swish (alpha 1.702, bias x 1.702; fc2 alpha
# 1/1.702): encoder parity tests, CLIP legs vs hand-written, the numerics printout.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py tests/test_compat_gpu.py tests/test_embedder_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s17_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r3s17_tests.log; exit 4; }
tail -12 gpurun_out/r3s17_tests.log
for round in 1 2; do
  for b in 0 1; do
    for f in 1 3; do
      MRAG_GEMM_BLASLT=$b timeout -k 10 200 python scripts/clip_bench.py 30 $f > gpurun_out/r3s17_clip.json 2>gpurun_out/r3s17_clip.err || { echo "clip $b $f failed"; tail -5 gpurun_out/r3s17_clip.err; exit 2; }
      echo "clip blaslt=$b inflight=$f $(grep -v amdgpu gpurun_out/r3s17_clip.json | cut -c1-140)" >> gpurun_out/r3s17_legs.log
    done
  done
done
cat gpurun_out/r3s17_legs.log
