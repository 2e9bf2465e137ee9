#!/bin/bash
# Round 3, session 5: K7 group test on v_max3 + cached threshold, label read at the tile tail,
# five A-fragment buffers, A/B against the previous commit (lib/libmrag_base.so); K7 stamps;
# K3f (register-staged 4-wave GEMM, pinned AGPR accumulators) vs K3d; kNN + encoder tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
for k in 0 1 2; do
  MRAG_GEMM_K3F=$k timeout -k 10 200 python scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_fc1 t_fc2 m_fc1 > gpurun_out/r3s5_gemm_k3f$k.log 2>&1 || { echo "gemm k3f=$k failed"; tail -5 gpurun_out/r3s5_gemm_k3f$k.log; exit 1; }
done
for round in 1 2; do
  for lib in libmrag_base.so libmrag.so; do
    MRAG_LIB=$L/$lib timeout -k 10 120 python scripts/knn_scan_ab.py 30 >> gpurun_out/r3s5_ab.log 2>&1 || { echo "ab $lib failed"; tail -5 gpurun_out/r3s5_ab.log; exit 2; }
  done
done
MRAG_LIB=$L/libmrag_k7stamp.so timeout -k 10 120 python scripts/k7_stamps.py > gpurun_out/r3s5_stamps.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/r3s5_stamps.log; exit 3; }
for k in 0 1 2; do echo "== K3F=$k"; grep -v amdgpu.ids gpurun_out/r3s5_gemm_k3f$k.log; done
grep -v amdgpu.ids gpurun_out/r3s5_ab.log gpurun_out/r3s5_stamps.log
MRAG_GEMM_K3F=1 timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3s5_tests_k3f.log 2>&1 || { echo "k3f encoder tests failed"; tail -30 gpurun_out/r3s5_tests_k3f.log; exit 4; }
timeout -k 10 900 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_generic_gpu.py tests/test_full_configs_gpu.py tests/test_encoders_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s5_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s5_tests.log; exit 5; }
tail -2 gpurun_out/r3s5_tests_k3f.log gpurun_out/r3s5_tests.log
