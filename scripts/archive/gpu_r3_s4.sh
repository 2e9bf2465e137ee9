#!/bin/bash
# Round 3, session 4: K3d with compile-time steady-state waits (GEMM shapes + digests vs r3s3),
# K7 defaults after the A/B (guard only on masked tiles, no K7s pre-pass), encoder + kNN GPU tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 200 python scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_fc1 t_fc2 m_fc1 > gpurun_out/r3s4_gemm.log 2>&1 || { echo "gemm_bench failed"; tail -5 gpurun_out/r3s4_gemm.log; exit 1; }
timeout -k 10 120 python scripts/knn_scan_ab.py 30 > gpurun_out/r3s4_k7.log 2>&1 || { echo "knn ab failed"; tail -5 gpurun_out/r3s4_k7.log; exit 2; }
timeout -k 10 900 python -u -m pytest tests/test_encoders_gpu.py tests/test_knn_gpu.py tests/test_compat_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3s4_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s4_tests.log; exit 3; }
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r3s4_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3s4_bench.log; exit 4; }
grep -v amdgpu.ids gpurun_out/r3s4_gemm.log gpurun_out/r3s4_k7.log; tail -3 gpurun_out/r3s4_tests.log; tail -c 1500 gpurun_out/r3s4_bench.log
