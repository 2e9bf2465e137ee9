#!/bin/bash
# K7g tests + the fused kNN tests
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_knn_generic_gpu.py tests/test_knn_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_k7g_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_k7g_tests.log; exit 2; }
