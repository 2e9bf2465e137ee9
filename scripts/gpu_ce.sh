#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_cross_encoder_gpu.py tests/test_encoders_gpu.py tests/test_compat_gpu.py -x -q -m gpu > gpurun_out/ce_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/ce_tests.log; exit 1; }
