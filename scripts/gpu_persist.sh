#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_compat_gpu.py -x -q -m gpu > gpurun_out/persist_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/persist_tests.log; exit 1; }
