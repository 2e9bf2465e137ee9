#!/bin/bash
# retrieve_batch with the image branch in a worker thread: drop-in parity tests
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 600 python -u -m pytest tests/test_compat_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_rb_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_rb_tests.log; exit 1; }
