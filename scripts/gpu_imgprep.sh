#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_imgprep_gpu.py tests/test_compat_gpu.py -x -q -m gpu > gpurun_out/imgprep_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/imgprep_tests.log; exit 1; }
timeout -k 10 300 python scripts/imgprep_bench.py > gpurun_out/imgprep_bench.log 2>&1 || exit 2
