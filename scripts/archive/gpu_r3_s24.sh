#!/bin/bash
# Round 3, session 24: hipBLASLt workspaces sized per stream; encoder tests incl. CLIP batches in
# flight across the library threshold.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_encoders_gpu.py tests/test_compat_gpu.py tests/test_configs_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s24_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s24_tests.log; exit 1; }
tail -1 gpurun_out/r3s24_tests.log
timeout -k 10 200 python scripts/clip_bench.py 30 3 | grep -v amdgpu | cut -c1-200
