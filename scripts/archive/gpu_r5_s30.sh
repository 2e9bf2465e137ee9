#!/bin/bash
# Round 5, session 30: K13 on damaged files as Pillow (libjpeg's insufficient-data rule, truncated
# files refused, restart markers in order); JPEG / PNG tests and the decode timing.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jpeg_gpu.py tests/test_png_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s30_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s30_tests.log; exit 3; }
tail -1 gpurun_out/r5s30_tests.log
timeout -k 10 300 python3 -u scripts/jpeg_bench.py 1024 > gpurun_out/r5s30_jpeg_bench.json 2>gpurun_out/r5s30.err || { echo "jpeg bench failed"; tail -20 gpurun_out/r5s30.err; exit 4; }
cat gpurun_out/r5s30_jpeg_bench.json
