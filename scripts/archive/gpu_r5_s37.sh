#!/bin/bash
# Round 5, session 37: the group host half as one library call (csrc/files.hip, NativePrepared):
# JPEG / PNG / imgprep / compat GPU tests, then the three-way ingest A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_png_gpu.py tests/test_jpeg_gpu.py tests/test_imgprep_gpu.py tests/test_compat_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5s37_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s37_tests.log; exit 3; }
tail -1 gpurun_out/r5s37_tests.log
O=gpurun_out/r5s37_native_ab.jsonl
timeout -k 10 400 python3 -u scripts/ingest_native_ab.py 2048 > $O 2> gpurun_out/r5s37.err || { echo "ab failed"; tail -20 gpurun_out/r5s37.err; exit 4; }
cat $O
