#!/bin/bash
# kNN round on the GPU box: parity tests, bench (normal + epilogue ablation), rocprof kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 400 python -m pytest tests/test_knn_gpu.py -x -q -m gpu > gpurun_out/knn_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/knn_tests.log; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_norm.log 2>&1 || exit 2
MRAG_SCAN_ABLATE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ablate.log 2>&1 || exit 3
MRAG_SCAN_ABLATE=2 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ablate2.log 2>&1 || exit 3
if [ "${PROF:-0}" = "1" ]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_knn -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_knn.log 2>&1 || exit 4
fi
