#!/bin/bash
# K7 v2 round: parity (v2 default + forced v1), then kNN-only bench A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_knn_gpu.py tests/test_compat_gpu.py -x -q -m gpu > gpurun_out/knn_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/knn_tests.log; exit 1; }
if [ "${V1TESTS:-0}" = "1" ]; then
MRAG_SCAN_V1=1 timeout -k 10 400 python -m pytest tests/test_knn_gpu.py -x -q -m gpu > gpurun_out/knn_tests_v1.log 2>&1 || { echo "pytest v1 failed" >> gpurun_out/knn_tests_v1.log; exit 1; }
fi
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip > gpurun_out/bench_v2.log 2>&1 || exit 2
MRAG_SCAN_NO_SAMPLE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip > gpurun_out/bench_v2ns.log 2>&1 || exit 3
MRAG_SCAN_V1=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip > gpurun_out/bench_v1.log 2>&1 || exit 3
if [ "${PROF:-0}" = "1" ]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_knn -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip > $R/gpurun_out/prof_knn.log 2>&1 || exit 4
fi
