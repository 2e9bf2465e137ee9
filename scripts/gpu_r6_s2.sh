#!/bin/bash
# Round 6 session 2: K7 with the counting sample pass (MODE 2): kNN parity suites, then the
# kNN-only bench line (one and two searches in flight) and a kernel trace of it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_configs_gpu.py tests/test_sharded_nccl_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6s2_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r6s2_tests.log; exit 3; }
tail -3 gpurun_out/r6s2_tests.log
KNN="python3 $R/bench.py --no-cpu-baseline --no-clip --no-fusion --no-call-pattern --no-retrieve-pattern --no-ingest"
timeout -k 10 300 $KNN > gpurun_out/r6s2_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r6s2_bench.log; exit 5; }
grep '"metric"' gpurun_out/r6s2_bench.log | tail -1 | cut -c1-1500
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6s2_prof -o run -- $KNN --knn-streams 1 --steps 20 > $R/gpurun_out/r6s2_prof.log 2>&1 || { echo "prof failed"; exit 6; }
cd $R
f=$(find gpurun_out/r6s2_prof -name "*kernel_trace.csv" | head -1); python3 scripts/trace_by_grid.py "$f" > gpurun_out/r6s2_by_grid.txt 2>/dev/null; head -12 gpurun_out/r6s2_by_grid.txt
find gpurun_out/r6s2_prof -name "*kernel_trace.csv" -delete
