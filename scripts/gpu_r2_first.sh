#!/bin/bash
# Round-2 first GPU call: counter list, full GPU tests, full bench, kernel stats of the bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
(cd /tmp && timeout -k 5 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1) || echo "rocprofv3 -L rc=$?" >> gpurun_out/counters_list.txt
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_tests.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r2_bench.log 2>&1 || { echo "bench failed rc=$?" >> gpurun_out/r2_bench.log; exit 2; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_prof_stats -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/r2_prof_stats.log 2>&1 || exit 3
