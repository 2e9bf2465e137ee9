#!/bin/bash
# Full GPU test suite, full bench (CPU baselines), kernel stats of the bench, smoke.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_full_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_full_tests.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/r2_full_bench.log 2>&1 || { echo "bench failed rc=$?" >> gpurun_out/r2_full_bench.log; exit 2; }
cd $R && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_full_stats -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/r2_full_stats.log 2>&1 || exit 4
