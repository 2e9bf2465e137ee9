#!/bin/bash
# Round validation: full GPU test suite, full bench (CPU baselines), kernel stats, K7 PMC traffic.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/round_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/round_tests.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench failed rc=$?" >> gpurun_out/bench_full.log; exit 2; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stats -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fusion > $R/gpurun_out/prof_stats.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-clip --no-fusion > $R/gpurun_out/prof_fetch.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-clip --no-fusion > $R/gpurun_out/prof_write.log 2>&1 || exit 5
cd $R && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 6
