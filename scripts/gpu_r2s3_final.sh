#!/bin/bash
# Round-2 session-3 validation: full GPU suite, smoke, full bench (CPU baselines), kernel stats of
# the bench with ONE search in flight (so the K7 trace durations compare with the in-bench HIP
# events), K7 HBM traffic (FETCH_SIZE / WRITE_SIZE in separate passes), CLIP + config-5 stats
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/s3f_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/s3f_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3f_smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py > gpurun_out/s3f_bench.log 2>&1 || { echo "bench failed rc=$?" >> gpurun_out/s3f_bench.log; exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s3f_stats -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --knn-streams 1 > $R/gpurun_out/s3f_stats.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-clip --no-fusion --knn-streams 1 > $R/gpurun_out/prof_fetch.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-clip --no-fusion --knn-streams 1 > $R/gpurun_out/prof_write.log 2>&1 || exit 6
