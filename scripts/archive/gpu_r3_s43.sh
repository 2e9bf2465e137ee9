#!/bin/bash
# Round 3, session 43 (final validation of the session tree: K7c sizing, big-k stride, K8 changes): full GPU suite, smoke, bench, and the
# kernel-trace summary of the bench (one search in flight).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread > gpurun_out/r3s43_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s43_tests.log; exit 3; }
tail -1 gpurun_out/r3s43_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s43_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r3s43_smoke.log; exit 4; }
timeout -k 10 900 python bench.py > gpurun_out/r3s43_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3s43_bench.log; exit 5; }
grep '"metric"' gpurun_out/r3s43_bench.log | tail -1 > gpurun_out/r3s43_bench.json
cut -c1-300 gpurun_out/r3s43_bench.json
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s43_prof -o bench -- python3 bench.py --steps 20 --knn-streams 1 --no-cpu-baseline > gpurun_out/r3s43_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r3s43_prof.log; exit 6; }
f=$(find gpurun_out/r3s43_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r3s43_kernel_stats.csv
find gpurun_out/r3s43_prof -name "*kernel_trace.csv" -delete
python3 scripts/kstats.py gpurun_out/r3s43_kernel_stats.csv > gpurun_out/r3s43_kstats.txt
head -14 gpurun_out/r3s43_kstats.txt
