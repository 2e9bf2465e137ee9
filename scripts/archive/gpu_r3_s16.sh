#!/bin/bash
# Round 3, session 16: the tree with hipBLASLt for the plain encoder GEMMs at M >= 4096 (default):
# full GPU suite, smoke, bench, kernel-trace stats of the bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread > gpurun_out/r3s16_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s16_tests.log; exit 3; }
tail -1 gpurun_out/r3s16_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s16_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r3s16_smoke.log; exit 4; }
timeout -k 10 900 python bench.py > gpurun_out/r3s16_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3s16_bench.log; exit 5; }
grep '"metric"' gpurun_out/r3s16_bench.log | tail -1 > gpurun_out/r3s16_bench.json
cut -c1-400 gpurun_out/r3s16_bench.json
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s16_prof -o bench -- python3 bench.py --steps 20 --knn-streams 1 --no-cpu-baseline > gpurun_out/r3s16_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r3s16_prof.log; exit 6; }
f=$(find gpurun_out/r3s16_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r3s16_kernel_stats.csv
find gpurun_out/r3s16_prof -name "*kernel_trace.csv" -size +20M -delete
python3 scripts/kstats.py gpurun_out/r3s16_kernel_stats.csv | head -16
