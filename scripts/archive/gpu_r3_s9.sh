#!/bin/bash
# Round 3, session 9 (re-entry): the tree at HEAD on a fresh box — full GPU suite, smoke, bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread > gpurun_out/r3s9_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s9_tests.log; exit 3; }
tail -1 gpurun_out/r3s9_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s9_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r3s9_smoke.log; exit 4; }
timeout -k 10 900 python bench.py > gpurun_out/r3s9_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3s9_bench.log; exit 5; }
grep '"metric"' gpurun_out/r3s9_bench.log | tail -1 > gpurun_out/r3s9_bench.json
cut -c1-1500 gpurun_out/r3s9_bench.json
