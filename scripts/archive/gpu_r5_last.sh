#!/bin/bash
# Round 5, last tree (after the pinned-arena ingest staging, 8f0db95): the full GPU suite, smoke
# and the driver's bench line only (K7 and the encoders are unchanged since the r5_final traces).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/r5k_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r5k_tests.log; exit 3; }
tail -1 gpurun_out/r5k_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5k_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r5k_smoke.log; exit 4; }
timeout -k 10 900 python -u bench.py > gpurun_out/r5k_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r5k_bench.log; exit 5; }
grep '"metric"' gpurun_out/r5k_bench.log | tail -1 > gpurun_out/r5k_bench.json
cut -c1-900 gpurun_out/r5k_bench.json
