#!/bin/bash
# final tree check: full -m gpu suite, smoke, default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/chk_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/chk_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk_smoke.log 2>&1 || exit 2
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/chk_bench.log 2>&1 || exit 3
