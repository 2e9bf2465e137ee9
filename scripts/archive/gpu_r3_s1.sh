#!/bin/bash
# Round 3, first check: GPU suite (incl. full-size C4 / C5, workspace regrowth, null-stream
# ordering, text-tower pools), smoke, call-pattern A/B (K7s vs the 256-query scan), bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3s1_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r3s1_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s1_smoke.log 2>&1 || exit 2
timeout -k 10 200 python scripts/knn_call_pattern.py > gpurun_out/r3s1_cp_k7s.log 2>&1 || exit 3
MRAG_SCAN_SMALLQ=0 timeout -k 10 200 python scripts/knn_call_pattern.py > gpurun_out/r3s1_cp_k7.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r3s1_bench.log 2>&1 || { echo "bench failed rc=$?" >> gpurun_out/r3s1_bench.log; exit 5; }
