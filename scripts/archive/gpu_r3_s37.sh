#!/bin/bash
# Round 3, session 37: K8 merge with its loads in flight together (keys, rescoring rows) + wave sort: kNN tests, Q = 1 timeline, kNN bench leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_knn_gpu.py tests/test_knn_generic_gpu.py tests/test_fusion_gpu.py > gpurun_out/r3s37_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3s37_tests.log; exit 2; }
tail -1 gpurun_out/r3s37_tests.log
timeout -k 10 120 python3 scripts/q1_profile.py > gpurun_out/r3s37_plain.log 2>&1 || { echo "plain failed"; tail -5 gpurun_out/r3s37_plain.log; exit 2; }
cat gpurun_out/r3s37_plain.log
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3s37_prof -o q1 -- python3 scripts/q1_profile.py > gpurun_out/r3s37_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r3s37_prof.log; exit 3; }
f=$(find gpurun_out/r3s37_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/q1_profile.py --trace "$f" > gpurun_out/r3s37_timeline.log
rm -f "$f"
cat gpurun_out/r3s37_timeline.log
timeout -k 10 300 python bench.py --no-clip --no-fusion --no-cpu-baseline > gpurun_out/r3s37_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3s37_bench.log; exit 4; }
grep '"metric"' gpurun_out/r3s37_bench.log | tail -1 | cut -c1-200
python3 -c "import json; d=json.loads(open('gpurun_out/r3s37_bench.log').read().strip().splitlines()[-1]); print(d['config']['one_search_in_flight'], d['roofline']['avg_launch_ms'], d['call_pattern']['device_q1'])"
