#!/bin/bash
# Round 5, session 9: the two query encodes of _get_embeddings overlapped (CLIP text on a worker
# thread and its own stream). Compat tests, then the bench's retrieve leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_compat_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s9_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r5s9_tests.log; exit 3; }
tail -1 gpurun_out/r5s9_tests.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-clip --no-fusion --no-ingest > gpurun_out/r5s9_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5s9_bench.log; exit 4; }
grep '"metric"' gpurun_out/r5s9_bench.log | tail -1 > gpurun_out/r5s9_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r5s9_bench.json'))
print(json.dumps(d.get('call_pattern',{}).get('retrieve')))"
