#!/bin/bash
# Session 39: K3w NB = 3 for K = 384 (MiniLM fc1): encoder suite, then the twelve tower GEMM shapes.
set -o pipefail
mkdir -p gpurun_out
P=${1:-r6s39}
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${P}_tests.log; exit 1; }
tail -1 gpurun_out/${P}_tests.log
timeout -k 10 300 python3 scripts/gemm_roofline.py 2>/dev/null | grep "^{" > gpurun_out/${P}_gemm_roofline.jsonl || { echo "roofline failed"; exit 2; }
python3 -c "
import json
for l in open('gpurun_out/${P}_gemm_roofline.jsonl'):
    d=json.loads(l); print(d['tower'], d['gemm'], d['us'], d['frac_of_bound'])"
