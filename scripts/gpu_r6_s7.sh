#!/bin/bash
# Round 6 session 7: K3w with the epilogue stores left in flight across the tile barrier and the
# weight loads overlapping the first tile's fill: bit identity, probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encoders_gpu.py -x -q -m gpu -k weight_stationary --timeout 240 --timeout-method thread > gpurun_out/r6s7_ws.log 2>&1 || { echo "K3w test failed"; tail -30 gpurun_out/r6s7_ws.log; exit 3; }
tail -1 gpurun_out/r6s7_ws.log
for s in "1536 512 0" "2048 512 1" "1152 384 0" "1536 384 2"; do
  timeout -k 10 200 python3 scripts/gemm_ws_probe.py $s >> gpurun_out/r6s7_probe.jsonl 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r6s7_probe.jsonl; exit 2; }
done
grep '^{' gpurun_out/r6s7_probe.jsonl | grep -v '"M": 2560'
