#!/bin/bash
# v5 failure isolation: the seeded pre-pass test under v3 / v5 / v5 without the pre-pass
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
T="tests/test_knn_gpu.py -q -m gpu --timeout 200 --timeout-method thread -k seeded_threshold"
MRAG_SCAN_V5=0 timeout -k 10 300 python -u -m pytest $T > gpurun_out/r2_v5dbg_v3.log 2>&1; echo "v3 rc=$?" >> gpurun_out/r2_v5dbg_v3.log
MRAG_SCAN_V5=1 MRAG_SCAN_NO_SAMPLE=1 timeout -k 10 300 python -u -m pytest $T > gpurun_out/r2_v5dbg_v5ns.log 2>&1; echo "v5ns rc=$?" >> gpurun_out/r2_v5dbg_v5ns.log
MRAG_SCAN_V5=1 timeout -k 10 300 python -u -m pytest $T > gpurun_out/r2_v5dbg_v5.log 2>&1; echo "v5 rc=$?" >> gpurun_out/r2_v5dbg_v5.log
exit 0
