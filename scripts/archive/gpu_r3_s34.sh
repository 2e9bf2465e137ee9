#!/bin/bash
# Round 3, session 34: K7c sized to the failing queries (failure count read after K8) and the
# k > 16 sample stride 4: kNN GPU tests, the k sweep, the config-5 leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_knn_gpu.py tests/test_knn_generic_gpu.py tests/test_fusion_gpu.py tests/test_configs_gpu.py > gpurun_out/r3s34_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3s34_tests.log; exit 2; }
tail -3 gpurun_out/r3s34_tests.log
timeout -k 10 240 python scripts/knn_k_sweep.py > gpurun_out/r3s34_sweep.log 2>gpurun_out/r3s34.err || { echo "sweep failed"; tail -5 gpurun_out/r3s34.err; exit 2; }
cat gpurun_out/r3s34_sweep.log
for i in 1 2; do
timeout -k 10 300 python scripts/fusion_bench.py 24 > gpurun_out/r3s34_fusion.json 2>gpurun_out/r3s34_fusion.err || { echo "fusion failed"; tail -5 gpurun_out/r3s34_fusion.err; exit 2; }
grep -v amdgpu gpurun_out/r3s34_fusion.json | cut -c1-400
done
