#!/bin/bash
# theta_init coalesced loads (kNN parity + step), K3/K3d tie rule on the config-5 leg (alternating A/B)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_configs_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tie_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/tie_tests.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-clip --no-fusion > gpurun_out/tie_knn.log 2>&1 || exit 2
for r in 1 2 3; do
for v in 0 1; do
MRAG_GEMM_TIE_K3=$v timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/tie_fus${v}_$r.log 2>&1 || exit 3
done
done
