#!/bin/bash
# K8 register top-64P selection: kNN parity, then K8 time (kernel stats) and bench A/B vs the sort
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_generic_gpu.py tests/test_compat_gpu.py tests/test_configs_gpu.py tests/test_fusion_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_k8sel_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_k8sel_tests.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  MRAG_K8_SORT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_k8sel_$v -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-clip --no-fusion > $R/gpurun_out/r2_k8sel_$v.log 2>&1 || exit 2
done
