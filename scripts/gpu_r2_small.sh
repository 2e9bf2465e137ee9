#!/bin/bash
# small-kernel rewrites (LN one butterfly, token embed, l2norm compile-time tree, K12 wave per
# query): encoder / fusion / l2norm parity, then config-5 and CLIP timings
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
timeout -k 10 900 python -u -m pytest tests/test_encoders_gpu.py tests/test_fusion_gpu.py tests/test_configs_gpu.py tests/test_embedder_gpu.py tests/test_knn_gpu.py -k "not full_size and not seeded and not clustered" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2_small_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/r2_small_tests.log; exit 1; }
timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/r2_small_fus.log 2>&1 || exit 2
timeout -k 10 200 python scripts/clip_bench.py 10 > gpurun_out/r2_small_clip.log 2>&1 || exit 3
