#!/bin/bash
# last-layer pooled-row pruning: bit identity vs the full last layer, encoder/config parity, timing
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
MRAG_ENC_FULL_LAST=1 timeout -k 10 200 python scripts/enc_dump.py gpurun_out/pr1.npz > gpurun_out/pr_dump1.log 2>&1 || exit 1
timeout -k 10 200 python scripts/enc_dump.py gpurun_out/pr2.npz > gpurun_out/pr_dump2.log 2>&1 || exit 2
python -c "
import numpy as np; a=np.load('gpurun_out/pr1.npz'); b=np.load('gpurun_out/pr2.npz')
for k in a.files: print(k, a[k].shape, 'bit-identical' if np.array_equal(a[k], b[k]) else 'DIFFER max %g' % abs(a[k]-b[k]).max())
" > gpurun_out/pr_cmp.log 2>&1 || exit 3
rm -f gpurun_out/pr1.npz gpurun_out/pr2.npz
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py tests/test_embedder_gpu.py tests/test_compat_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pr_tests.log 2>&1 || { echo "pytest failed" >> gpurun_out/pr_tests.log; exit 4; }
for v in 1 0; do
MRAG_ENC_FULL_LAST=$v timeout -k 10 200 python scripts/clip_bench.py 20 > gpurun_out/pr_clip$v.log 2>&1 || exit 5
MRAG_ENC_FULL_LAST=$v timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/pr_fus$v.log 2>&1 || exit 6
done
