#!/bin/bash
# LayerNorm RPW=2 vs 1: bit identity on all three towers, timing of CLIP and the config-5 leg
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_SYNTHETIC_WEIGHTS=1
MRAG_LN_RPW=1 timeout -k 10 200 python scripts/enc_dump.py gpurun_out/ln1.npz > gpurun_out/ln_dump1.log 2>&1 || exit 1
MRAG_LN_RPW=2 timeout -k 10 200 python scripts/enc_dump.py gpurun_out/ln2.npz > gpurun_out/ln_dump2.log 2>&1 || exit 2
python -c "
import numpy as np; a=np.load('gpurun_out/ln1.npz'); b=np.load('gpurun_out/ln2.npz')
for k in a.files: print(k, a[k].shape, 'bit-identical' if np.array_equal(a[k], b[k]) else 'DIFFER max %g' % abs(a[k]-b[k]).max())
" > gpurun_out/ln_cmp.log 2>&1 || exit 3
rm -f gpurun_out/ln1.npz gpurun_out/ln2.npz
for v in 1 2; do
MRAG_LN_RPW=$v timeout -k 10 200 python scripts/clip_bench.py 20 > gpurun_out/ln_clip$v.log 2>&1 || exit 4
MRAG_LN_RPW=$v timeout -k 10 200 python scripts/fusion_bench.py 20 > gpurun_out/ln_fus$v.log 2>&1 || exit 5
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ln_clipprof -o run -- python3 $R/scripts/clip_bench.py 10 > $R/gpurun_out/ln_clipprof.log 2>&1 || exit 6
