#!/bin/bash
# K3d CFG 2 (128 x 256): bit-identity with the default selection, then timing on the text shapes
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 150 python scripts/gemm_dump.py /tmp/c_ref.npz > gpurun_out/r2_cfg2_dump0.log 2>&1 || exit 1
MRAG_G8_CFG=2 timeout -k 10 150 python scripts/gemm_dump.py /tmp/c_new.npz > gpurun_out/r2_cfg2_dump2.log 2>&1 || exit 2
python - > gpurun_out/r2_cfg2_cmp.log 2>&1 <<'PY' || exit 3
import numpy as np
a = np.load("/tmp/c_ref.npz"); b = np.load("/tmp/c_new.npz")
bad = 0
for k in a.files:
    same = np.array_equal(a[k], b[k])
    print(k, "identical" if same else "DIFF max %.3g" % float(np.abs(a[k] - b[k]).max()))
    bad += not same
print("bad", bad)
PY
rm -f /tmp/c_ref.npz /tmp/c_new.npz
for v in 0 2; do
  MRAG_G8_CFG=$v timeout -k 10 150 python scripts/gemm_bench.py t_qkv t_out t_fc1 t_fc2 m_qkv m_out m_fc1 m_fc2 qkv fc2 > gpurun_out/r2_cfg2_bench_$v.log 2>&1 || exit 4
done
