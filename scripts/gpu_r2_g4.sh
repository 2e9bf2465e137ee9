#!/bin/bash
# K3e (4-wave GEMM): bit-identity with K3d / K3 on seeded shapes, timing A/B, CLIP A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
MRAG_GEMM_4W=0 timeout -k 10 120 python scripts/gemm_dump.py /tmp/g4_ref.npz > gpurun_out/r2_g4_dump0.log 2>&1 || exit 1
MRAG_GEMM_4W=1 timeout -k 10 120 python scripts/gemm_dump.py /tmp/g4_new.npz > gpurun_out/r2_g4_dump1.log 2>&1 || exit 2
python - > gpurun_out/r2_g4_cmp.log 2>&1 <<'PY' || exit 3
import numpy as np
a = np.load("/tmp/g4_ref.npz"); b = np.load("/tmp/g4_new.npz")
bad = 0
for k in a.files:
    same = np.array_equal(a[k], b[k])
    d = float(np.abs(a[k] - b[k]).max())
    print(k, "identical" if same else "DIFF max %.3g n %d" % (d, int((a[k] != b[k]).sum())))
    bad += not same
print("bad", bad)
PY
rm -f /tmp/g4_ref.npz /tmp/g4_new.npz
for v in 0 1; do
  MRAG_GEMM_4W=$v timeout -k 10 120 python scripts/gemm_bench.py qkv fc1 fc2 out sq4k t_qkv t_fc1 > gpurun_out/r2_g4_bench_$v.log 2>&1 || exit 4
done
for v in 0 1; do
  MRAG_GEMM_4W=$v timeout -k 10 120 python scripts/clip_bench.py 10 > gpurun_out/r2_g4_clip_$v.log 2>&1 || exit 5
done
