#!/bin/bash
# Round 3, session 8: streaming LayerNorm (MRAG_LN_WPC workgroups per CU) vs one row per wave:
# bit identity of all three towers, LN kernel times (kernel trace of the CLIP and config-5 legs),
# CLIP img/s one batch in flight, config-5 q/s.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 0 1 2; do
  MRAG_G8_CFG=$c timeout -k 10 200 python scripts/gemm_bench.py qkv fc1 fc2 out t_qkv t_fc1 t_fc2 m_fc1 > gpurun_out/r3s8_gemm_cfg$c.log 2>&1 || { echo "gemm cfg=$c failed"; tail -5 gpurun_out/r3s8_gemm_cfg$c.log; exit 9; }
  echo "== G8_CFG=$c"; grep -v amdgpu.ids gpurun_out/r3s8_gemm_cfg$c.log
done
MRAG_G8_CFG=2 timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3s8_tests_cfg2.log 2>&1 || { echo "cfg2 encoder tests failed"; tail -30 gpurun_out/r3s8_tests_cfg2.log; exit 8; }
tail -1 gpurun_out/r3s8_tests_cfg2.log
for w in 0 2 4 8; do
  MRAG_LN_WPC=$w timeout -k 10 200 python scripts/enc_dump.py gpurun_out/r3s8_enc_$w.npz > gpurun_out/r3s8_dump_$w.log 2>&1 || { echo "dump $w failed"; tail -5 gpurun_out/r3s8_dump_$w.log; exit 1; }
done
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/r3s8_enc_0.npz")
for w in (2, 4, 8):
    b = np.load(f"gpurun_out/r3s8_enc_{w}.npz")
    print("wpc", w, {k: bool(np.array_equal(a[k], b[k])) for k in a.files})
PY
for w in 0 4 8 2; do
  MRAG_LN_WPC=$w timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s8_prof_$w -o p -- python3 scripts/clip_bench.py 10 1 > gpurun_out/r3s8_clip_$w.log 2>&1 || { echo "clip prof $w failed"; tail -5 gpurun_out/r3s8_clip_$w.log; exit 2; }
  f=$(find gpurun_out/r3s8_prof_$w -name "*kernel_stats.csv" | head -1); echo "== wpc $w"; grep -i "layernorm" "$f" | cut -d, -f1-4
  find gpurun_out/r3s8_prof_$w -name "*kernel_trace.csv" -delete
done
for c in 0 1 0 1; do
  MRAG_G8_CFG=$c timeout -k 10 200 python scripts/clip_bench.py 30 1 | tail -1 | cut -c1-200 | sed "s/^/cfg $c clip1 /"
  MRAG_G8_CFG=$c timeout -k 10 200 python scripts/clip_bench.py 30 3 | tail -1 | cut -c1-200 | sed "s/^/cfg $c clip3 /"
done
for w in 0 4 0 4; do
  MRAG_LN_WPC=$w timeout -k 10 200 python scripts/clip_bench.py 30 1 | tail -1 | cut -c1-200 | sed "s/^/wpc $w clip1 /"
  MRAG_LN_WPC=$w timeout -k 10 200 python scripts/fusion_bench.py 20 | tail -1 | cut -c1-160 | sed "s/^/wpc $w fusion /"
done
