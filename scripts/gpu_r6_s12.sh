#!/bin/bash
# Round 6 session 12: K3w output image, unit u of row j at u ^ (j & 15). Bit-identity tests,
# the twelve tower GEMM shapes (scripts/gemm_roofline.py) with this library and the previous one
# (libmrag_k3wold), LDS conflict counters of K3w, and the config-5 leg interleaved.
P=r6s12
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=$R/multimodal-rag-for-image-text-search_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py -x -v --timeout 300 --timeout-method thread -k "weight_stationary or gelu or golden or skinny" > gpurun_out/${P}_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${P}_tests.log; exit 3; }
tail -1 gpurun_out/${P}_tests.log
for lib in libmrag libmrag_k3wold; do
  MRAG_LIB=$L/$lib.so timeout -k 10 300 python3 scripts/gemm_roofline.py 2>/dev/null | grep '^{' | sed "s/^{/{\"lib\": \"$lib\", /" >> gpurun_out/${P}_gemm.jsonl || { echo "roofline failed $lib"; exit 4; }
done
python3 - gpurun_out/${P}_gemm.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["lib"], d["tower"], d["gemm"], d["us"], d["tflops"], d["bound"], d["frac_of_bound"])
PY
cd /tmp && export TMPDIR=/tmp
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
i=0
for PP in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PP --output-format csv -d $R/gpurun_out/${P}_p$i -o run -- python3 $R/scripts/gemm_ws_probe.py 1536 512 0 k3w 16000 > $R/gpurun_out/${P}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/${P}_p$i.log; exit $((10+i)); }
done
cd $R && python3 scripts/pmc_kernels.py gpurun_out/${P}_pmc.json gpurun_out/${P}_p1 gpurun_out/${P}_p2 || exit 21
rm -rf gpurun_out/${P}_p1 gpurun_out/${P}_p2
python3 -c "
import json; d=json.load(open('gpurun_out/${P}_pmc.json'))
for r in d['kernels'][:2]: print(r['kernel'][:50], 'mfma', r.get('mfma_busy_frac'), 'lds_conflict', r.get('lds_conflict_frac'), 'wall', r.get('avg_wall_ms'))"
for round in 1 2; do
  for lib in libmrag_k3wold libmrag; do
    MRAG_LIB=$L/$lib.so timeout -k 10 200 python3 -c "
import json, sys
sys.path[:0] = ['$R', '$R/multimodal-rag-for-image-text-search_amd']
import bench
out = bench.fusion_leg(1, 0, 0, 40, 4)
print(json.dumps({'lib': '$lib', 'round': $round, 'value': out['value'], 'ms_per_step': out['ms_per_step']}))
" 2>/dev/null | grep '^{' >> gpurun_out/${P}_fusion_ab.jsonl || { echo "fusion failed $lib"; exit 2; }
  done
done
cat gpurun_out/${P}_fusion_ab.jsonl
