#!/bin/bash
# Round 3, session 26: attention_seq64 with every staging load issued before the first LDS store (one round trip per workgroup) vs the flash kernel: bit-identity, CLIP legs, kernel trace, encoder tests.
# (attention_seq64_kernel) vs the per-wave flash kernel (MRAG_ATTN_SEQ64=0): bit-identity of all
# three towers' embeddings, CLIP legs, kernel trace of the CLIP leg, encoder tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
for v in 0 1; do
  MRAG_ATTN_SEQ64=$v timeout -k 10 300 python scripts/enc_dump.py gpurun_out/r3s26_enc_$v.npz > gpurun_out/r3s26_dump_$v.log 2>&1 || { echo "dump $v failed"; tail -5 gpurun_out/r3s26_dump_$v.log; exit 1; }
done
python3 -c "
import numpy as np
a=np.load('gpurun_out/r3s26_enc_0.npz'); b=np.load('gpurun_out/r3s26_enc_1.npz')
print({k: bool(np.array_equal(a[k], b[k])) for k in a.files})
"
for round in 1 2; do
  for v in 0 1; do
    for f in 1 3; do
      MRAG_ATTN_SEQ64=$v timeout -k 10 200 python scripts/clip_bench.py 30 $f > gpurun_out/r3s26_clip.json 2>gpurun_out/r3s26_clip.err || { echo "clip failed"; tail -5 gpurun_out/r3s26_clip.err; exit 2; }
      echo "seq64=$v inflight=$f $(grep -v amdgpu gpurun_out/r3s26_clip.json | cut -c1-130)" >> gpurun_out/r3s26_legs.log
    done
  done
done
cat gpurun_out/r3s26_legs.log
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s26_prof -o clip -- python3 scripts/clip_bench.py 20 1 > gpurun_out/r3s26_prof.log 2>&1 || { echo "prof failed"; exit 3; }
f=$(find gpurun_out/r3s26_prof -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > gpurun_out/r3s26_kstats.txt
find gpurun_out/r3s26_prof -name "*trace.csv" -delete
head -8 gpurun_out/r3s26_kstats.txt
timeout -k 10 900 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s26_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s26_tests.log; exit 4; }
tail -1 gpurun_out/r3s26_tests.log
