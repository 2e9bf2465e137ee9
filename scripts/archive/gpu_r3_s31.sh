#!/bin/bash
# Round 3, session 31: flash attention with unconditional (clamped) loads and a mask instance (a key
# block's loads in one round trip, was ~5) vs HEAD (libmrag_base.so): embeddings bit-identical,
# config-5 legs, config-5 kernel trace, encoder / cross-encoder / compat tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
for lib in libmrag_base.so libmrag.so; do
  MRAG_LIB=$L/$lib timeout -k 10 300 python scripts/enc_dump.py gpurun_out/r3s31_enc_$lib.npz > gpurun_out/r3s31_dump.log 2>&1 || { echo "dump failed"; tail -5 gpurun_out/r3s31_dump.log; exit 1; }
done
python3 -c "
import numpy as np
a=np.load('gpurun_out/r3s31_enc_libmrag_base.so.npz'); b=np.load('gpurun_out/r3s31_enc_libmrag.so.npz')
print({k: bool(np.array_equal(a[k], b[k])) for k in a.files})
"
for round in 1 2 3; do
  for lib in libmrag_base.so libmrag.so; do
    MRAG_LIB=$L/$lib timeout -k 10 300 python scripts/fusion_bench.py 20 > gpurun_out/r3s31_fusion.json 2>gpurun_out/r3s31_fusion.err || { echo "fusion failed"; tail -5 gpurun_out/r3s31_fusion.err; exit 3; }
    echo "$lib fusion $(grep -v amdgpu gpurun_out/r3s31_fusion.json | cut -c1-130)" >> gpurun_out/r3s31_legs.log
  done
done
cat gpurun_out/r3s31_legs.log
cd /tmp && export TMPDIR=/tmp && cd $R
for lib in libmrag_base.so libmrag.so; do
  MRAG_LIB=$R/$L/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s31_prof_$lib -o f -- python3 scripts/fusion_bench.py 10 > gpurun_out/r3s31_prof.log 2>&1 || { echo "prof failed"; exit 4; }
  f=$(find gpurun_out/r3s31_prof_$lib -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > gpurun_out/r3s31_kstats_$lib.txt
  find gpurun_out/r3s31_prof_$lib -name "*trace.csv" -delete
  echo "== $lib"; grep attention gpurun_out/r3s31_kstats_$lib.txt
done
timeout -k 10 900 python -u -m pytest tests/test_encoders_gpu.py tests/test_cross_encoder_gpu.py tests/test_compat_gpu.py tests/test_configs_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s31_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s31_tests.log; exit 5; }
tail -1 gpurun_out/r3s31_tests.log
