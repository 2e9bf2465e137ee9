#!/bin/bash
# Round 3, session 30: streaming LayerNorm with unconditional loads (the prefetch now overlaps the
# reductions: vmcnt(4) instead of vmcnt(0)) vs HEAD (libmrag_base.so): embeddings bit-identical,
# CLIP and config-5 legs, LN kernel time in the CLIP trace, encoder tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
for lib in libmrag_base.so libmrag.so; do
  MRAG_LIB=$L/$lib timeout -k 10 300 python scripts/enc_dump.py gpurun_out/r3s30_enc_$lib.npz > gpurun_out/r3s30_dump.log 2>&1 || { echo "dump failed"; tail -5 gpurun_out/r3s30_dump.log; exit 1; }
done
python3 -c "
import numpy as np
a=np.load('gpurun_out/r3s30_enc_libmrag_base.so.npz'); b=np.load('gpurun_out/r3s30_enc_libmrag.so.npz')
print({k: bool(np.array_equal(a[k], b[k])) for k in a.files})
"
for round in 1 2; do
  for lib in libmrag_base.so libmrag.so; do
    for f in 1 3; do
      MRAG_LIB=$L/$lib timeout -k 10 200 python scripts/clip_bench.py 30 $f > gpurun_out/r3s30_clip.json 2>gpurun_out/r3s30_clip.err || { echo "clip failed"; tail -5 gpurun_out/r3s30_clip.err; exit 2; }
      echo "$lib clip inflight=$f $(grep -v amdgpu gpurun_out/r3s30_clip.json | cut -c1-110)" >> gpurun_out/r3s30_legs.log
    done
    MRAG_LIB=$L/$lib timeout -k 10 300 python scripts/fusion_bench.py 20 > gpurun_out/r3s30_fusion.json 2>gpurun_out/r3s30_fusion.err || { echo "fusion failed"; tail -5 gpurun_out/r3s30_fusion.err; exit 3; }
    echo "$lib fusion $(grep -v amdgpu gpurun_out/r3s30_fusion.json | cut -c1-130)" >> gpurun_out/r3s30_legs.log
  done
done
cat gpurun_out/r3s30_legs.log
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s30_prof -o clip -- python3 scripts/clip_bench.py 20 1 > gpurun_out/r3s30_prof.log 2>&1 || { echo "prof failed"; exit 4; }
f=$(find gpurun_out/r3s30_prof -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > gpurun_out/r3s30_kstats.txt
find gpurun_out/r3s30_prof -name "*trace.csv" -delete
head -6 gpurun_out/r3s30_kstats.txt
timeout -k 10 900 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s30_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s30_tests.log; exit 5; }
tail -1 gpurun_out/r3s30_tests.log
