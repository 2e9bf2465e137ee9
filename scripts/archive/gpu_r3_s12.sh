#!/bin/bash
# Round 3, session 12: K7 straight-line fire path (best row first, the rest only if one passes the raised threshold) A/B vs the previous build and with the early barrier; stamps; kNN tests under both.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
for lib in libmrag.so libmrag_eb.so; do MRAG_LIB=$L/$lib timeout -k 10 900 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_generic_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s12_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s12_tests.log; exit 1; }; done
tail -1 gpurun_out/r3s12_tests.log
for round in 1 2 3; do
  for lib in libmrag_prev.so libmrag.so libmrag_eb.so; do
    MRAG_LIB=$L/$lib timeout -k 10 120 python scripts/knn_scan_ab.py 30 >> gpurun_out/r3s12_ab.log 2>&1 || { echo "ab $lib failed"; tail -5 gpurun_out/r3s12_ab.log; exit 2; }
  done
done
grep -v amdgpu.ids gpurun_out/r3s12_ab.log
for lib in libmrag_k7stamp.so; do
  MRAG_LIB=$L/$lib timeout -k 10 120 python scripts/k7_stamps.py >> gpurun_out/r3s12_stamps.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/r3s12_stamps.log; exit 3; }
done
grep -v amdgpu.ids gpurun_out/r3s12_stamps.log
