#!/bin/bash
# Round 3, session 11: K7 early barrier (wait + barrier before the last row block's MFMAs, next
# tile's first fragments read under them) A/B: base (before the tail change), default, EB; stamps
# of default and EB with group-fire counts; kNN tests under EB.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
MRAG_LIB=$L/libmrag_eb.so timeout -k 10 900 python -u -m pytest tests/test_knn_gpu.py tests/test_knn_generic_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/r3s11_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s11_tests.log; exit 1; }
tail -1 gpurun_out/r3s11_tests.log
for round in 1 2; do
  for lib in libmrag_base.so libmrag.so libmrag_eb.so; do
    MRAG_LIB=$L/$lib timeout -k 10 120 python scripts/knn_scan_ab.py 30 >> gpurun_out/r3s11_ab.log 2>&1 || { echo "ab $lib failed"; tail -5 gpurun_out/r3s11_ab.log; exit 2; }
  done
done
grep -v amdgpu.ids gpurun_out/r3s11_ab.log
for lib in libmrag_k7stamp.so libmrag_k7stamp_eb.so; do
  MRAG_LIB=$L/$lib timeout -k 10 120 python scripts/k7_stamps.py >> gpurun_out/r3s11_stamps.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/r3s11_stamps.log; exit 3; }
done
grep -v amdgpu.ids gpurun_out/r3s11_stamps.log
