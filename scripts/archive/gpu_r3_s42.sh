#!/bin/bash
# Round 3, session 42: K8 folding two chunks per step (+ pipelined reads, wave candidate sort): stamps vs base,
# kNN GPU tests, Q = 1 / Q = 1000 kernel timelines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
for v in k7stamp_base k7stamp; do
  MRAG_LIB=$L/libmrag_$v.so timeout -k 10 200 python scripts/k8_stamps.py >> gpurun_out/r3s42_k8.log 2>gpurun_out/r3s42.err || { echo "$v failed"; tail -5 gpurun_out/r3s42.err; exit 2; }
done
cat gpurun_out/r3s42_k8.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_knn_gpu.py tests/test_knn_generic_gpu.py tests/test_fusion_gpu.py tests/test_configs_gpu.py > gpurun_out/r3s42_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3s42_tests.log; exit 3; }
tail -1 gpurun_out/r3s42_tests.log
cd /tmp && export TMPDIR=/tmp && cd $R
for nq in 1 1000; do
  rm -rf gpurun_out/r3s42_prof
  NQ=$nq timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3s42_prof -o q1 -- python3 scripts/q1_profile.py > gpurun_out/r3s42_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r3s42_prof.log; exit 4; }
  f=$(find gpurun_out/r3s42_prof -name "*kernel_trace.csv" | head -1)
  echo "== nq=$nq $(grep ms_per_search gpurun_out/r3s42_prof.log)" >> gpurun_out/r3s42_timeline.log
  python3 scripts/q1_profile.py --trace "$f" >> gpurun_out/r3s42_timeline.log
done
rm -rf gpurun_out/r3s42_prof
cat gpurun_out/r3s42_timeline.log
