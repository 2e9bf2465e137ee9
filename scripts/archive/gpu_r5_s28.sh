#!/bin/bash
# Round 5, session 28: image lanes as hipGraph replays. Encoder GPU tests (lanes bit-identical,
# batch consistency, oracle parity), then CLIP one batch / three in flight: the tree (graphs) vs
# the previous commit's library (direct launches), three interleaved pairs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_clip_lanes_gpu.py tests/test_encoders_gpu.py tests/test_jpeg_gpu.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r5s28_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s28_tests.log; exit 3; }
tail -1 gpurun_out/r5s28_tests.log
O=gpurun_out/r5s28_graph_ab.jsonl; : > $O
for i in 1 2 3; do
  timeout -k 10 200 python3 -u scripts/clip_lanes_ab.py 30 >> $O 2>> gpurun_out/r5s28.err || { echo "tree failed"; exit 4; }
  MRAG_LIB=$R/multimodal-rag-for-image-text-search_amd/lib/libmrag_nograph.so timeout -k 10 200 python3 -u scripts/clip_lanes_ab.py 30 >> $O 2>> gpurun_out/r5s28.err || { echo "ab failed"; exit 5; }
done
cat $O
