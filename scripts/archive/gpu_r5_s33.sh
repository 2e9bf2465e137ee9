#!/bin/bash
# Round 5, session 33: blocking-sync waits in K13 / K14 / K0 (the tree) vs stream synchronize
# (the previous commit's library): the ingest group A/B, two interleaved pairs; JPEG / PNG tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_png_gpu.py tests/test_jpeg_gpu.py tests/test_imgprep_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s33_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s33_tests.log; exit 3; }
tail -1 gpurun_out/r5s33_tests.log
O=gpurun_out/r5s33_wait_ab.jsonl; : > $O
for i in 1 2; do
  echo '{"lib": "blocking (tree)"}' >> $O
  timeout -k 10 300 python3 -u scripts/ingest_group_ab.py 2048 >> $O 2>> gpurun_out/r5s33.err || { echo "tree failed"; exit 4; }
  echo '{"lib": "spin (previous)"}' >> $O
  MRAG_LIB=$R/multimodal-rag-for-image-text-search_amd/lib/libmrag_spinwait.so timeout -k 10 300 python3 -u scripts/ingest_group_ab.py 2048 >> $O 2>> gpurun_out/r5s33.err || { echo "ab failed"; exit 5; }
done
cat $O
