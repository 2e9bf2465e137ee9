#!/bin/bash
# Round 5, session 39: two-literal inflate table entries (the tree) vs the previous inflate
# (lib/libmrag_oldinfl.so): embed_images_batch from files, two interleaved pairs; PNG GPU tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_png_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s39_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s39_tests.log; exit 3; }
tail -1 gpurun_out/r5s39_tests.log
O=gpurun_out/r5s39_inflate_ab.jsonl; : > $O
for i in 1 2; do
  timeout -k 10 300 python3 -u scripts/ingest_calls.py 2048 >> $O 2>> gpurun_out/r5s39.err || { echo "tree failed"; tail gpurun_out/r5s39.err; exit 4; }
  MRAG_LIB=$R/multimodal-rag-for-image-text-search_amd/lib/libmrag_oldinfl.so timeout -k 10 300 python3 -u scripts/ingest_calls.py 2048 >> $O 2>> gpurun_out/r5s39.err || { echo "old failed"; exit 5; }
done
cat $O
