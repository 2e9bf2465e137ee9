#!/bin/bash
# Round 5, session 42: the group's host half stages the JPEG segments (unstuffed) and PNG
# scanlines (inflated) in a pinned arena on its threads; mrag_files_decode only copies and
# launches (the tree) vs the previous commit (lib/libmrag_prev.so): image GPU tests, the
# device-decode stage alone, embed_images_batch from files, two interleaved pairs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=$R/multimodal-rag-for-image-text-search_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_png_gpu.py tests/test_jpeg_gpu.py tests/test_imgprep_gpu.py tests/test_compat_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s42_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s42_tests.log; exit 3; }
tail -1 gpurun_out/r5s42_tests.log
O=gpurun_out/r5s42_ab.jsonl; : > $O
for i in 1 2; do
  for v in libmrag libmrag_prev; do
    MRAG_LIB=$L/$v.so timeout -k 10 300 python3 -u scripts/decode_stage_split.py >> $O 2>> gpurun_out/r5s42.err || { echo "split $v failed"; tail gpurun_out/r5s42.err; exit 4; }
    MRAG_LIB=$L/$v.so timeout -k 10 300 python3 -u scripts/ingest_calls.py 2048 >> $O 2>> gpurun_out/r5s42.err || { echo "calls $v failed"; tail gpurun_out/r5s42.err; exit 5; }
  done
done
cat $O
