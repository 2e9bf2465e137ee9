#!/bin/bash
# Round 5, session 8: image lanes only for a lone batch (no other image handle busy on the
# device). Encoder / compat / embedder tests on the tree, then CLIP one / three in flight:
# lanes1 (one stream) vs the tree, three interleaved rounds; then the bench's ingest leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_clip_lanes_gpu.py tests/test_encoders_gpu.py tests/test_compat_gpu.py tests/test_embedder_gpu.py tests/test_imgprep_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s8c_enc_tests.log 2>&1 || { echo "encoder tests failed"; tail -30 gpurun_out/r5s8c_enc_tests.log; exit 3; }
tail -1 gpurun_out/r5s8c_enc_tests.log
for v in lanes1 tree lanes1 tree lanes1 tree; do
  if [ $v = tree ]; then unset MRAG_LIB; else export MRAG_LIB=$R/$L/libmrag_$v.so; fi
  timeout -k 10 240 python3 -u scripts/clip_lanes_ab.py 20 >> gpurun_out/r5s8c_lanes_ab.jsonl 2>/dev/null || { echo "lanes $v failed"; exit 4; }
  tail -1 gpurun_out/r5s8c_lanes_ab.jsonl
done
unset MRAG_LIB
