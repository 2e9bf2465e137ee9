#!/bin/bash
# Round 5, session 7: image-lane split of a CLIP call (two or three sub-batches on their own
# workspaces and streams). Encoder tests on lanes2, then CLIP one / three in flight for lanes1
# (= one stream), lanes2, lanes3, lanes2 from 64 images, two interleaved rounds; then the counter
# passes and the config-5 in-flight re-check on the committed in-tree library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
MRAG_LIB=$R/$L/libmrag_lanes2.so timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_compat_gpu.py tests/test_embedder_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s7_enc_tests.log 2>&1 || { echo "encoder tests failed"; tail -30 gpurun_out/r5s7_enc_tests.log; exit 3; }
tail -1 gpurun_out/r5s7_enc_tests.log
for v in lanes1 lanes2 lanes3 lanes2m64 lanes1 lanes2 lanes3 lanes2m64; do
  MRAG_LIB=$R/$L/libmrag_$v.so timeout -k 10 240 python3 -u scripts/clip_lanes_ab.py 20 >> gpurun_out/r5s7_lanes_ab.jsonl 2>/dev/null || { echo "lanes $v failed"; exit 4; }
  tail -1 gpurun_out/r5s7_lanes_ab.jsonl
done
bash scripts/gpu_r5_pmc2.sh
