#!/bin/bash
# Round 6 session 6: K3w timing ablations (same box): no epilogue (1), no next-tile LDS-DMA (2),
# neither (3), against the product build, CLIP q|k|v and MiniLM fc1 shapes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
for lib in libmrag libmrag_wsabl1 libmrag_wsabl2 libmrag_wsabl3; do
  for s in "1536 512 0" "1536 384 2"; do
    echo "{\"lib\": \"$lib\"}" >> gpurun_out/r6s6_abl.jsonl
    MRAG_LIB=$R/$L/$lib.so timeout -k 10 120 python3 scripts/gemm_ws_probe.py $s k3w >> gpurun_out/r6s6_abl.jsonl 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r6s6_abl.jsonl; exit 2; }
  done
done
grep '^{' gpurun_out/r6s6_abl.jsonl | grep -v '"M": 2560'
