#!/bin/bash
# Round 5, session 27: K3 / K3d rule for the ViT image-lane halves (M = 6400): the tree vs K3d for
# every M >= 4096 (scripts/k3_rule_ab.sh), CLIP one batch and three in flight, three pairs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
O=gpurun_out/r5s27_k3_rule_ab.jsonl; : > $O
for i in 1 2 3; do
  timeout -k 10 200 python3 -u scripts/clip_lanes_ab.py 30 >> $O 2>> gpurun_out/r5s27.err || { echo "tree failed"; exit 3; }
  MRAG_LIB=$R/multimodal-rag-for-image-text-search_amd/lib/libmrag_ab_k3d4096.so timeout -k 10 200 python3 -u scripts/clip_lanes_ab.py 30 >> $O 2>> gpurun_out/r5s27.err || { echo "ab failed"; exit 4; }
done
cat $O
# config 5 (fusion leg) of the r5h validation tree's library vs this tree's, two pairs
F=gpurun_out/r5s27_fusion_ab.jsonl; : > $F
for i in 1 2; do
  for lib in libmrag_r5h.so libmrag.so; do
    MRAG_LIB=$R/multimodal-rag-for-image-text-search_amd/lib/$lib timeout -k 10 400 python3 -u bench.py --steps 20 --no-cpu-baseline --no-clip --no-ingest --no-call-pattern --no-retrieve-pattern > gpurun_out/r5s27_f.log 2>&1 || { echo "fusion $lib failed"; tail -5 gpurun_out/r5s27_f.log; exit 5; }
    python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/r5s27_f.log') if l.startswith('{\"metric')][-1])
print(json.dumps({'lib': '$lib', 'knn': d['value'], 'fusion': d['fusion']['value'], 'fusion_one': d['fusion']['one_step_in_flight']['queries_per_s']}))" >> $F
  done
done
cat $F
