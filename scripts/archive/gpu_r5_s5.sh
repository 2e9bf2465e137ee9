#!/bin/bash
# Round 5, session 5: K7 class bound (6 < k <= 16). kNN + encoder/compat GPU tests on the working
# tree, then main-scan A/B: base (HEAD, no class bound) vs cb (re-read every 8 tiles), cb4, cb16;
# then the bench's retrieve / ingest legs (hipGraph replay of small token batches, pipelined decode).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_configs_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5s5_knn_tests.log 2>&1 || { echo "knn tests failed"; tail -30 gpurun_out/r5s5_knn_tests.log; exit 3; }
tail -1 gpurun_out/r5s5_knn_tests.log
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_compat_gpu.py tests/test_imgprep_gpu.py tests/test_embedder_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s5_enc_tests.log 2>&1 || { echo "encoder tests failed"; tail -30 gpurun_out/r5s5_enc_tests.log; exit 4; }
tail -1 gpurun_out/r5s5_enc_tests.log
for v in base cb cb4 cb16 base cb cb4 cb16 base cb cb4 cb16; do
  MRAG_LIB=$R/$L/libmrag_$v.so timeout -k 10 240 python3 -u scripts/knn_scan_ab.py 40 > gpurun_out/r5s5_ab_$v.json 2>/dev/null || { echo "ab $v failed"; exit 5; }
  echo "$v $(cat gpurun_out/r5s5_ab_$v.json)" | tee -a gpurun_out/r5s5_ab.txt
done
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-clip --no-fusion > gpurun_out/r5s5_bench_legs.log 2>&1 || { echo "bench legs failed"; tail -30 gpurun_out/r5s5_bench_legs.log; exit 6; }
grep '"metric"' gpurun_out/r5s5_bench_legs.log | tail -1 > gpurun_out/r5s5_bench_legs.json
python3 -c "
import json; d=json.load(open('gpurun_out/r5s5_bench_legs.json'))
print(d['value'], d['roofline']['frac']); print(json.dumps(d.get('call_pattern',{}).get('retrieve'))); print(json.dumps(d.get('call_pattern',{}).get('ingest_embed_images_batch')))"
