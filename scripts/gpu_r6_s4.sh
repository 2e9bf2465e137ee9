#!/bin/bash
# Round 6 session 4: K3w (weight-stationary GEMM for the text towers' K <= 512 GEMMs): bit
# identity against K3, the encoder suites, per-shape times (auto = K3w vs K3 / K3d forced), the
# config-5 leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encoders_gpu.py -x -q -m gpu -k weight_stationary --timeout 240 --timeout-method thread > gpurun_out/r6s4_ws.log 2>&1 || { echo "K3w test failed"; tail -30 gpurun_out/r6s4_ws.log; exit 3; }
tail -1 gpurun_out/r6s4_ws.log
timeout -k 10 300 python3 scripts/gemm_roofline.py --only minilm:fc1,minilm:qkv,clip_text:fc1,clip_text:qkv > gpurun_out/r6s4_gemm.jsonl 2>&1 || { echo "gemm failed"; tail gpurun_out/r6s4_gemm.jsonl; exit 2; }
grep '^{' gpurun_out/r6s4_gemm.jsonl | cut -c1-300
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_configs_gpu.py tests/test_embedder_gpu.py tests/test_cross_encoder_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6s4_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r6s4_tests.log; exit 4; }
tail -1 gpurun_out/r6s4_tests.log
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-clip --no-call-pattern --no-retrieve-pattern --no-ingest > gpurun_out/r6s4_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r6s4_bench.log; exit 5; }
grep '"metric"' gpurun_out/r6s4_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); f=d.get('fusion',{}); print('knn', d['value'], 'fusion', f.get('value'), f.get('ms_per_step'), json.dumps(f.get('roofline'))[:300])"
