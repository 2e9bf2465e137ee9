#!/bin/bash
# Round 5, session 6: K3s skinny GEMM (M <= 64). Skinny-vs-K3 parity, encoder tests, then small
# token batch timing (base = HEAD without K3s vs the working tree) and kernel traces of B = 1.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
L=multimodal-rag-for-image-text-search_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_encoders_gpu.py tests/test_compat_gpu.py tests/test_embedder_gpu.py tests/test_cross_encoder_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s6_enc_tests.log 2>&1 || { echo "encoder tests failed"; tail -30 gpurun_out/r5s6_enc_tests.log; exit 3; }
tail -1 gpurun_out/r5s6_enc_tests.log
for v in base tree base tree; do
  if [ $v = base ]; then export MRAG_LIB=$R/$L/libmrag_base.so; else unset MRAG_LIB; fi
  timeout -k 10 240 python3 -u scripts/enc_small_batch_timing.py 200 > gpurun_out/r5s6_small_$v.jsonl 2>/dev/null || { echo "timing $v failed"; exit 4; }
  echo "== $v"; cat gpurun_out/r5s6_small_$v.jsonl
done
unset MRAG_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/r5s6_mini_trace2 -o run -- python3 $R/scripts/enc_small_trace.py minilm 1 12 100 > $R/gpurun_out/r5s6_mini_trace2.log 2>&1 || { echo "trace 1 failed"; exit 5; }
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/r5s6_clipt_trace2 -o run -- python3 $R/scripts/enc_small_trace.py clip_text 1 12 100 > $R/gpurun_out/r5s6_clipt_trace2.log 2>&1 || { echo "trace 2 failed"; exit 6; }
cd $R && python3 scripts/trace_db_summary.py gpurun_out/r5s6_mini_trace2/run_results.db 12 && python3 scripts/trace_db_summary.py gpurun_out/r5s6_clipt_trace2/run_results.db 12
