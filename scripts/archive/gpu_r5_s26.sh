#!/bin/bash
# Round 5, session 26: K0 tap tables deduplicated and cached, K0 horizontal pass per pixel with LDS taps, K13b / K13c vector stores.
# The JPEG / PNG GPU tests (embed_images_batch equal with and without device decode), the group
# A/B and the bench's ingest leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_png_gpu.py tests/test_jpeg_gpu.py tests/test_imgprep_gpu.py tests/test_compat_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s26_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s26_tests.log; exit 3; }
tail -1 gpurun_out/r5s26_tests.log
timeout -k 10 300 python3 -u scripts/ingest_group_ab.py 2048 > gpurun_out/r5s26_ingest_group_ab.jsonl 2>gpurun_out/r5s26.err || { echo "ab failed"; tail -5 gpurun_out/r5s26.err; exit 4; }
cat gpurun_out/r5s26_ingest_group_ab.jsonl
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-clip --no-fusion --no-retrieve-pattern > gpurun_out/r5s26_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5s26_bench.log; exit 6; }
grep '"metric"' gpurun_out/r5s26_bench.log | tail -1 > gpurun_out/r5s26_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r5s26_bench.json'))
print(json.dumps(d.get('call_pattern',{}).get('ingest_embed_images_batch')))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5s26_prof -o run -- python3 $R/scripts/ingest_group_ab.py 2048 > $R/gpurun_out/r5s26_prof.log 2>&1 || { echo "prof failed"; tail -5 $R/gpurun_out/r5s26_prof.log; exit 5; }
cd $R
f=$(find gpurun_out/r5s26_prof -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" > gpurun_out/r5s26_ingest_kernel_stats_full.txt; head -16 gpurun_out/r5s26_ingest_kernel_stats_full.txt > gpurun_out/r5s26_ingest_kernel_stats.txt; cat gpurun_out/r5s26_ingest_kernel_stats.txt
find gpurun_out/r5s26_prof -name "*trace*.csv" -delete
