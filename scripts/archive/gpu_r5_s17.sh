#!/bin/bash
# Round 5, session 17: K13a, the self-synchronising parallel Huffman decode. JPEG / image tests,
# the decode timing (and its kernel trace), then the bench's ingest leg (2048 files).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jpeg_gpu.py tests/test_imgprep_gpu.py tests/test_compat_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s17_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s17_tests.log; exit 3; }
tail -1 gpurun_out/r5s17_tests.log
timeout -k 10 300 python3 -u scripts/jpeg_bench.py 1024 > gpurun_out/r5s17_jpeg_bench.json 2>gpurun_out/r5s17_jpeg_bench.err || { echo "jpeg bench failed"; tail -20 gpurun_out/r5s17_jpeg_bench.err; exit 4; }
cat gpurun_out/r5s17_jpeg_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5s17_prof -o run -- python3 $R/scripts/jpeg_bench.py 1024 > $R/gpurun_out/r5s17_prof.log 2>&1 || { echo "prof failed"; exit 5; }
cd $R
f=$(find gpurun_out/r5s17_prof -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" | head -8 | tee gpurun_out/r5s17_k13_kernel_stats.txt
find gpurun_out/r5s17_prof -name "*trace*.csv" -delete
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-clip --no-fusion --no-retrieve-pattern > gpurun_out/r5s17_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5s17_bench.log; exit 6; }
grep '"metric"' gpurun_out/r5s17_bench.log | tail -1 > gpurun_out/r5s17_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r5s17_bench.json'))
print(json.dumps(d.get('call_pattern',{}).get('ingest_embed_images_batch')))"
