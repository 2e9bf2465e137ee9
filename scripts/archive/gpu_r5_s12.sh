#!/bin/bash
# Round 5, session 14 (12: byte loads; 13: 16-byte window, 32-bit tables; 14: window through the scalar cache; 15: packed tables): K13 (GPU JPEG decode). Its GPU tests + the image / compat tests, the decode
# A/B (Pillow pool vs K13), a kernel trace of it, then the bench's ingest leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jpeg_gpu.py tests/test_imgprep_gpu.py tests/test_compat_gpu.py tests/test_clip_lanes_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s15_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s15_tests.log; exit 3; }
tail -1 gpurun_out/r5s15_tests.log
timeout -k 10 300 python3 -u scripts/jpeg_bench.py 1024 > gpurun_out/r5s15_jpeg_bench.json 2>gpurun_out/r5s15_jpeg_bench.err || { echo "jpeg bench failed"; tail -20 gpurun_out/r5s15_jpeg_bench.err; exit 4; }
cat gpurun_out/r5s15_jpeg_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5s15_jpeg_prof -o run -- python3 $R/scripts/jpeg_bench.py 512 > $R/gpurun_out/r5s15_jpeg_prof.log 2>&1 || { echo "jpeg prof failed"; exit 5; }
cd $R
f=$(find gpurun_out/r5s15_jpeg_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5s15_jpeg_kernel_stats.csv; python3 scripts/kstats.py gpurun_out/r5s15_jpeg_kernel_stats.csv 2>/dev/null | head -8 || true
find gpurun_out/r5s15_jpeg_prof -name "*trace*.csv" -delete
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-clip --no-fusion --no-retrieve-pattern > gpurun_out/r5s15_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5s15_bench.log; exit 6; }
grep '"metric"' gpurun_out/r5s15_bench.log | tail -1 > gpurun_out/r5s15_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r5s15_bench.json'))
print(json.dumps(d.get('call_pattern',{}).get('ingest_embed_images_batch')))"
