#!/bin/bash
# Round 5, session 20: K14 as a multi-wave pipelined wavefront. PNG / JPEG / image tests, the bench's
# ingest leg, and a kernel trace of the ingest group A/B (K13 / K14 / K0 / ViT per launch).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_png_gpu.py tests/test_jpeg_gpu.py tests/test_imgprep_gpu.py tests/test_compat_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5s20_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5s20_tests.log; exit 3; }
tail -1 gpurun_out/r5s20_tests.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-clip --no-fusion --no-retrieve-pattern > gpurun_out/r5s20_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5s20_bench.log; exit 6; }
grep '"metric"' gpurun_out/r5s20_bench.log | tail -1 > gpurun_out/r5s20_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/r5s20_bench.json'))
print(json.dumps(d.get('call_pattern',{}).get('ingest_embed_images_batch')))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5s20_prof -o run -- python3 $R/scripts/ingest_group_ab.py 2048 > $R/gpurun_out/r5s20_prof.log 2>&1 || { echo "prof failed"; tail -5 $R/gpurun_out/r5s20_prof.log; exit 5; }
cd $R
cat gpurun_out/r5s20_prof.log | grep images_per_s
f=$(find gpurun_out/r5s20_prof -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" | head -14 | tee gpurun_out/r5s20_ingest_kernel_stats.txt
find gpurun_out/r5s20_prof -name "*trace*.csv" -delete
