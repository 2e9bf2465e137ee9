#!/bin/bash
# Round 5, last tree: kernel trace (--kernel-trace --stats) of the bench's ingest leg
# (embed_images_batch from 2,048 JPEG/PNG files: K13a-c, K14, K0, the ViT tower) beside a short kNN leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5k_ingest_prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --knn-streams 1 --no-cpu-baseline --no-clip --no-fusion --no-retrieve-pattern > $R/gpurun_out/r5k_ingest_prof.log 2>&1 || { echo "ingest prof failed"; tail -5 $R/gpurun_out/r5k_ingest_prof.log; exit 3; }
cd $R
f=$(find gpurun_out/r5k_ingest_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5k_ingest_kernel_stats.csv
find gpurun_out/r5k_ingest_prof -name "*trace*.csv" -delete
grep '"metric"' gpurun_out/r5k_ingest_prof.log | tail -1 > gpurun_out/r5k_ingest_prof_bench.json
python3 scripts/kstats.py gpurun_out/r5k_ingest_kernel_stats.csv | head -16
