#!/bin/bash
# Round 6 final profiles of this tree on one box (prefix $1, default r6p; the suite, smoke and the bench line
# come from scripts/gpu_r6_val.sh): a K7-only kernel trace of the roofline leg (config 3, one search in flight: the line's
# avg_launch_ms / frac must agree with it), the K7 HBM traffic passes (FETCH_SIZE / WRITE_SIZE,
# separate) reduced into knn_scan_pmc.json, and a kernel trace of the whole bench, and the twelve tower GEMM shapes (scripts/gemm_roofline.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=${1:-r6p}
cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
KNN="python3 $R/bench.py --no-cpu-baseline --no-clip --no-fusion --no-call-pattern --no-retrieve-pattern --no-ingest --knn-streams 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${P}_knn_prof -o run -- $KNN --steps 20 > $R/gpurun_out/${P}_knn_prof.log 2>&1 || { echo "knn prof failed"; exit 6; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- $KNN --steps 3 --warmup 1 > $R/gpurun_out/${P}_fetch.log 2>&1 || { echo "fetch pass failed"; exit 7; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- $KNN --steps 3 --warmup 1 > $R/gpurun_out/${P}_write.log 2>&1 || { echo "write pass failed"; exit 8; }
cd $R
f=$(find gpurun_out/${P}_knn_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${P}_knn_kernel_stats.csv
mkdir -p gpurun_out/prof_stats; cp "$f" gpurun_out/prof_stats/run_kernel_stats.csv
f=$(find gpurun_out/${P}_knn_prof -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/${P}_knn_kernel_trace.csv
f=$(find gpurun_out/prof_fetch -name "*counter_collection.csv" | head -1); [ "$f" = gpurun_out/prof_fetch/run_counter_collection.csv ] || cp "$f" gpurun_out/prof_fetch/run_counter_collection.csv
f=$(find gpurun_out/prof_write -name "*counter_collection.csv" | head -1); [ "$f" = gpurun_out/prof_write/run_counter_collection.csv ] || cp "$f" gpurun_out/prof_write/run_counter_collection.csv
python3 scripts/pmc_summary.py "knn_scan3_kernel<512, 0, 4>" gpurun_out/knn_scan_pmc.json 1074765824 || exit 9
python3 scripts/kstats.py gpurun_out/${P}_knn_kernel_stats.csv | head -8
cat gpurun_out/knn_scan_pmc.json
find gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/${P}_knn_prof -name "*trace*.csv" -delete
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${P}_prof -o bench -- python3 $R/bench.py --steps 20 --knn-streams 1 --no-cpu-baseline --no-ingest > $R/gpurun_out/${P}_prof.log 2>&1 || { echo "bench prof failed"; exit 10; }
cd $R
f=$(find gpurun_out/${P}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${P}_kernel_stats.csv
f=$(find gpurun_out/${P}_prof -name "*kernel_trace.csv" | head -1); python3 scripts/trace_by_grid.py "$f" > gpurun_out/${P}_bench_by_grid.txt 2>/dev/null
find gpurun_out/${P}_prof -name "*kernel_trace.csv" -size +20M -delete
python3 scripts/kstats.py gpurun_out/${P}_kernel_stats.csv | head -14
timeout -k 10 300 python3 scripts/gemm_roofline.py 2>/dev/null | grep "^{" > gpurun_out/${P}_gemm_roofline.jsonl || { echo "roofline failed"; exit 11; }
wc -l gpurun_out/${P}_gemm_roofline.jsonl
du -sh gpurun_out
