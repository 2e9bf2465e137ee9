#!/bin/bash
# Round 4 final validation of this tree on one box: the full GPU suite, smoke, the driver's
# bench line, a K7-only kernel trace of the roofline leg (config 3, one search in flight: the
# line's avg_launch_ms / frac must agree with it), the K7 HBM traffic passes (FETCH_SIZE /
# WRITE_SIZE, separate) reduced into knn_scan_pmc.json, and a kernel trace of the whole bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4f_tests.log; exit 3; }
tail -1 gpurun_out/r4f_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r4f_smoke.log; exit 4; }
timeout -k 10 900 python bench.py > gpurun_out/r4f_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4f_bench.log; exit 5; }
grep '"metric"' gpurun_out/r4f_bench.log | tail -1 > gpurun_out/r4f_bench.json
cut -c1-900 gpurun_out/r4f_bench.json
cd /tmp && export TMPDIR=/tmp
KNN="python3 $R/bench.py --no-cpu-baseline --no-clip --no-fusion --no-call-pattern --knn-streams 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4f_knn_prof -o run -- $KNN --steps 20 > $R/gpurun_out/r4f_knn_prof.log 2>&1 || { echo "knn prof failed"; exit 6; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o run -- $KNN --steps 3 --warmup 1 > $R/gpurun_out/r4f_fetch.log 2>&1 || { echo "fetch pass failed"; exit 7; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o run -- $KNN --steps 3 --warmup 1 > $R/gpurun_out/r4f_write.log 2>&1 || { echo "write pass failed"; exit 8; }
cd $R
f=$(find gpurun_out/r4f_knn_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r4f_knn_kernel_stats.csv
mkdir -p gpurun_out/prof_stats; cp "$f" gpurun_out/prof_stats/run_kernel_stats.csv
f=$(find gpurun_out/r4f_knn_prof -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/r4f_knn_kernel_trace.csv
f=$(find gpurun_out/prof_fetch -name "*counter_collection.csv" | head -1); [ "$f" = gpurun_out/prof_fetch/run_counter_collection.csv ] || cp "$f" gpurun_out/prof_fetch/run_counter_collection.csv
f=$(find gpurun_out/prof_write -name "*counter_collection.csv" | head -1); [ "$f" = gpurun_out/prof_write/run_counter_collection.csv ] || cp "$f" gpurun_out/prof_write/run_counter_collection.csv
python3 scripts/pmc_summary.py "knn_scan3_kernel<512, 0, 4>" gpurun_out/knn_scan_pmc.json 1074765824 || exit 9
python3 scripts/kstats.py gpurun_out/r4f_knn_kernel_stats.csv | head -8
cat gpurun_out/knn_scan_pmc.json
find gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/r4f_knn_prof -name "*trace*.csv" -delete
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4f_prof -o bench -- python3 $R/bench.py --steps 20 --knn-streams 1 --no-cpu-baseline > $R/gpurun_out/r4f_prof.log 2>&1 || { echo "bench prof failed"; exit 10; }
cd $R
f=$(find gpurun_out/r4f_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r4f_kernel_stats.csv
find gpurun_out/r4f_prof -name "*kernel_trace.csv" -size +20M -delete
python3 scripts/kstats.py gpurun_out/r4f_kernel_stats.csv | head -14
du -sh gpurun_out
