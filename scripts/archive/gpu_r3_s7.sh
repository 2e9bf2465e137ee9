#!/bin/bash
# Round 3, session 7: the N > 1 path rehearsed on one GPU (2 ranks, gloo: sharded search ==
# single index; bench.py --gpus 2), then the full GPU suite, smoke, bench (N = 1) and its
# kernel-trace summary.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/sharded_rehearsal.py > gpurun_out/r3s7_rehearsal.log 2>&1 || { echo "rehearsal failed"; tail -20 gpurun_out/r3s7_rehearsal.log; exit 1; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-clip > gpurun_out/r3s7_bench_n2.log 2>&1 || { echo "bench n2 failed"; tail -20 gpurun_out/r3s7_bench_n2.log; exit 2; }
unset MRAG_DIST_BACKEND
grep -v amdgpu.ids gpurun_out/r3s7_rehearsal.log | grep world; grep '"metric"' gpurun_out/r3s7_bench_n2.log | cut -c1-600
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread > gpurun_out/r3s7_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3s7_tests.log; exit 3; }
tail -1 gpurun_out/r3s7_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s7_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r3s7_smoke.log; exit 4; }
timeout -k 10 900 python bench.py > gpurun_out/r3s7_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r3s7_bench.log; exit 5; }
grep '"metric"' gpurun_out/r3s7_bench.log | tail -1 > gpurun_out/r3s7_bench.json
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s7_prof -o bench -- python3 bench.py --steps 20 --knn-streams 1 --no-cpu-baseline > gpurun_out/r3s7_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r3s7_prof.log; exit 6; }
f=$(find gpurun_out/r3s7_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r3s7_kernel_stats.csv
find gpurun_out/r3s7_prof -name "*kernel_trace.csv" -size +20M -delete
python3 scripts/kstats.py gpurun_out/r3s7_kernel_stats.csv | head -12
