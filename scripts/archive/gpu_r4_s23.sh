#!/bin/bash
# Round 4, session 23: bench.py's N = 4 path rehearsed on one GPU (4 ranks, gloo; numbers are four
# ranks sharing one GPU, not a scaling point) and the sharded search at world 4 (== one index).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 scripts/sharded_rehearsal.py > gpurun_out/r4s23_rehearsal4.log 2>&1 || { echo "rehearsal failed"; tail -20 gpurun_out/r4s23_rehearsal4.log; exit 1; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 4 --steps 5 --warmup 2 --no-cpu-baseline --no-clip > gpurun_out/r4s23_bench_n4.log 2>&1 || { echo "bench n4 failed"; tail -20 gpurun_out/r4s23_bench_n4.log; exit 2; }
grep -v amdgpu.ids gpurun_out/r4s23_rehearsal4.log | grep world | head -2; grep '"metric"' gpurun_out/r4s23_bench_n4.log | cut -c1-300
