#!/bin/bash
# Round 4, session 15: the N > 1 path of this tree rehearsed on one GPU (2 ranks, gloo): sharded
# search == one index, and bench.py --gpus 2 end to end (numbers are two ranks on one GPU).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/sharded_rehearsal.py > gpurun_out/r4s15_rehearsal.log 2>&1 || { echo "rehearsal failed"; tail -20 gpurun_out/r4s15_rehearsal.log; exit 1; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-clip > gpurun_out/r4s15_bench_n2.log 2>&1 || { echo "bench n2 failed"; tail -20 gpurun_out/r4s15_bench_n2.log; exit 2; }
grep -v amdgpu.ids gpurun_out/r4s15_rehearsal.log | grep -i "world\|ok\|identical" | head -5; grep '"metric"' gpurun_out/r4s15_bench_n2.log | cut -c1-400
