#!/bin/bash
# Round 3, session 28: the N > 1 bench path rehearsed on one GPU after this session's changes (two
# ranks, gloo; their numbers are two ranks sharing one GPU, not a scaling point) and the sharded
# search bit-identical to one index.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export MRAG_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/sharded_rehearsal.py > gpurun_out/r3s28_rehearsal.log 2>&1 || { echo "rehearsal failed"; tail -20 gpurun_out/r3s28_rehearsal.log; exit 1; }
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3s28_bench_n2.log 2>&1 || { echo "bench n2 failed"; tail -20 gpurun_out/r3s28_bench_n2.log; exit 2; }
grep -v amdgpu.ids gpurun_out/r3s28_rehearsal.log | grep world
grep '"metric"' gpurun_out/r3s28_bench_n2.log | cut -c1-400
