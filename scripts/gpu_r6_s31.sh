#!/bin/bash
# Session 31: the CLIP in-flight sweep with and without one tiny kernel per stream at creation
# (does a stream's hardware queue depend on its first launch?), two processes, same box.
set -o pipefail
mkdir -p gpurun_out
P=${1:-r6s31}
timeout -k 10 300 python -u scripts/clip_inflight_sweep.py --rounds 2 --steps 30 --inflight 3,4,5 --warm > gpurun_out/${P}_warm.jsonl 2> gpurun_out/${P}_warm.err || { echo "warm sweep failed"; tail -20 gpurun_out/${P}_warm.err; exit 1; }
timeout -k 10 300 python -u scripts/clip_inflight_sweep.py --rounds 2 --steps 30 --inflight 3,4,5 > gpurun_out/${P}_cold.jsonl 2> gpurun_out/${P}_cold.err || { echo "cold sweep failed"; tail -20 gpurun_out/${P}_cold.err; exit 1; }
cat gpurun_out/${P}_warm.jsonl gpurun_out/${P}_cold.jsonl
