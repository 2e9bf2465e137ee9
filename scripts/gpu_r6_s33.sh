#!/bin/bash
# Session 33: the retrieve leg's CLIP-text side stream (pool / high priority / caller's stream) at
# 8 and 4 hardware queues, one process each.
set -o pipefail
mkdir -p gpurun_out
P=${1:-r6s33}
timeout -k 10 300 python -u scripts/retrieve_stream_ab.py 3 > gpurun_out/${P}_q8.jsonl 2> gpurun_out/${P}_q8.err || { echo "q8 failed"; tail -20 gpurun_out/${P}_q8.err; exit 1; }
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python -u scripts/retrieve_stream_ab.py 3 > gpurun_out/${P}_q4.jsonl 2> gpurun_out/${P}_q4.err || { echo "q4 failed"; tail -20 gpurun_out/${P}_q4.err; exit 1; }
cat gpurun_out/${P}_q8.jsonl gpurun_out/${P}_q4.jsonl
