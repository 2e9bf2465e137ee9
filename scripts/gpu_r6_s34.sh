#!/bin/bash
# Session 34: the retrieve side-stream A/B again, a discarded warm-up round and rotated arm order,
# six rounds, at the box's hardware-queue setting.
set -o pipefail
mkdir -p gpurun_out
P=${1:-r6s34}
timeout -k 10 400 python -u scripts/retrieve_stream_ab.py 6 > gpurun_out/${P}.jsonl 2> gpurun_out/${P}.err || { echo "failed"; tail -20 gpurun_out/${P}.err; exit 1; }
cat gpurun_out/${P}.jsonl
