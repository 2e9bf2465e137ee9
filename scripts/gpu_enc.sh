#!/bin/bash
# Encoder round on the GPU box: parity tests + CLIP image bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python -m pytest tests/test_encoders_gpu.py -x -q -m gpu > gpurun_out/enc_tests.log 2>&1; echo "rc=$?" >> gpurun_out/enc_tests.log
timeout -k 10 300 python -c "
import sys, json; sys.path[:0]=['multimodal-rag-for-image-text-search_amd','.']
from app.encoders import bench_clip_images
print(json.dumps(bench_clip_images(steps=10, warmup=2)))
" > gpurun_out/clip_bench.log 2>&1; echo "rc=$?" >> gpurun_out/clip_bench.log
