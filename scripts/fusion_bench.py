"""BASELINE config 5 leg alone (one GPU): python scripts/fusion_bench.py [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    print(json.dumps(bench.fusion_leg(1, 0, 0, steps=steps, warmup=2)), flush=True)
