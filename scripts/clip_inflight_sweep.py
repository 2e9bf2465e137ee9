"""CLIP image tower batches in flight (2..6) with every stream created up front.

Repeats the round-4 sweep (1 -> 66.8k, 2 -> 66.8k, 3 -> 81.9k, 4 -> 81.1k img/s) the way bench.py
runs the leg now. GPU_MAX_HW_QUEUES=8 only when the environment does not set it (the GPU pool's
boxes export 4). Rounds are interleaved; one JSON line per (round, inflight).

    python scripts/clip_inflight_sweep.py [--rounds 2] [--steps 30]
"""
import argparse
import json
import os
import sys

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
os.environ.setdefault("MRAG_SYNTHETIC_WEIGHTS", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "multimodal-rag-for-image-text-search_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--inflight", default="2,3,4,5,6")
    ap.add_argument("--warm", action="store_true",
                    help="launch one tiny kernel on each stream right after creating it (bench._early_streams)")
    args = ap.parse_args()
    import torch
    from app.encoders import bench_clip_images

    dev = torch.device("cuda", 0)
    counts = [int(x) for x in args.inflight.split(",")]
    streams = [torch.cuda.Stream(device=dev) for _ in range(max(counts))]
    if args.warm:
        for s in streams:
            with torch.cuda.stream(s):
                torch.zeros(1, device=dev).add_(1)
        torch.cuda.synchronize(dev)
    for r in range(args.rounds):
        for n in counts:
            res = bench_clip_images(steps=args.steps, warmup=4, inflight=n, streams=streams[:n])
            print(json.dumps({"round": r, "warm": args.warm, "inflight": n, "images_per_s": res["value"],
                              "ms_per_batch": res["ms_per_batch"]}), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
