#!/usr/bin/env python3
"""Probe: the bench's CLIP in-flight leg after the other legs (bench.main with the CLIP leg
wrapped): run it with 0..3 extra torch streams taken from the pool first, to see whether which
pool streams the leg gets (their hardware queues, GPU_MAX_HW_QUEUES = 4) sets its rate."""
import json
import os
import sys

sys.path[:0] = [os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))]
sys.argv = ["bench.py", "--no-cpu-baseline"]
import bench  # noqa: E402

orig = bench.clip_leg


def wrapped(steps, warmup):
    import torch

    from app.encoders import bench_clip_images

    res = []
    for shift in (0, 1, 2, 3, 0):
        for _ in range(shift):
            torch.cuda.Stream(device=torch.device("cuda", 0))
        out = bench_clip_images(steps=steps, warmup=warmup)
        res.append({"shift": shift, "clip": out["value"]})
        print(json.dumps(res[-1]), file=sys.stderr, flush=True)
    return orig(steps, warmup)


bench.clip_leg = wrapped
bench.main()
