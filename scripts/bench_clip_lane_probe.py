#!/usr/bin/env python3
"""Probe: bench.main with the CLIP leg extended by the one-batch case on the start-up stream (the
case whose image lanes shared a hardware queue, 53k img/s): prints the one-batch rate on a pool
stream and on the start-up stream. Run once per library (MRAG_LIB)."""
import json
import os
import sys

sys.path[:0] = [os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))]
sys.argv = ["bench.py", "--no-cpu-baseline"]
import bench  # noqa: E402

orig = bench.clip_leg


def wrapped(steps, warmup, streams=None):
    from app.encoders import bench_clip_images

    out = orig(steps, warmup, streams=streams)
    early = bench_clip_images(steps=steps, warmup=warmup, inflight=1, streams=streams)
    print(json.dumps({"lib": os.path.basename(os.environ.get("MRAG_LIB", "libmrag.so")), "inflight3": out["value"],
                      "one_pool_stream": out["one_batch_in_flight"]["images_per_s"],
                      "one_startup_stream": early["value"]}), file=sys.stderr, flush=True)
    return out


bench.clip_leg = wrapped
bench.main()
