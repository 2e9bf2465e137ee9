#!/usr/bin/env python3
"""Config-5 leg alone (bench.fusion_leg, N = 1), for a kernel trace of its step:
    MRAG_FUSION_STREAMS=1 rocprofv3 --kernel-trace --stats -d DIR -- python3 scripts/fusion_profile.py STEPS
MRAG_FUSION_STREAMS=1 serialises the two branches so per-kernel times add up to the step."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd")]

import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
out = bench.fusion_leg(1, 0, 0, steps, 3)
print(json.dumps({k: out[k] for k in ("value", "ms_per_step", "steps", "steps_in_flight")}), flush=True)
