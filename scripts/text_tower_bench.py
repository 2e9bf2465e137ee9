"""Text towers at the config-5 query batch (1000 queries x 16 tokens): MiniLM-L6 and CLIP text,
HIP-event time per embed_tokens call (device ids in, device embeddings out).
python scripts/text_tower_bench.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]
os.environ.setdefault("MRAG_SYNTHETIC_WEIGHTS", "1")

import torch  # noqa: E402

from app.encoders import CLIP_TEXT_B32, MINILM_L6, GpuEncoder  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
g = torch.Generator(device="cuda").manual_seed(0)
out = {"env_rowln": os.environ.get("MRAG_ROWLN", "1")}
for name, cfg, vocab in (("minilm", MINILM_L6, 30000), ("clip_text", CLIP_TEXT_B32, 49000)):
    enc = GpuEncoder(cfg)
    ids = torch.randint(1000, vocab, (1000, 16), generator=g, device="cuda", dtype=torch.int32)
    mask = torch.ones_like(ids)
    for _ in range(3):
        e = enc.embed_tokens(ids, mask)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        e = enc.embed_tokens(ids, mask)
    e1.record()
    torch.cuda.synchronize()
    out[name + "_ms"] = round(e0.elapsed_time(e1) / reps, 4)
    import hashlib
    out[name + "_digest"] = hashlib.sha256(e.float().cpu().numpy().tobytes()).hexdigest()[:16]
print(json.dumps(out), flush=True)
