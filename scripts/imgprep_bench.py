"""Resize + centre-crop throughput on decoded 640x480 RGB images (decode excluded):
PIL on host threads (app.encoders.preprocess.to_u8_224) vs K0 on the GPU (upload incl.)."""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multimodal-rag-for-image-text-search_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from app.encoders.preprocess import resize_crop_device, to_u8_224  # noqa: E402

n, w, h = 256, 640, 480
rng = np.random.default_rng(0)
arrays = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for _ in range(n)]
pils = [Image.fromarray(a) for a in arrays]
threads = 16
with ThreadPoolExecutor(threads) as ex:
    list(ex.map(to_u8_224, pils[:32]))
    t0 = time.perf_counter()
    host = np.stack(list(ex.map(to_u8_224, pils)))
    t_host = time.perf_counter() - t0
resize_crop_device(arrays[:8])
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    dev = resize_crop_device(arrays)
torch.cuda.synchronize()
t_dev = (time.perf_counter() - t0) / 5
assert np.array_equal(dev.cpu().numpy(), host)
print(json.dumps({"images": n, "src": f"{w}x{h}", "host_pil_img_per_s": round(n / t_host, 1), "host_threads": threads,
                  "gpu_img_per_s_incl_upload": round(n / t_dev, 1), "bit_exact": True}))
