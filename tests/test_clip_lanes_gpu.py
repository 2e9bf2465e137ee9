"""Image lanes (csrc/encoder.hip, mrag_encoder_embed_images): the process's sole image handle runs a
batch of >= 128 images as two sub-batches on two workspaces and streams; with a second handle alive
calls run as one lane. Both must give the same rows bit for bit, for device and host pointers.

This module sorts first among the GPU tests, so no other image handle exists when it starts."""
from __future__ import annotations

import gc

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_lone_handle_lanes_bit_identical(cuda):
    import torch

    from app.encoders import CLIP_VISION_B32, GpuEncoder

    gc.collect()
    g = torch.Generator(device=cuda).manual_seed(17)
    imgs = torch.randint(0, 256, (257, 224, 224, 3), generator=g, dtype=torch.uint8, device=cuda)
    h1 = GpuEncoder(CLIP_VISION_B32)
    lone = h1.embed_images(imgs).cpu()                 # sole handle: lanes of 129 + 128
    part_a = h1.embed_images(imgs[:100]).cpu()         # below the lane minimum: one lane
    part_b = h1.embed_images(imgs[100:]).cpu()         # 157 images: lanes of 79 + 78
    host = h1.embed_images(imgs.cpu().numpy())         # host pointers, lanes as well
    h2 = GpuEncoder(CLIP_VISION_B32)
    shared = h2.embed_images(imgs).cpu()               # two handles: one lane
    torch.cuda.synchronize()
    assert torch.equal(lone, shared)
    assert torch.equal(lone[:100], part_a)
    assert torch.equal(lone[100:], part_b)
    np.testing.assert_array_equal(host, lone.numpy())
    h2.close()
    again = h1.embed_images(imgs).cpu()                # sole again after the close
    assert torch.equal(again, lone)
    h1.close()
