"""Generate tests/golden/preprocess.npz (survey container; needs Pillow, not /root/reference).

The reference's augmented test loader (hardnet/HardNet.py:333-337) is
``np_reshape64 -> ToPILImage -> transforms.Resize(32) -> ToTensor``.  torchvision is not
installed here, so the transform steps are spelled with the calls torchvision makes:
``Image.fromarray(x, 'L')`` (ToPILImage of an HxWx1 uint8 array), ``img.resize((32, 32),
Image.BILINEAR)`` (Resize of a square image to 32) and ``torch.from_numpy(a).float()
.div(255)`` (ToTensor).  The non-augmented loader (HardNet.py:345-349) adds
``Normalize((mean,), (std,))`` = ``sub_(mean).div_(std)`` in fp32; its cv2 resize cannot be
run here (cv2 absent), so only the Normalize arithmetic is pinned, applied to the PIL output.

Run from the repo root:  python tests/golden/make_preprocess_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import PIL
import torch
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from hardnetnas_amd import synth  # noqa: E402


def patches64() -> np.ndarray:
    rng = np.random.default_rng(20240611)
    x = rng.integers(0, 256, (112, 64, 64), dtype=np.uint8)
    yy, xx = np.mgrid[0:64, 0:64]
    edge = [np.zeros((64, 64)), np.full((64, 64), 255), (yy + xx) % 2 * 255,
            (yy * 4) % 256, (xx * 4) % 256, np.where((yy // 8 + xx // 8) % 2 == 0, 250, 3),
            np.full((64, 64), 128), (yy * 64 + xx) % 256]
    # blurred random blobs (natural-image-like smooth patches)
    for s in range(8):
        r = np.random.default_rng(s).random((9, 9))
        big = np.kron(r, np.ones((8, 8)))[:64, :64]
        edge.append(np.round(big * 255))
    return np.concatenate([np.stack(edge).astype(np.uint8), x])


def main():
    u8 = patches64()
    pil = np.stack([np.array(Image.fromarray(p, "L").resize((32, 32), Image.BILINEAR)) for p in u8])
    t = torch.from_numpy(pil).float().div(255).unsqueeze(1)
    mean = torch.as_tensor(synth.MEAN_IMAGE, dtype=torch.float32)
    std = torch.as_tensor(synth.STD_IMAGE, dtype=torch.float32)
    tn = t.clone().sub_(mean).div_(std)
    np.savez_compressed(os.path.join(HERE, "preprocess.npz"), u8_64=u8, pil_u8_32=pil,
                        pil_f32=t.numpy(), pil_norm_f32=tn.numpy(),
                        meta=np.array(json.dumps({"pillow": PIL.__version__, "torch": torch.__version__})))
    print("wrote preprocess.npz", u8.shape)


if __name__ == "__main__":
    main()
