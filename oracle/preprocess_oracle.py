"""ORACLE -- test infrastructure only (tests/, smoke(), bench cpu_baseline may use it).

numpy restatement of the reference's patch preprocessing: a 64×64
uint8 PhotoTour patch becomes the fp32 [1,32,32] network input.

Two loader pipelines exist in hardnet/HardNet.py:

* ``transform`` (no augmentation, HardNet.py:345-349): ``cv2_scale`` (Utils.py:10-11,
  ``cv2.resize(x, (32, 32), INTER_LINEAR)``) -> ``np_reshape`` -> ``ToTensor`` (/255) ->
  ``Normalize(mean_image, std_image)``.
  OpenCV (third-party, pinned only as ``opencv 4.8.1.78`` by FDLNet's requirements and
  absent from this image) turns INTER_LINEAR with an exact integer factor of 2 into its
  fast area path (imgproc/src/resize.cpp: ``is_area_fast && iscale == 2`` ->
  ``INTER_AREA`` -> ``ResizeAreaFastVec<uchar>``), i.e. ``(a + b + c + d + 2) >> 2`` over
  each 2×2 block.  cv2 cannot be run here, so this branch is **parity unpinned**.
* ``transform_test`` with augmentation (HardNet.py:333-337): ``ToPILImage`` ->
  ``transforms.Resize(32)`` (= ``PIL.Image.resize((32, 32), BILINEAR)``) -> ``ToTensor``
  (no Normalize).  Pillow's resampler (libImaging/Resample.c, published algorithm):
  triangle filter with support ``1 * scale``, coefficients normalised per output pixel,
  quantised to 22 fractional bits, separable horizontal-then-vertical passes each
  rounding (+2^21) and clipping to uint8.  Pinned against Pillow 12.2 by
  ``tests/golden/preprocess.npz`` (``tests/golden/make_preprocess_golden.py``).

``ToTensor`` is ``x.float().div(255)`` and ``Normalize`` is ``sub_(mean).div_(std)`` with
fp32 mean/std, all IEEE fp32 -- restated here with float32 numpy ops in the same order.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2  # Resample.c


def _pil_bilinear_coeffs(in_size: int, out_size: int):
    """Pillow precompute_coeffs + normalize_coeffs_8bpc for the bilinear filter."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds, coeffs = [], np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w.append(1.0 - t if t < 1.0 else 0.0)
        ww = sum(w)
        w = [v / ww if ww != 0.0 else v for v in w]
        for x, v in enumerate(w):
            coeffs[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else \
                int(0.5 + v * (1 << PRECISION_BITS))
        bounds.append((xmin, xmax))
    return bounds, coeffs


def _clip8(ss: np.ndarray) -> np.ndarray:
    return np.clip(ss >> PRECISION_BITS, 0, 255)


def pil_resize_bilinear(u8: np.ndarray, out_hw: int = 32) -> np.ndarray:
    """[B,H,W] uint8 -> [B,out,out] uint8 exactly as Pillow's BILINEAR resize."""
    b, h, w = u8.shape
    if h == out_hw and w == out_hw:
        return u8.copy()  # Image.resize returns a copy when the size is unchanged
    src = u8.astype(np.int64)
    bx, kx = _pil_bilinear_coeffs(w, out_hw)
    tmp = np.empty((b, h, out_hw), np.int64)
    for xx, (x0, n) in enumerate(bx):
        ss = (1 << (PRECISION_BITS - 1)) + (src[:, :, x0:x0 + n] * kx[xx, :n]).sum(-1)
        tmp[:, :, xx] = _clip8(ss)
    by, ky = _pil_bilinear_coeffs(h, out_hw)
    out = np.empty((b, out_hw, out_hw), np.int64)
    for yy, (y0, n) in enumerate(by):
        ss = (1 << (PRECISION_BITS - 1)) + (tmp[:, y0:y0 + n, :] * ky[yy, :n, None]).sum(1)
        out[:, yy, :] = _clip8(ss)
    return out.astype(np.uint8)


def cv2_resize_linear_2x(u8: np.ndarray) -> np.ndarray:
    """[B,2n,2n] uint8 -> [B,n,n]: OpenCV INTER_LINEAR at factor 2 (area-fast path)."""
    b, h, w = u8.shape
    if h == 32 and w == 32:
        return u8.copy()
    s = u8.astype(np.int32)
    q = s[:, 0::2, 0::2] + s[:, 0::2, 1::2] + s[:, 1::2, 0::2] + s[:, 1::2, 1::2]
    return ((q + 2) >> 2).astype(np.uint8)


def to_tensor_normalize(u8: np.ndarray, mean=None, std=None) -> np.ndarray:
    """ToTensor (/255 in fp32) then optional Normalize((mean,), (std,)) -> [B,1,H,W] fp32."""
    x = u8.astype(np.float32) / np.float32(255.0)
    if mean is not None:
        x = (x - np.float32(mean)) / np.float32(std)
    return x[:, None, :, :].astype(np.float32)


def preprocess(u8: np.ndarray, mode: str, mean=None, std=None) -> np.ndarray:
    """mode 'cv2' = HardNet.py:345-349 pipeline, 'pil' = HardNet.py:333-337 pipeline."""
    r = cv2_resize_linear_2x(u8) if mode == "cv2" else pil_resize_bilinear(u8)
    return to_tensor_normalize(r, mean, std)
