"""Deterministic synthetic weights and patches (no torch RNG, no network).

Everything here is derived from a counter-based splitmix64 stream so that the
same bytes can be regenerated on any host (this container, the GPU box) without
depending on the torch RNG implementation.  The golden fixtures under
``tests/golden`` store a SHA-256 of every generated tensor so that drift is caught.

Synthetic patches follow SURVEY.md section 8(d): ``round(U[0,255])/255`` then the
global loader normalisation ``(x - 0.443728476019) / 0.20197947209``
(hardnet/HardNet.py:346-350, hardnetNAS/general_functions/dataloader.py:118-122).
"""
from __future__ import annotations

import hashlib
import zlib
from typing import Dict

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

MEAN_IMAGE = 0.443728476019
STD_IMAGE = 0.20197947209


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n consecutive outputs of splitmix64 started at ``seed`` (uint64)."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, n: int) -> np.ndarray:
    """Uniform float64 in [0, 1) with 53 random bits."""
    return (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def normal(seed: int, n: int) -> np.ndarray:
    """Standard normal float64 via Box-Muller on two interleaved uniform streams."""
    m = (n + 1) // 2
    u = uniform(seed, 2 * m)
    u1 = u[0::2] + (0.5 / (1 << 53))   # (0, 1]
    u2 = u[1::2]
    r = np.sqrt(-2.0 * np.log(u1))
    out = np.empty(2 * m, dtype=np.float64)
    out[0::2] = r * np.cos(2.0 * np.pi * u2)
    out[1::2] = r * np.sin(2.0 * np.pi * u2)
    return out[:n]


def _stream(seed: int, name: str) -> int:
    return (seed * 0x100000001B3 + zlib.crc32(name.encode())) & 0xFFFFFFFFFFFFFFFF


def synth_patches(n: int, seed: int = 0) -> np.ndarray:
    """[n,1,32,32] float32 patches: uint8-quantised, globally normalised."""
    u = uniform(_stream(seed, "patches"), n * 32 * 32)
    q = np.floor(u * 256.0).clip(0, 255).astype(np.float32) / np.float32(255.0)
    x = (q - np.float32(MEAN_IMAGE)) / np.float32(STD_IMAGE)
    return x.astype(np.float32).reshape(n, 1, 32, 32)


def synth_tensor(seed: int, name: str, shape, kind: str) -> np.ndarray:
    """One synthetic parameter tensor.

    kind: "conv" -- N(0, (0.6)^2 / fan_in), the scale of orthogonal(gain=0.6)
                   (hardnet/HardNet.py:317-324);
          "bn_weight" -- U[0.5, 1.5];  "bn_bias" -- N(0, 0.1^2);
          "bias" -- N(0, 0.05^2);  "mean" -> zeros;  "var" -> ones.
    """
    n = int(np.prod(shape))
    s = _stream(seed, name)
    if kind == "conv":
        fan_in = int(np.prod(shape[1:]))
        v = normal(s, n) * (0.6 / np.sqrt(fan_in))
    elif kind == "bn_weight":
        v = 0.5 + uniform(s, n)
    elif kind == "bn_bias":
        v = 0.1 * normal(s, n)
    elif kind == "bias":
        v = 0.05 * normal(s, n)
    elif kind == "mean":
        v = np.zeros(n)
    elif kind == "var":
        v = np.ones(n)
    else:
        raise ValueError(kind)
    return v.astype(np.float32).reshape(shape)


def kind_of(key: str, shape) -> str:
    """Classify a state_dict key into a synth_tensor kind."""
    if key.endswith("running_mean"):
        return "mean"
    if key.endswith("running_var"):
        return "var"
    if len(shape) == 4:
        return "conv"
    leaf = key.rsplit(".", 1)[-1]
    parent = key.rsplit(".", 2)[-2] if key.count(".") >= 1 else ""
    if leaf == "weight":
        return "bn_weight"
    if leaf == "bias":
        # SE convs carry a bias (fbnet_builder.py:410-411); BN bias otherwise
        return "bias" if parent.isdigit() else "bn_bias"
    raise ValueError(f"cannot classify {key} {shape}")


def synth_state_dict(template: Dict[str, "np.ndarray"], seed: int) -> Dict[str, np.ndarray]:
    """Fill every float tensor of a state_dict template (key -> shape) synthetically.

    ``num_batches_tracked`` entries are skipped (caller keeps them as-is).
    """
    out = {}
    for k, shape in template.items():
        if k.endswith("num_batches_tracked"):
            continue
        out[k] = synth_tensor(seed, k, tuple(shape), kind_of(k, tuple(shape)))
    return out


def sha256_f32(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()
