"""fp16 range of the NAS / FDL fp16x3 kernels.

The hi half of an fp16x3 operand overflows at |v| >= 65520.  BN-folded weights out of range
make hn_create fail (csrc/hn_api.hip put_f16_split); activations are data-dependent, so
hardnetnas_amd.model.fp16_split_margin measures them on a calibration batch with the module's
torch layers.  These tests pin both, and check that large-but-in-range activations keep parity.
"""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

from fixtures import build_module, golden_inputs
from hardnetnas_amd.model import fp16_split_margin


def _scale_stem(m, s):
    """Multiply the NAS stem's BatchNorm output by ~s (running_var / s^2): every later
    activation grows with it."""
    bn = next(mod for mod in m.first.modules() if isinstance(mod, nn.BatchNorm2d))
    with torch.no_grad():
        bn.running_var.div_(s * s)
        if bn.affine:
            bn.bias.mul_(s)
    return m


@pytest.mark.parametrize("name", ["wang2", "wang3", "wang4", "fdl_NASNet", "fdl_NASNet_01"])
def test_golden_checkpoints_have_fp16_headroom(name):
    m, fx, _ = build_module(name)
    r = fp16_split_margin(m, torch.from_numpy(golden_inputs(fx)))
    assert r["margin"] > 1000, r


def test_margin_flags_out_of_range_activations():
    m, fx, _ = build_module("wang2")
    x = torch.from_numpy(golden_inputs(fx))
    base = fp16_split_margin(m, x)
    r = fp16_split_margin(_scale_stem(m, 1e5), x)
    assert r["margin"] < 1 < base["margin"], (base, r)


@pytest.mark.gpu
def test_hn_create_rejects_weights_outside_fp16(cuda_device):
    m, fx, _ = build_module("wang2")
    with torch.no_grad():
        m.stages[0].pw.conv.weight.mul_(1e7)
    m = m.to(cuda_device)
    x = torch.from_numpy(golden_inputs(fx)[:8]).to(cuda_device)
    with torch.no_grad(), pytest.raises(RuntimeError, match="fp16 range"):
        m(x)


@pytest.mark.gpu
@pytest.mark.parametrize("s", [30.0, 300.0])
def test_large_in_range_activations_keep_parity(s, cuda_device):
    m, fx, _ = build_module("wang2")
    _scale_stem(m, s)
    x = torch.from_numpy(golden_inputs(fx))
    r = fp16_split_margin(m, x)
    assert r["margin"] > 1, r
    with torch.no_grad():
        ref = copy.deepcopy(m).double()(x.double()).numpy()
        y = m.to(cuda_device)(x.to(cuda_device)).cpu().numpy()
    err = np.abs(y - ref).max()
    print(f"stem x{s}: peak {r['peak']:.1f} (margin {r['margin']:.1f}), max|hip - fp64| = {err:.2e}")
    assert np.isfinite(y).all() and err <= 1e-4
