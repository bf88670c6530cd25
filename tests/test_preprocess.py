"""Patch preprocessing: uint8 patches -> fp32 network input.

CPU tests pin the numpy oracle (oracle/preprocess_oracle.py) to the Pillow-generated
fixtures (tests/golden/preprocess.npz) and check argument validation at the C ABI.
GPU tests compare hn_preprocess bit-exactly with the oracle / fixtures, and run the
preprocess -> HardNet forward chain against the oracle chain.

The cv2 branch (HardNet.py:345-349) is parity unpinned: cv2 is absent here, so the device
result is checked against the restated OpenCV 2x area-fast rule only.
"""
import numpy as np
import pytest
import torch

from fixtures import build_module, load
from hardnetnas_amd import _native as N
from hardnetnas_amd import synth
from oracle import hardnet_oracle as O
from oracle import preprocess_oracle as P

MEAN, STD = synth.MEAN_IMAGE, synth.STD_IMAGE


def _fx():
    return load("preprocess")


# ---------------------------------------------------------------- CPU ----
def test_oracle_pil_resize_matches_pillow_fixture():
    fx = _fx()
    assert np.array_equal(P.pil_resize_bilinear(fx["u8_64"]), fx["pil_u8_32"])


def test_oracle_to_tensor_and_normalize_match_fixture():
    fx = _fx()
    assert np.array_equal(P.to_tensor_normalize(fx["pil_u8_32"]), fx["pil_f32"])
    assert np.array_equal(P.to_tensor_normalize(fx["pil_u8_32"], MEAN, STD), fx["pil_norm_f32"])


def test_oracle_cv2_rule_known_answers():
    # 2x2 blocks: sums 0, 1, 2, 6, 10, 1020 -> (s + 2) >> 2 = 0, 0, 1, 2, 3, 255
    blocks = [(0, 0, 0, 0), (1, 0, 0, 0), (1, 1, 0, 0), (2, 2, 1, 1), (3, 3, 2, 2),
              (255, 255, 255, 255)]
    u = np.zeros((1, 64, 64), np.uint8)
    for i, (a, b, c, d) in enumerate(blocks):
        u[0, 0, 2 * i], u[0, 0, 2 * i + 1], u[0, 1, 2 * i], u[0, 1, 2 * i + 1] = a, b, c, d
    r = P.cv2_resize_linear_2x(u)
    assert r[0, 0, :6].tolist() == [0, 0, 1, 2, 3, 255]


def test_abi_rejects_bad_preprocess_args_without_gpu():
    lib = N.load_library()
    assert lib.hn_preprocess(None, 4, 32, 1, 1, 0.0, 1.0, None, None) == 1
    assert b"in_hw" in lib.hn_last_error()
    assert lib.hn_preprocess(None, 4, 64, 7, 1, 0.0, 1.0, None, None) == 1
    assert b"resize" in lib.hn_last_error()
    assert lib.hn_preprocess(None, 4, 64, 2, 0, 0.0, 1.0, None, None) == 1
    assert b"NULL" in lib.hn_last_error()
    assert lib.hn_preprocess(None, 0, 64, 2, 0, 0.0, 1.0, None, None) == 0  # empty batch


# ---------------------------------------------------------------- GPU ----
@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 3, 5, 128])
def test_pil_mode_matches_pillow_fixture(n, cuda_device):
    fx = _fx()
    u = torch.from_numpy(fx["u8_64"][:n].copy()).to(cuda_device)
    y = N.preprocess(u, resize="pil", normalize=False).cpu().numpy()
    assert np.array_equal(y, fx["pil_f32"][:n])
    y = N.preprocess(u, resize="pil", normalize=True, mean=MEAN, std=STD).cpu().numpy()
    assert np.array_equal(y, fx["pil_norm_f32"][:n])


@pytest.mark.gpu
def test_cv2_and_none_modes_match_oracle(cuda_device):
    rng = np.random.default_rng(5)
    u64 = np.concatenate([load("preprocess")["u8_64"],
                          rng.integers(0, 256, (1001, 64, 64), dtype=np.uint8)])
    y = N.preprocess(torch.from_numpy(u64).to(cuda_device), resize="cv2").cpu().numpy()
    assert np.array_equal(y, P.preprocess(u64, "cv2", MEAN, STD))
    u32 = rng.integers(0, 256, (77, 1, 32, 32), dtype=np.uint8)
    y = N.preprocess(torch.from_numpy(u32).to(cuda_device), resize="none", normalize=False)
    assert np.array_equal(y.cpu().numpy(), P.to_tensor_normalize(u32[:, 0]))


@pytest.mark.gpu
def test_large_batch_pil_checksum(cuda_device):
    """65,536 patches: every output equals the oracle on a strided sample and the per-patch
    means agree (size-independent property at bench scale)."""
    g = torch.Generator(device=cuda_device).manual_seed(3)
    u = torch.randint(0, 256, (65536, 64, 64), device=cuda_device, generator=g,
                      dtype=torch.int32).to(torch.uint8)
    y = N.preprocess(u, resize="pil")
    idx = torch.arange(0, 65536, 997, device=cuda_device)
    ref = P.preprocess(u[idx].cpu().numpy(), "pil", MEAN, STD)
    assert np.array_equal(y[idx].cpu().numpy(), ref)
    assert torch.isfinite(y).all()


@pytest.mark.gpu
def test_preprocess_then_forward_matches_oracle_chain(cuda_device):
    m, fx, p = build_module("hardnet")
    m = m.to(cuda_device)
    u = load("preprocess")["u8_64"]
    with torch.no_grad():
        x = N.preprocess(torch.from_numpy(u).to(cuda_device), resize="cv2")
        y = m(x).cpu().numpy()
    xr = P.preprocess(u, "cv2", MEAN, STD)
    ref = O.hardnet_forward({k: torch.as_tensor(v) for k, v in p.items()},
                            torch.from_numpy(xr)).numpy()
    # patches that become constant after the resize (all-0, all-255, the 1-px checkerboard)
    # hit input_norm's std=0 path, where (x - mean)/(0 + 1e-7) amplifies the rounding of the
    # mean by 1e7 in any implementation, so the result depends on summation order
    ok = xr.reshape(len(xr), -1).std(1) > 1e-3
    assert ok.sum() >= len(xr) - 4
    assert np.abs(y[ok] - ref[ok]).max() <= 1e-4


@pytest.mark.gpu
def test_preprocess_rejects_wrong_shapes(cuda_device):
    with pytest.raises(ValueError):
        N.preprocess(torch.zeros((2, 32, 32), dtype=torch.uint8, device=cuda_device), resize="cv2")
    with pytest.raises(ValueError):
        N.preprocess(torch.zeros((2, 64, 64), dtype=torch.float32, device=cuda_device))


# ------------------------------------------------- fused preprocessing (hn_forward_u8) ----
def _u8_batch(n, seed, hw=64):
    """The Pillow fixture patches, tiled and perturbed to n patches (edges: 0 / 255 blocks)."""
    fx = _fx()
    base = fx["u8_64"] if hw == 64 else fx["pil_u8_32"]
    g = np.random.default_rng(seed)
    reps = -(-n // base.shape[0])
    u = np.concatenate([base] * reps)[:n].astype(np.int32)
    u = (u + g.integers(-3, 4, size=u.shape)).clip(0, 255).astype(np.uint8)
    u[0] = 0
    if n > 1:
        u[1] = 255
    return u


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["hardnet", "wang2", "wang3", "wang4", "fdl_NASNet", "fdl_NASNet_01"])
@pytest.mark.parametrize("resize,normalize", [("pil", False), ("pil", True), ("cv2", True), ("none", True)])
@pytest.mark.parametrize("n", [1, 37, 3001])
def test_forward_u8_equals_preprocess_then_forward(name, resize, normalize, n, cuda_device):
    """hn_forward_u8 == hn_preprocess followed by hn_forward, bit for bit, with the preprocessing fused
    into the first kernel's patch load in every mode (HardNet: k_c12's; FDLNet: k_fdl_front_mfma's; NAS:
    k_front's -- wang2 the k3 no-fold form, wang3 k5, wang4 the maxpool form; PIL through the staged
    raw patch in the pw ring, except on the k5 front (wang3), where the separate pass is faster);
    3,001 patches run every persistent workgroup over several patches and end on a ragged one."""
    m, _, _ = build_module(name)
    nm = N.NativeModel.from_module(m, cuda_device)
    hw = 32 if resize == "none" else 64
    u = torch.from_numpy(_u8_batch(n, 7, hw)).to(cuda_device)
    ref = nm.forward(N.preprocess(u, resize=resize, normalize=normalize))
    nm.set_profiling(True)
    got = nm.forward_u8(u, resize=resize, normalize=normalize)
    st = nm.stage_times()
    assert ("preprocess" in st) == (name == "wang3" and resize == "pil")
    assert torch.equal(got, ref)


@pytest.mark.gpu
def test_forward_u8_nas_fold_form_preprocesses_apart(cuda_device, monkeypatch):
    """HN_FRONT_FOLD (the round-2 front, no uint8 load) takes the hn_preprocess path, same result."""
    m, _, _ = build_module("wang2")
    u = torch.from_numpy(_u8_batch(37, 5, 64)).to(cuda_device)
    ref = N.NativeModel.from_module(m, cuda_device).forward_u8(u, resize="cv2")
    monkeypatch.setenv("HN_FRONT_FOLD", "1")
    nm = N.NativeModel.from_module(m, cuda_device)
    nm.set_profiling(True)
    got = nm.forward_u8(u, resize="cv2")
    assert "preprocess" in nm.stage_times()
    assert (got - ref).abs().max().item() <= 2e-5


@pytest.mark.gpu
def test_forward_u8_matches_the_reference_chain(cuda_device):
    """PIL fixtures -> (Pillow resize, ToTensor, Normalize) -> the fp32 oracle forward, against
    the fused uint8 forward: the whole reference data path at the descriptor tolerance."""
    fx = _fx()
    m, _, p = build_module("hardnet")
    nm = N.NativeModel.from_module(m, cuda_device)
    got = nm.forward_u8(torch.from_numpy(fx["u8_64"]).to(cuda_device), resize="pil").cpu()
    t = {k: torch.from_numpy(v) for k, v in p.items()}
    x = torch.from_numpy(fx["pil_norm_f32"])
    ref = O.hardnet_forward(t, x)
    # constant patches (fixture rows 0 / 1, all 0 / all 255) are excluded: after Normalize their
    # pixels are one fp32 value whose mean rounds differently per summation order, and
    # input_norm's 1 / (0 + 1e-7) turns that rounding into the descriptor (ill-posed in fp32 for
    # the reference itself); the same patches through hn_forward agree bit for bit above
    keep = x.flatten(1).std(dim=1) > 1e-3
    assert int(keep.sum()) >= x.shape[0] - 4
    assert (got[keep] - ref[keep]).abs().max().item() <= 1e-4


def test_abi_rejects_bad_forward_u8_args_without_gpu():
    lib = N.load_library()
    assert lib.hn_forward_u8(None, None, 4, 64, 1, 1, 0.0, 1.0, None, None, 0, None) == 1
    assert b"model" in lib.hn_last_error()
