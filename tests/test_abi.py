"""C ABI checks that need no GPU: the library loads, exports every symbol declared in
include/hardnet_mi355x.h, validates descriptors, and agrees with the Python side on the
parameter-blob layout."""
import ctypes
import os
import re

import numpy as np
import pytest

from fixtures import NAS_NAMES, build_module
from hardnetnas_amd import _native as N
from hardnetnas_amd import arch as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "hardnet_mi355x.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(hn_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree():
    assert _declared_symbols() == sorted(N.EXPORTED)


def test_library_exports_every_symbol():
    lib = N.load_library()
    for s in _declared_symbols():
        assert hasattr(lib, s), s
    assert lib.hn_abi_version() == 2


def test_param_count_hardnet_matches_state_dict():
    m, _, _ = build_module("hardnet")
    blob = N.state_dict_blob(m.state_dict())
    n = ctypes.c_size_t()
    assert N.load_library().hn_param_count(ctypes.byref(N.hardnet_desc()), ctypes.byref(n)) == 0
    assert n.value == blob.size == 1334560 + 2 * 576


@pytest.mark.parametrize("name", NAS_NAMES)
def test_param_count_nas_matches_state_dict(name):
    m, _, _ = build_module(name)
    blob = N.state_dict_blob(m.state_dict())
    n = ctypes.c_size_t()
    d = N.nas_desc(m.arch_ops)
    assert N.load_library().hn_param_count(ctypes.byref(d), ctypes.byref(n)) == 0
    assert n.value == blob.size


@pytest.mark.parametrize("variant", A.FDL_VARIANTS)
def test_param_count_fdl_matches_state_dict(variant):
    """FDLNet HardNetNeiMask: the front + IRFBlock + head parameters hn_create parses equal
    the module's state_dict blob (reference layout, tests/test_oracle_golden.py)."""
    from hardnetnas_amd.model import HardNetNeiMask
    m = HardNetNeiMask(variant=variant)
    n = ctypes.c_size_t()
    d = N.desc_for_module(m)
    assert d.kind == (N.HN_KIND_FDL_NASNET if variant == "NASNet" else N.HN_KIND_FDL_NASNET01)
    assert N.load_library().hn_param_count(ctypes.byref(d), ctypes.byref(n)) == 0
    assert n.value == N.state_dict_blob(m.state_dict()).size
    d.c_in[0] = 32  # the FDL front leaves 64 channels
    assert N.load_library().hn_param_count(ctypes.byref(d), ctypes.byref(n)) == 1


def test_every_candidate_op_param_count():
    """Single-op archs for each of the 17 CANDIDATE_BLOCKS at every layer slot."""
    from hardnetnas_amd.model import HardNetNAS
    lib = N.load_library()
    for op in A.CANDIDATE_BLOCKS:
        ops = [op] * 6
        m = HardNetNAS(ops)
        n = ctypes.c_size_t()
        assert lib.hn_param_count(ctypes.byref(N.nas_desc(ops)), ctypes.byref(n)) == 0, op
        assert n.value == N.state_dict_blob(m.state_dict()).size, op


def test_bad_descriptors_are_rejected_with_message():
    lib = N.load_library()
    n = ctypes.c_size_t()
    d = N.nas_desc(A.MODEL_ARCH["wang2"])
    d.op[2] = 99
    assert lib.hn_param_count(ctypes.byref(d), ctypes.byref(n)) == 1
    assert b"op index" in lib.hn_last_error()
    d = N.nas_desc(A.MODEL_ARCH["wang2"])
    d.c_in[3] = 48
    assert lib.hn_param_count(ctypes.byref(d), ctypes.byref(n)) == 1
    assert b"chain" in lib.hn_last_error()
    d = N.HnArchDesc()
    d.kind = 7
    assert lib.hn_param_count(ctypes.byref(d), ctypes.byref(n)) == 1


def test_create_rejects_wrong_blob_size_without_touching_gpu():
    lib = N.load_library()
    h = ctypes.c_void_p()
    blob = np.zeros(10, np.float32)
    rc = lib.hn_create(ctypes.byref(N.hardnet_desc()), blob.ctypes.data, blob.size, ctypes.byref(h))
    assert rc == 1 and b"expected" in lib.hn_last_error()
    assert not h.value


def test_eval_cuda_path_has_no_silent_fallback(monkeypatch):
    """If the library is missing, the native entry point raises (no CPU fallback)."""
    monkeypatch.setattr(N, "_lib", None)
    monkeypatch.setenv("HN_LIB", "/nonexistent/libhardnet_mi355x.so")
    with pytest.raises(RuntimeError, match="not found"):
        N.load_library()


def test_bench_knows_every_hardnet_stage():
    """bench.py's per-stage FLOP/byte tables cover every stage name hn_forward records."""
    import bench
    src = open(os.path.join(ROOT, "hardnetnas_amd", "csrc", "hn_api.hip")).read()
    fwd = src[src.index("static int forward_hardnet("):src.index("static int forward_nas(")]
    names = set(re.findall(r'STAGE\("([^"]+)"', fwd))
    assert names and names <= set(bench.HARDNET_STAGE_MAC) and names <= set(bench.HARDNET_STAGE_BYTES)


def test_bench_knows_every_nas_stage(monkeypatch):
    """bench.py's NAS byte / FLOP tables cover every stage name forward_nas records, and its mirror of the
    dispatch puts wang3's layers 2-4 in k_irf_skip ("irf+skip": the block's input in, the skip's 4x4x128 out,
    both layers' FLOP) unless HN_NO_IRFSKIP; the FLOP table sums to the architecture's total either way."""
    import bench
    from hardnetnas_amd import arch as A
    src = open(os.path.join(ROOT, "hardnetnas_amd", "csrc", "hn_api.hip")).read()
    fwd = src[src.index("static int forward_nas("):src.index('extern "C" int hn_forward(')]
    names = set(re.findall(r'STAGE\("([^"]+)"', fwd))
    assert "irf+skip" in names and names <= set(bench.nas_stage_bytes("wang2"))
    assert bench.irf_skip_layers("wang3") == {2: 4} and bench.irf_skip_layers("wang2") == {}
    assert bench.irf_skip_layers(["ir_k3_e1", "skip", "ir_k5_e3_se", "skip", "skip", "skip"]) == {}  # SE: unfused
    b, f = bench.nas_stage_bytes("wang3"), bench.nas_stage_flop("wang3")
    assert b["irf+skip"] == 4 * 32 * 16 * 16 + 4 * 128 * 4 * 4 and b["irf"] == b["skip"] == 0
    assert sum(f.values()) == 2 * A.nas_macs("wang3")
    monkeypatch.setenv("HN_NO_IRFSKIP", "1")
    assert bench.irf_skip_layers("wang3") == {}
    b, f = bench.nas_stage_bytes("wang3"), bench.nas_stage_flop("wang3")
    assert b["irf+skip"] == 0 and b["irf"] > 0 and b["skip"] > 0 and sum(f.values()) == 2 * A.nas_macs("wang3")


def test_bench_knows_the_maxpool_front_fusion(monkeypatch):
    """bench.py's mirror of forward_nas's k_mpfront_irf dispatch: wang4 (layers 0 / 1 "skip", layer 2 ir_k5_s2)
    runs its front, the identity and layer 2 as one "front+irf" stage (the patch in, 8x8x64 out, all three
    layers' FLOP), and a layer-2 block with SE, or HN_NO_MPFRONT, keeps the separate kernels."""
    import bench
    from hardnetnas_amd import arch as A
    assert bench.mpfront_irf("wang4") and not bench.mpfront_irf("wang2") and not bench.mpfront_irf("wang3")
    assert not bench.mpfront_irf(["skip", "skip", "ir_k5_e1_se", "skip", "skip", "skip"])
    b, f = bench.nas_stage_bytes("wang4"), bench.nas_stage_flop("wang4")
    assert b["front+irf"] == 4096 + 4 * 64 * 8 * 8 and b["front"] == 0
    assert f["front"] == 0 and sum(f.values()) == 2 * A.nas_macs("wang4")
    monkeypatch.setenv("HN_NO_MPFRONT", "1")
    b, f = bench.nas_stage_bytes("wang4"), bench.nas_stage_flop("wang4")
    assert b["front+irf"] == 0 and b["front"] > 0 and sum(f.values()) == 2 * A.nas_macs("wang4")


def _kernel_template_args(kernel: str):
    """Template argument lists of every `kernel<...>` symbol in the product library (nm -C)."""
    import subprocess
    out = subprocess.run(["nm", "-C", "--defined-only", N.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    return [m.split(",") for m in re.findall(kernel + r"<([^<>]*)>\(", out)]


def test_product_library_has_no_ablation_builds():
    """The timing-only ablation builds (wrong results by construction) live only in the
    HN_EXPERIMENTS library: no k_conv_ws / k_conv_pipe (ABL = 10th template argument) or k_c12
    (ABL = 1st) instantiation in libhardnet_mi355x.so carries a nonzero ABL."""
    ws = _kernel_template_args("k_conv_ws")
    pipe = _kernel_template_args("k_conv_pipe")
    c12 = _kernel_template_args("k_c12")
    assert ws and pipe and c12
    for args in ws + pipe:
        assert int(args[9]) == 0, args
    for args in c12:
        assert int(args[0]) == 0, args


def test_product_library_has_one_tiling_per_layer_plus_fallbacks():
    """Measured-and-rejected kernels live only in the HN_EXPERIMENTS library:
    no 2-D Winograd kernel (hn_wino.hip), and of k_conv_pipe only conv5's production instantiation
    (the store-through-LDS form, CST = last template argument true)."""
    import subprocess
    out = subprocess.run(["nm", "-C", "--defined-only", N.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    assert "k_wino<" not in out and "hn_launch_wino(" not in out  # the 2-D F(2x2,3x3) form
    assert "k_conv_w1<" in out  # the 1-D F(2,3) conv3 / conv5 (hn_wino1.hip), the default
    pipe = _kernel_template_args("k_conv_pipe")
    assert pipe and all(a[-1].strip() == "true" for a in pipe), pipe


@pytest.mark.parametrize("env,val", [("HN_VARIANT", "888888"), ("HN_VARIANT", "004000"),
                                     ("HN_VARIANT", "00000z"), ("HN_VARIANT", "000h00"),
                                     ("HN_VARIANT", "111111"), ("HN_C12_CFG", "13"),
                                     ("HN_C12_CFG", "14"), ("HN_C12_CFG", "7"), ("HN_VARIANT", "605wil"),
                                     ("HN_VARIANT", "605jij"), ("HN_VARIANT", "605565"), ("HN_HEAD", "5")])
def test_create_rejects_ablation_and_unknown_builds(env, val, monkeypatch):
    """hn_create validates the A/B switches before touching the GPU: an ablation tiling or an
    unknown k_c12 configuration is HN_ERR_ARG, never a silently wrong model."""
    m, _, _ = build_module("hardnet")
    blob = N.state_dict_blob(m.state_dict())
    monkeypatch.setenv(env, val)
    lib = N.load_library()
    h = ctypes.c_void_p()
    rc = lib.hn_create(ctypes.byref(N.hardnet_desc()), blob.ctypes.data, blob.size, ctypes.byref(h))
    assert rc == 1, lib.hn_last_error()
    assert env.encode() in lib.hn_last_error()
    assert not h.value


def test_registered_torch_op_and_fake_kernel():
    """torch.ops.hardnet_mi355x.forward exists (registered at import) and its fake kernel gives
    the [B,128] result shape that torch.compile traces with."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode
    assert hasattr(torch.ops.hardnet_mi355x, "forward")
    with FakeTensorMode():
        y = torch.ops.hardnet_mi355x.forward(torch.empty(7, 1, 32, 32), 1)
    assert tuple(y.shape) == (7, 128)


def test_cpu_and_train_calls_use_the_torch_layers():
    """CPU tensors and train mode never reach the native path (reference semantics), with or
    without strict."""
    import torch
    from hardnetnas_amd.model import HardNet
    m = HardNet(strict=True).eval()
    x = torch.randn(3, 1, 32, 32)
    with torch.no_grad():
        assert m(x).shape == (3, 128)
    m.train()
    y = m(torch.randn(4, 1, 32, 32))
    y.sum().backward()
    assert getattr(m, "_hn_handle", None) is None


@pytest.mark.parametrize("kind", ["wang2", "cov_b", "supernet", "fdl_NASNet", "fdl_NASNet_01"])
def test_train_tensor_count_matches_module(kind):
    """hn_nas_train_tensor_count walks the same float tensors, in the same order, as the module's
    state_dict minus num_batches_tracked / thetas (_native.train_tensors): NAS, supernet, FDLNet."""
    from hardnetnas_amd.model import HardNetNASSupernet
    if kind == "supernet":
        m, d = HardNetNASSupernet(), N.supernet_desc()
    else:
        m, _, _ = build_module(kind)
        d = N.desc_for_module(m)
    n = ctypes.c_size_t()
    assert N.load_library().hn_nas_train_tensor_count(ctypes.byref(d), ctypes.byref(n)) == 0, \
        N.load_library().hn_last_error()
    assert n.value == len(N.train_tensors(m)[1])


def test_train_rejects_fdl_without_input_norm():
    d = N.fdl_desc("NASNet")
    d.input_norm_eps = -1.0
    n = ctypes.c_size_t()
    assert N.load_library().hn_nas_train_tensor_count(ctypes.byref(d), ctypes.byref(n)) == 1
    assert b"input_norm" in N.load_library().hn_last_error()


def test_bench_supernet_train_leg_flop_count():
    """bench.py's train_supernet leg prices its roofline with FlopCounterMode over the supernet's torch layers:
    that count equals the analytic per-patch MACs of the stem, all 17 candidate ops of all six searched
    layers (arch.layer_macs) and the 4x4 head, x 2 (within the SE modules' pooling / bias terms)."""
    import bench
    from hardnetnas_amd import arch as A
    hw, macs = 32, A.STEM_CHANNELS * 9 * 32 * 32
    for ci, co, s in A.SEARCH_SPACE2:
        macs += sum(A.layer_macs(ci, co, s, op, hw) for op in A.CANDIDATE_BLOCKS)
        hw //= s
    macs += A.SEARCH_SPACE2[-1][1] * A.DESC_DIM * A.HEAD_KERNEL ** 2
    assert abs(bench.supernet_flop_per_patch() / (2 * macs) - 1) < 1e-4
    assert bench.SUPERNET_PAIRS == 128


def test_bench_three_block_fusion_is_experiments_only(monkeypatch):
    """k_irf3 (layers 3 -> 4 -> 5 in one kernel) measured slower and lives in the experiments library: bench.py's
    stage mirror counts an "irf3" stage only for HN_IRF3=1 on that library, else wang4 keeps irf2 + irf."""
    import bench
    from hardnetnas_amd import arch as A
    monkeypatch.setenv("HN_IRF3", "1")
    assert bench.irf3_triples("wang4") == set()
    b = bench.nas_stage_bytes("wang4")
    assert b["irf3"] == 0 and b["irf2"] > 0 and b["irf"] > 0
    monkeypatch.setenv("HN_LIB", "/x/abl/libhardnet_mi355x.so")
    assert bench.irf3_triples("wang4") == {3} and bench.irf3_triples("wang2") == set()
    b, f = bench.nas_stage_bytes("wang4"), bench.nas_stage_flop("wang4")
    assert b["irf3"] == 4 * 64 * 8 * 8 + 4 * 128 * 16 and b["irf2"] == 0 and b["irf"] == 0
    assert sum(f.values()) == 2 * A.nas_macs("wang4")


@pytest.mark.parametrize("kind", ["supernet", "wang2", "fdl"])
def test_nas_train_walk_matches_train_tensors(kind):
    """The NAS train path gathers its tensor list and BatchNorms in one pass over the module tree
    (model._nas_train_walk); the list must be _native.train_tensors' (the float state_dict minus
    num_batches_tracked and the thetas, in order -- the order hn_nas_train_* walks), object for object,
    and a wrong-device or non-contiguous tensor, or a BatchNorm the kernels do not implement, refuses."""
    import torch
    from hardnetnas_amd import model as MD
    from hardnetnas_amd._native import train_tensors
    m = {"supernet": lambda: MD.HardNetNASSupernet(), "wang2": lambda: MD.HardNetNAS("wang2"),
         "fdl": lambda: MD.HardNetNeiMask(variant="NASNet")}[kind]().train()
    walk = MD._nas_train_walk(m, torch.device("cpu"))
    assert walk is not None
    bns, tensors = walk
    ref = train_tensors(m)[1]
    assert len(tensors) == len(ref) and all(a is b for a, b in zip(tensors, ref))
    assert bns == [b for b in m.modules() if isinstance(b, torch.nn.BatchNorm2d)]
    assert MD._nas_train_walk(m, torch.device("meta")) is None
    bns[0].eps = 1e-3
    assert MD._nas_train_walk(m, torch.device("cpu")) is None
