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
    assert lib.hn_abi_version() == 1


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
