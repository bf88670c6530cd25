"""ctypes binding of the C ABI in include/hardnet_mi355x.h (libhardnet_mi355x.so).

PyTorch is only plumbing here: it owns device memory (inputs, outputs, workspace via
the caching allocator) and the current HIP stream; all arithmetic of the forward runs
in the library's gfx950 kernels.  ``torch`` is imported before the library is loaded so
that both share the one HIP runtime already mapped by torch (SONAME libamdhip64.so.7).

There is no fallback: if the library cannot be loaded, every entry point raises.
"""
from __future__ import annotations

import ctypes
import itertools
import os
import threading
import weakref
from typing import Dict, List, Optional

import numpy as np
import torch

from . import arch as A

_LIB_NAME = "libhardnet_mi355x.so"
_lib = None
_lib_lock = threading.Lock()

HN_KIND_HARDNET = 0
HN_KIND_NAS = 1
HN_KIND_FDL_NASNET = 2
HN_KIND_FDL_NASNET01 = 3
HN_KIND_NAS_SUPERNET = 4  # train mode only (hn_nas_train_*)
HN_MAX_LAYERS = 8
ABI_VERSION = 2   # HN_ABI_VERSION of include/hardnet_mi355x.h


class HnArchDesc(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("n_layers", ctypes.c_int32),
        ("op", ctypes.c_int32 * HN_MAX_LAYERS),
        ("c_in", ctypes.c_int32 * HN_MAX_LAYERS),
        ("c_out", ctypes.c_int32 * HN_MAX_LAYERS),
        ("stride", ctypes.c_int32 * HN_MAX_LAYERS),
        ("input_norm_eps", ctypes.c_float),
        ("l2_eps", ctypes.c_float),
        ("bn_eps", ctypes.c_float),
    ]


EXPORTED = ["hn_param_count", "hn_create", "hn_workspace_bytes", "hn_forward",
            "hn_pairdist_workspace_bytes", "hn_pairdist_hardneg", "hn_pairdist_rows_workspace_bytes",
            "hn_pairdist_rows", "hn_hardnet_loss", "hn_workspace_bytes_u8", "hn_forward_u8",
            "hn_hardnet_train_workspace_bytes", "hn_hardnet_train_forward", "hn_hardnet_train_backward",
            "hn_nas_train_tensor_count", "hn_nas_train_workspace_bytes", "hn_nas_train_forward",
            "hn_nas_train_backward", "hn_hardnet_loss_train_workspace_bytes", "hn_hardnet_loss_train_forward",
            "hn_hardnet_loss_backward", "hn_fpr95_workspace_bytes",
            "hn_fpr95", "hn_preprocess", "hn_set_profiling",
            "hn_stage_times", "hn_destroy", "hn_last_error", "hn_abi_version"]


def lib_path() -> str:
    env = os.environ.get("HN_LIB")
    if env:
        return env
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", _LIB_NAME)


def load_library():
    """Load (once) and type the C ABI.  Raises if the library is missing."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(
                f"hardnetnas_amd native library not found at {path}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (make -C hardnetnas_amd/csrc)")
        lib = ctypes.CDLL(path)
        P, S, I32, I64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int64
        lib.hn_param_count.argtypes = [ctypes.POINTER(HnArchDesc), ctypes.POINTER(S)]
        lib.hn_create.argtypes = [ctypes.POINTER(HnArchDesc), P, S, ctypes.POINTER(P)]
        lib.hn_workspace_bytes.argtypes = [P, I64, ctypes.POINTER(S)]
        lib.hn_forward.argtypes = [P, P, I64, P, P, S, P]
        lib.hn_workspace_bytes_u8.argtypes = [P, I64, ctypes.POINTER(S)]
        PP = ctypes.POINTER(P)
        lib.hn_hardnet_train_workspace_bytes.argtypes = [I64, ctypes.POINTER(S), ctypes.POINTER(S)]
        lib.hn_hardnet_train_forward.argtypes = [P, I64, PP, PP, PP, ctypes.c_float, ctypes.c_float,
                                                 ctypes.c_uint64, P, P, S, P, S, P]
        lib.hn_hardnet_train_backward.argtypes = [P, I64, PP, PP, P, ctypes.c_float, ctypes.c_uint64, P, S, P, S, P]
        lib.hn_forward_u8.argtypes = [P, P, I64, I32, I32, I32, ctypes.c_float, ctypes.c_float, P, P, S, P]
        D = ctypes.POINTER(HnArchDesc)
        lib.hn_nas_train_tensor_count.argtypes = [D, ctypes.POINTER(S)]
        lib.hn_nas_train_workspace_bytes.argtypes = [D, I64, ctypes.POINTER(S), ctypes.POINTER(S)]
        lib.hn_nas_train_forward.argtypes = [D, P, I64, PP, ctypes.c_float, P, P, P, S, P, S, P]
        lib.hn_nas_train_backward.argtypes = [D, P, P, I64, PP, P, PP, P, P, S, P, S, P]
        lib.hn_pairdist_workspace_bytes.argtypes = [I64, ctypes.POINTER(S)]
        lib.hn_pairdist_hardneg.argtypes = [P, P, I64, I32, I32, P, P, P, S, P]
        lib.hn_pairdist_rows_workspace_bytes.argtypes = [I64, I64, ctypes.POINTER(S)]
        lib.hn_pairdist_rows.argtypes = [P, I64, I64, P, I64, I32, P, P, P, P, S, P]
        lib.hn_hardnet_loss.argtypes = [P, P, P, I64, ctypes.c_float, I32, ctypes.c_float, P, P, P]
        lib.hn_hardnet_loss_train_workspace_bytes.argtypes = [I64, ctypes.POINTER(S)]
        lib.hn_hardnet_loss_train_forward.argtypes = [P, P, I64, I32, I32, ctypes.c_float, I32, P, P, S, P]
        lib.hn_hardnet_loss_backward.argtypes = [P, P, I64, I32, I32, ctypes.c_float, I32, P, P, P, P, S, P]
        lib.hn_fpr95_workspace_bytes.argtypes = [I64, ctypes.POINTER(S)]
        lib.hn_fpr95.argtypes = [P, P, P, I64, I32, P, P, P, S, P]
        lib.hn_preprocess.argtypes = [P, I64, I32, I32, I32, ctypes.c_float, ctypes.c_float, P, P]
        lib.hn_set_profiling.argtypes = [P, ctypes.c_int]
        lib.hn_stage_times.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                       ctypes.POINTER(ctypes.c_double), ctypes.POINTER(I64)]
        lib.hn_destroy.argtypes = [P]
        lib.hn_destroy.restype = None
        lib.hn_last_error.restype = ctypes.c_char_p
        for name in ("hn_param_count", "hn_create", "hn_workspace_bytes", "hn_forward",
                     "hn_pairdist_workspace_bytes", "hn_pairdist_hardneg", "hn_abi_version",
                     "hn_set_profiling", "hn_stage_times", "hn_fpr95_workspace_bytes",
                     "hn_fpr95", "hn_pairdist_rows_workspace_bytes", "hn_pairdist_rows",
                     "hn_hardnet_loss", "hn_workspace_bytes_u8", "hn_forward_u8",
                     "hn_hardnet_train_workspace_bytes", "hn_hardnet_train_forward",
                     "hn_hardnet_train_backward", "hn_nas_train_tensor_count", "hn_nas_train_workspace_bytes",
                     "hn_nas_train_forward", "hn_nas_train_backward", "hn_hardnet_loss_train_workspace_bytes",
                     "hn_hardnet_loss_train_forward", "hn_hardnet_loss_backward"):
            getattr(lib, name).restype = ctypes.c_int
        if lib.hn_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{path}: ABI version {lib.hn_abi_version()}, expected {ABI_VERSION}; rebuild it")
        _lib = lib
        return lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = load_library().hn_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")


# ----------------------------------------------------------------------------------
# descriptors and parameter blobs
# ----------------------------------------------------------------------------------
def hardnet_desc(input_norm_eps: float = 1e-7, l2_eps: float = 1e-10) -> HnArchDesc:
    d = HnArchDesc()
    d.kind = HN_KIND_HARDNET
    d.input_norm_eps = input_norm_eps
    d.l2_eps = l2_eps
    d.bn_eps = 1e-5
    return d


def nas_desc(ops: List[str], layers=None, input_norm_eps: float = -1.0,
             l2_eps: float = 0.0) -> HnArchDesc:
    layers = layers or A.SEARCH_SPACE2
    d = HnArchDesc()
    d.kind = HN_KIND_NAS
    d.n_layers = len(ops)
    for i, (op, (ci, co, s)) in enumerate(zip(ops, layers)):
        d.op[i] = A.CANDIDATE_BLOCKS.index(op)
        d.c_in[i], d.c_out[i], d.stride[i] = ci, co, s
    d.input_norm_eps = input_norm_eps
    d.l2_eps = l2_eps
    d.bn_eps = 1e-5
    return d


def fdl_desc(variant: str = "NASNet", input_norm_eps: float = A.FDL_INPUT_NORM_EPS) -> HnArchDesc:
    """FDLNet HardNetNeiMask (latency/NASNet{,_0.1}/model/des.py): the fixed front is implied
    by the kind; the three IRFBlocks are described like NAS layers."""
    d = nas_desc(A.FDL_OPS, A.FDL_LAYERS, input_norm_eps=input_norm_eps, l2_eps=0.0)
    d.kind = HN_KIND_FDL_NASNET if variant == "NASNet" else HN_KIND_FDL_NASNET01
    return d


def state_dict_blob(sd: Dict[str, torch.Tensor]) -> np.ndarray:
    """Concatenate every float tensor of a state_dict in state_dict order, skipping
    ``num_batches_tracked``.  This is exactly the order hn_create parses:
      HardNet: features.{0,3,...,19}.weight followed by the BN running_mean/var;
      NAS:     first.conv/bn(w,b,mean,var), per block pw/dw/pwl ConvBNRelu (and
               se4.op.{1,3}.{weight,bias}) or the skip's 1x1 ConvBNRelu, then
               last_stages.conv_k1.weight + last_stages.batchnorm running stats;
      FDL:     features.0.{weight,bias}, the front's BN stats / 1x1 ConvBN(Relu)s, the
               IRFBlocks as for NAS, the head conv weight + BN running stats."""
    parts = [v.detach().to("cpu", torch.float32).contiguous().reshape(-1).numpy()
             for k, v in sd.items() if not k.endswith("num_batches_tracked")]
    return np.ascontiguousarray(np.concatenate(parts), dtype=np.float32)


def desc_for_module(module) -> HnArchDesc:
    from .model import HardNet, HardNetNAS, HardNetNeiMask
    if isinstance(module, HardNet):
        return hardnet_desc(module.input_norm_eps, module.l2_eps)
    if isinstance(module, HardNetNeiMask):
        return fdl_desc(module.variant, module.input_norm_eps)
    if isinstance(module, HardNetNAS):
        return nas_desc(module.arch_ops, module.layers)
    raise TypeError(type(module))


_OP_IDS = itertools.count(1)
_BY_ID: "weakref.WeakValueDictionary[int, NativeModel]" = weakref.WeakValueDictionary()


class NativeModel:
    """A device model (packed, BN-folded weights) created through hn_create."""

    def __init__(self, desc: HnArchDesc, blob: np.ndarray, device: torch.device):
        self.op_id = next(_OP_IDS)  # the ``handle`` argument of torch.ops.hardnet_mi355x.forward
        _BY_ID[self.op_id] = self
        self.lib = load_library()
        self.device = torch.device(device)
        self.desc = desc
        n = ctypes.c_size_t()
        _check(self.lib.hn_param_count(ctypes.byref(desc), ctypes.byref(n)), "hn_param_count")
        if n.value != blob.size:
            raise ValueError(f"parameter blob has {blob.size} floats, library expects {n.value}")
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _check(self.lib.hn_create(ctypes.byref(desc), blob.ctypes.data, blob.size,
                                      ctypes.byref(h)), "hn_create")
        self._h = h

    @classmethod
    def from_module(cls, module, device) -> "NativeModel":
        return cls(desc_for_module(module), state_dict_blob(module.state_dict()), device)

    def workspace_bytes(self, batch: int) -> int:
        n = ctypes.c_size_t()
        _check(self.lib.hn_workspace_bytes(self._h, batch, ctypes.byref(n)), "hn_workspace_bytes")
        return n.value

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None,
                workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
        if x.device != self.device:
            raise ValueError(f"input on {x.device}, model on {self.device}")
        if x.dtype != torch.float32 or x.dim() != 4 or tuple(x.shape[1:]) != (1, 32, 32):
            raise ValueError(f"expected fp32 [B,1,32,32], got {x.dtype} {tuple(x.shape)}")
        x = x.contiguous()
        b = x.shape[0]
        if out is None:
            out = torch.empty((b, 128), device=self.device, dtype=torch.float32)
        elif (tuple(out.shape) != (b, 128) or out.dtype != torch.float32 or out.device != self.device
              or not out.is_contiguous()):
            raise ValueError(f"out must be a contiguous fp32 [{b},128] tensor on {self.device}, got "
                             f"{out.dtype} {tuple(out.shape)} on {out.device}")
        ws_bytes = self.workspace_bytes(b)
        if workspace is not None and (workspace.dtype != torch.uint8 or workspace.device != self.device
                                      or not workspace.is_contiguous()):
            raise ValueError(f"workspace must be a contiguous uint8 tensor on {self.device}")
        if workspace is None or workspace.numel() < ws_bytes:
            workspace = torch.empty(max(ws_bytes, 16), device=self.device, dtype=torch.uint8)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        with torch.cuda.device(self.device):
            _check(self.lib.hn_forward(self._h, x.data_ptr(), b, out.data_ptr(),
                                       workspace.data_ptr(), workspace.numel(), stream),
                   "hn_forward")
        return out

    __call__ = forward

    def forward_u8(self, u8: torch.Tensor, resize: str = "cv2", normalize: bool = True,
                   mean: float = 0.443728476019, std: float = 0.20197947209,
                   out: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Descriptors straight from uint8 patches ([n,64,64] / [n,1,64,64]; [n,32,32] for
        resize='none'): the loader transforms (hardnet/HardNet.py:333-337, 345-349) fused into the
        forward -- equal to ``forward(preprocess(u8, ...))`` bit for bit."""
        if resize not in RESIZE_MODES:
            raise ValueError(f"resize must be one of {sorted(RESIZE_MODES)}")
        if u8.dtype != torch.uint8 or u8.device != self.device:
            raise ValueError(f"expected a uint8 tensor on {self.device}")
        hw = 32 if resize == "none" else 64
        b = u8.shape[0]
        if u8.numel() != b * hw * hw:
            raise ValueError(f"expected {hw}x{hw} patches, got shape {tuple(u8.shape)}")
        x = u8.contiguous()
        if out is None:
            out = torch.empty((b, 128), device=self.device, dtype=torch.float32)
        elif (tuple(out.shape) != (b, 128) or out.dtype != torch.float32 or out.device != self.device
              or not out.is_contiguous()):
            raise ValueError(f"out must be a contiguous fp32 [{b},128] tensor on {self.device}")
        n = ctypes.c_size_t()
        _check(self.lib.hn_workspace_bytes_u8(self._h, b, ctypes.byref(n)), "hn_workspace_bytes_u8")
        if workspace is not None and (workspace.dtype != torch.uint8 or workspace.device != self.device
                                      or not workspace.is_contiguous()):
            raise ValueError(f"workspace must be a contiguous uint8 tensor on {self.device}")
        if workspace is None or workspace.numel() < n.value:
            workspace = torch.empty(max(n.value, 16), device=self.device, dtype=torch.uint8)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        with torch.cuda.device(self.device):
            _check(self.lib.hn_forward_u8(self._h, x.data_ptr(), b, hw, RESIZE_MODES[resize], int(normalize),
                                          mean, std, out.data_ptr(), workspace.data_ptr(), workspace.numel(),
                                          stream), "hn_forward_u8")
        return out

    def workspace_bytes_u8(self, batch: int) -> int:
        n = ctypes.c_size_t()
        _check(self.lib.hn_workspace_bytes_u8(self._h, batch, ctypes.byref(n)), "hn_workspace_bytes_u8")
        return n.value

    def set_profiling(self, on: bool):
        _check(self.lib.hn_set_profiling(self._h, int(on)), "hn_set_profiling")

    def stage_times(self) -> Dict[str, tuple]:
        """{stage: (total_ms, launches)} accumulated since the last call (waits on the
        recorded events; call after the stream has been synchronised)."""
        n = 32
        names = (ctypes.c_char_p * n)()
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        k = self.lib.hn_stage_times(self._h, n, names, ms, cnt)
        if k < 0:
            _check(-k, "hn_stage_times")
        return {names[i].decode(): (ms[i], cnt[i]) for i in range(k)}

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.hn_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pairdist_hardneg(anchor: torch.Tensor, positive: torch.Tensor, anchor_swap: bool = False):
    """(pos, min_neg) of loss_HardNet's 'min' batch_reduce (hardnet/Losses.py:87-110),
    computed by the fused kernel without materialising the BxB distance matrix."""
    lib = load_library()
    if anchor.shape != positive.shape or anchor.dim() != 2:
        raise ValueError("anchor/positive must be equal [B,D]")
    a = anchor.contiguous().float()
    p = positive.contiguous().float()
    b, d = a.shape
    n = ctypes.c_size_t()
    _check(lib.hn_pairdist_workspace_bytes(b, ctypes.byref(n)), "hn_pairdist_workspace_bytes")
    ws = torch.empty(max(n.value, 16), device=a.device, dtype=torch.uint8)
    pos = torch.empty(b, device=a.device, dtype=torch.float32)
    mn = torch.empty(b, device=a.device, dtype=torch.float32)
    stream = torch.cuda.current_stream(a.device).cuda_stream
    with torch.cuda.device(a.device):
        _check(lib.hn_pairdist_hardneg(a.data_ptr(), p.data_ptr(), b, d, int(anchor_swap),
                                       pos.data_ptr(), mn.data_ptr(), ws.data_ptr(), ws.numel(),
                                       stream), "hn_pairdist_hardneg")
    return pos, mn


def pairdist_rows(anchor_rows: torch.Tensor, row0: int, positive: torch.Tensor, col_min: bool = False):
    """Rows [row0, row0 + n) of loss_HardNet's masked distance matrix (hardnet/Losses.py:95-108)
    between this rank's anchors and all positives: (pos, row_min, col_min or None); col_min[j]
    is the masked minimum of column j over these rows only (all-reduce it with MIN)."""
    lib = load_library()
    a = anchor_rows.contiguous().float()
    p = positive.contiguous().float()
    if a.dim() != 2 or p.dim() != 2 or a.shape[1] != p.shape[1] or a.device != p.device:
        raise ValueError("expected [n,D] anchors and [B,D] positives on one device")
    n, d = a.shape
    b = p.shape[0]
    sz = ctypes.c_size_t()
    _check(lib.hn_pairdist_rows_workspace_bytes(n, b, ctypes.byref(sz)), "hn_pairdist_rows_workspace_bytes")
    ws = torch.empty(max(sz.value, 16), device=a.device, dtype=torch.uint8)
    pos = torch.empty(n, device=a.device, dtype=torch.float32)
    rmin = torch.empty(n, device=a.device, dtype=torch.float32)
    cmin = torch.empty(b, device=a.device, dtype=torch.float32) if col_min else None
    stream = torch.cuda.current_stream(a.device).cuda_stream
    with torch.cuda.device(a.device):
        _check(lib.hn_pairdist_rows(a.data_ptr(), n, int(row0), p.data_ptr(), b, d, pos.data_ptr(),
                                    rmin.data_ptr(), cmin.data_ptr() if cmin is not None else None,
                                    ws.data_ptr(), ws.numel(), stream), "hn_pairdist_rows")
    return pos, rmin, cmin


LOSS_TYPES = {"triplet_margin": 0, "softmax": 1, "contrastive": 2}  # enum hn_loss_type


class HardNetLossFunction(torch.autograd.Function):
    """loss_HardNet with batch_reduce 'min' (hardnet/Losses.py:87-154) and its backward on the fused
    kernels of hn_loss.hip: no B x B matrix, the gradient routed to each row's positive and its
    selected hardest negative as autograd routes it through the reference formulation
    (HardNet.py:408-423).  anchor / positive: [B,128] fp32 HIP tensors."""

    @staticmethod
    def forward(ctx, anchor, positive, anchor_swap, margin, loss_type):
        lib = load_library()
        # the C ABI takes 16-byte aligned rows: a contiguous view at an odd storage offset is copied
        a, p = (x if x.data_ptr() % 16 == 0 else x.clone() for x in
                (anchor.detach().contiguous(), positive.detach().contiguous()))
        b = a.shape[0]
        n = ctypes.c_size_t()
        _check(lib.hn_hardnet_loss_train_workspace_bytes(b, ctypes.byref(n)), "hn_hardnet_loss_train_workspace_bytes")
        saved = torch.empty(n.value, device=a.device, dtype=torch.uint8)
        loss = torch.empty((), device=a.device, dtype=torch.float32)
        stream = torch.cuda.current_stream(a.device).cuda_stream
        with torch.cuda.device(a.device):
            _check(lib.hn_hardnet_loss_train_forward(a.data_ptr(), p.data_ptr(), b, a.shape[1], int(bool(anchor_swap)),
                                                     float(margin), LOSS_TYPES[loss_type], loss.data_ptr(),
                                                     saved.data_ptr(), saved.numel(), stream),
                   "hn_hardnet_loss_train_forward")
        ctx.args = (bool(anchor_swap), float(margin), LOSS_TYPES[loss_type])
        ctx.save_for_backward(a, p, saved)
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable  # the fused backward records no graph (no double backward)
    def backward(ctx, dloss):
        lib = load_library()
        a, p, saved = ctx.saved_tensors
        swap, margin, lt = ctx.args
        ga, gp = torch.empty_like(a), torch.empty_like(p)
        dl = dloss.detach().to(device=a.device, dtype=torch.float32).contiguous().reshape(1)
        stream = torch.cuda.current_stream(a.device).cuda_stream
        with torch.cuda.device(a.device):
            _check(lib.hn_hardnet_loss_backward(a.data_ptr(), p.data_ptr(), a.shape[0], a.shape[1], int(swap), margin,
                                                lt, dl.data_ptr(), ga.data_ptr(), gp.data_ptr(), saved.data_ptr(),
                                                saved.numel(), stream), "hn_hardnet_loss_backward")
        return ga, gp, None, None, None


def hardnet_loss(pos: torch.Tensor, row_min: torch.Tensor, col_min: Optional[torch.Tensor] = None,
                 margin: float = 1.0, loss_type: str = "triplet_margin", scale: Optional[float] = None):
    """scale * sum of loss_HardNet's per-row margin loss (Losses.py:142-153; scale defaults to
    1/n = torch.mean) with min_neg = min(row_min, col_min): (loss [1], min_neg [n])."""
    lib = load_library()
    if loss_type not in LOSS_TYPES:
        raise ValueError(f"loss_type must be one of {sorted(LOSS_TYPES)}")
    n = pos.shape[0]
    ps, rm = pos.contiguous().float(), row_min.contiguous().float()
    cm = col_min.contiguous().float() if col_min is not None else None
    mn = torch.empty(n, device=ps.device, dtype=torch.float32)
    loss = torch.empty(1, device=ps.device, dtype=torch.float32)
    stream = torch.cuda.current_stream(ps.device).cuda_stream
    with torch.cuda.device(ps.device):
        _check(lib.hn_hardnet_loss(ps.data_ptr(), rm.data_ptr(), cm.data_ptr() if cm is not None else None,
                                   n, float(margin), LOSS_TYPES[loss_type],
                                   float(1.0 / n if scale is None else scale), mn.data_ptr(),
                                   loss.data_ptr(), stream), "hn_hardnet_loss")
    return loss, mn


def fpr95(out_a: torch.Tensor, out_p: torch.Tensor, labels: torch.Tensor):
    """(fpr95, pair distances) on device: the eval loop of hardnet/HardNet.py:450-472
    (``sqrt(sum((a-p)^2))`` per pair) + ``ErrorRateAt95Recall`` (EvalMetrics.py:6-19)."""
    lib = load_library()
    if out_a.shape != out_p.shape or out_a.dim() != 2 or labels.numel() != out_a.shape[0]:
        raise ValueError("expected [n,D] descriptors and [n] labels")
    a = out_a.contiguous().float()
    p = out_p.contiguous().float()
    lab = labels.to(device=a.device, dtype=torch.int32).contiguous()
    n, d = a.shape
    sz = ctypes.c_size_t()
    _check(lib.hn_fpr95_workspace_bytes(n, ctypes.byref(sz)), "hn_fpr95_workspace_bytes")
    ws = torch.empty(max(sz.value, 16), device=a.device, dtype=torch.uint8)
    dists = torch.empty(n, device=a.device, dtype=torch.float32)
    res = torch.empty(1, device=a.device, dtype=torch.float64)
    stream = torch.cuda.current_stream(a.device).cuda_stream
    with torch.cuda.device(a.device):
        _check(lib.hn_fpr95(a.data_ptr(), p.data_ptr(), lab.data_ptr(), n, d, dists.data_ptr(),
                            res.data_ptr(), ws.data_ptr(), ws.numel(), stream), "hn_fpr95")
    return float(res.item()), dists


RESIZE_MODES = {"none": 0, "cv2": 1, "pil": 2}  # enum hn_resize


def preprocess(u8: torch.Tensor, resize: str = "cv2", normalize: bool = True,
               mean: float = 0.443728476019, std: float = 0.20197947209,
               out: torch.Tensor = None) -> torch.Tensor:
    """uint8 patches [n,64,64] (or [n,1,64,64] / [n,64,64,1]; [n,32,32] for resize='none')
    -> fp32 [n,1,32,32] on device, bit-exact with the reference loaders:
    resize='cv2' + normalize = ``transform`` (hardnet/HardNet.py:345-349, cv2_scale Utils.py:10-11);
    resize='pil', normalize=False = augmented ``transform_test`` (HardNet.py:333-337).
    Defaults for mean/std are the reference's --mean-image/--std-image (HardNet.py:86-89)."""
    lib = load_library()
    if resize not in RESIZE_MODES:
        raise ValueError(f"resize must be one of {sorted(RESIZE_MODES)}")
    if u8.dtype != torch.uint8 or not u8.is_cuda:
        raise ValueError("expected a uint8 HIP tensor")
    hw = 32 if resize == "none" else 64
    n = u8.shape[0]
    if u8.numel() != n * hw * hw:
        raise ValueError(f"expected {hw}x{hw} patches, got shape {tuple(u8.shape)}")
    x = u8.contiguous()
    if out is None:
        out = torch.empty((n, 1, 32, 32), device=x.device, dtype=torch.float32)
    elif out.shape != (n, 1, 32, 32) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("out must be a contiguous fp32 [n,1,32,32] tensor")
    stream = torch.cuda.current_stream(x.device).cuda_stream
    with torch.cuda.device(x.device):
        _check(lib.hn_preprocess(x.data_ptr(), n, hw, RESIZE_MODES[resize], int(normalize),
                                 mean, std, out.data_ptr(), stream), "hn_preprocess")
    return out


# ----------------------------------------------------------------------------------
# torch.library registration: hardnet_mi355x::forward(Tensor x, int handle) -> Tensor
# ----------------------------------------------------------------------------------
@torch.library.custom_op("hardnet_mi355x::forward", mutates_args=(), device_types="cuda")
def forward_op(x: torch.Tensor, handle: int) -> torch.Tensor:
    """Eval-mode descriptor forward of the NativeModel whose ``op_id`` is ``handle`` (the
    drop-in for HardNet.forward, hardnet/HardNet.py:312-315, under torch.no_grad -- :454).
    Registered as a custom op with a fake (meta) kernel so that torch.compile traces through
    the module's forward; there is no CPU kernel (the CPU path is the module's torch layers)."""
    nm = _BY_ID.get(int(handle))
    if nm is None:
        raise RuntimeError(f"hardnet_mi355x::forward: no live native model with handle {handle}")
    return nm.forward(x)


@forward_op.register_fake
def _forward_fake(x, handle):
    if x.dim() != 4 or tuple(x.shape[1:]) != (1, 32, 32):
        raise ValueError(f"expected [B,1,32,32], got {tuple(x.shape)}")
    return x.new_empty((x.shape[0], 128))


# ----------------------------------------------------------------------------------
# train-mode stock HardNet (hn_hardnet_train_*): an autograd.Function over the C ABI
# ----------------------------------------------------------------------------------
HARDNET_CONV_IDX = (0, 3, 6, 9, 12, 15, 19)   # features.{i}.weight (HardNet.py:280-301)
HARDNET_BN_IDX = (1, 4, 7, 10, 13, 16, 20)


def _ptr_array(ts):
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def train_workspace_bytes(batch: int):
    """(saved, scratch) bytes of hn_hardnet_train_forward / _backward for a batch."""
    lib = load_library()
    sv, sc = ctypes.c_size_t(), ctypes.c_size_t()
    _check(lib.hn_hardnet_train_workspace_bytes(batch, ctypes.byref(sv), ctypes.byref(sc)),
           "hn_hardnet_train_workspace_bytes")
    return sv.value, sc.value


class HardNetTrainFunction(torch.autograd.Function):
    """model.train() forward of the stock HardNet on the GPU kernels (BatchNorm batch
    statistics + running-statistics update, Dropout, L2Norm) and its backward to the 7 conv
    weights and the input -- what autograd does over the reference module in the training loop
    (hardnet/HardNet.py:379-441).  ``bn`` is a list of the 7 BatchNorm2d modules (their running
    buffers are updated in place, num_batches_tracked incremented).

    Each call keeps its own "saved" workspace (the BN outputs the backward reads) as a tensor
    saved for backward, so the loop's two forwards (anchors, positives; HardNet.py:392-393) each
    hold theirs until ``loss.backward()``, autograd frees it after the backward (or keeps it for
    ``retain_graph=True``: the backward only reads it), and a second backward without
    ``retain_graph`` raises torch's usual error.  The scratch workspace is transient."""

    @staticmethod
    def forward(ctx, x, drop_p, seed, bn, *weights):
        lib = load_library()
        b = x.shape[0]
        n_sv, n_sc = train_workspace_bytes(b)
        saved = torch.empty(n_sv, device=x.device, dtype=torch.uint8)
        scratch = torch.empty(n_sc, device=x.device, dtype=torch.uint8)
        out = torch.empty((b, 128), device=x.device, dtype=torch.float32)
        ws_w = [w.detach().contiguous() for w in weights]
        rm = [m.running_mean for m in bn]
        rv = [m.running_var for m in bn]
        stream = torch.cuda.current_stream(x.device).cuda_stream
        with torch.cuda.device(x.device):
            _check(lib.hn_hardnet_train_forward(x.data_ptr(), b, _ptr_array(ws_w), _ptr_array(rm), _ptr_array(rv),
                                                float(bn[0].momentum), float(drop_p), int(seed), out.data_ptr(),
                                                saved.data_ptr(), saved.numel(), scratch.data_ptr(), scratch.numel(),
                                                stream), "hn_hardnet_train_forward")
        del scratch
        torch._foreach_add_([m.num_batches_tracked for m in bn], 1)  # one launch for the 7 counters
        ctx.drop_p, ctx.seed, ctx.b = float(drop_p), int(seed), b
        ctx.save_for_backward(saved, *ws_w)
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = load_library()
        saved, *ws_w = ctx.saved_tensors
        dws = [torch.empty_like(w) for w in ws_w]
        need_x = ctx.needs_input_grad[0]
        din = torch.empty((ctx.b, 1, 32, 32), device=dout.device, dtype=torch.float32) if need_x else None
        _, n_sc = train_workspace_bytes(ctx.b)
        scratch = torch.empty(n_sc, device=dout.device, dtype=torch.uint8)
        stream = torch.cuda.current_stream(dout.device).cuda_stream
        with torch.cuda.device(dout.device):
            _check(lib.hn_hardnet_train_backward(dout.contiguous().data_ptr(), ctx.b, _ptr_array(ws_w),
                                                 _ptr_array(dws), din.data_ptr() if din is not None else None,
                                                 ctx.drop_p, ctx.seed, saved.data_ptr(), saved.numel(),
                                                 scratch.data_ptr(), scratch.numel(), stream),
                   "hn_hardnet_train_backward")
        return (din, None, None, None, *dws)


# ----------------------------------------------------------------------------------
# train-mode hardnetNAS (hn_nas_train_*): the sampled descriptor and the supernet
# ----------------------------------------------------------------------------------
def supernet_desc(layers=None) -> HnArchDesc:
    """HN_KIND_NAS_SUPERNET: every layer a MixedOperation over all 17 CANDIDATE_BLOCKS
    (model_supernet.py:10-36, 53-68)."""
    layers = layers or A.SEARCH_SPACE2
    d = nas_desc(["skip"] * len(layers), layers)
    d.kind = HN_KIND_NAS_SUPERNET
    return d


def train_tensors(module):
    """The float state_dict tensors the train ABI walks, in order (num_batches_tracked and the
    supernet's thetas left out), as (names, tensors)."""
    names, ts = [], []
    for k, v in module.state_dict(keep_vars=True).items():
        if k.endswith("num_batches_tracked") or k.endswith(".thetas"):
            continue
        names.append(k)
        ts.append(v)
    return names, ts


class NasTrainFunction(torch.autograd.Function):
    """model.train() forward of a hardnetNAS descriptor (``desc`` kind NAS) or of the supernet
    (kind NAS_SUPERNET, with the per-layer soft weights ``soft`` [n_layers, 17]) on the GPU
    kernels, and its backward to every parameter (and to ``soft``) -- what autograd does over the
    reference modules in hardnetNAS/supernet_functions/training_functions_supernet.py:88-103.
    ``tensors`` is the module's float state_dict in order (train_tensors); ``params`` are the ones
    among them that are parameters, in the same order; running buffers are updated in place."""

    @staticmethod
    def forward(ctx, x, soft, desc, tensors, momentum, *params):
        lib = load_library()
        b = x.shape[0]
        nt = ctypes.c_size_t()
        _check(lib.hn_nas_train_tensor_count(ctypes.byref(desc), ctypes.byref(nt)), "hn_nas_train_tensor_count")
        if len(tensors) != nt.value:
            raise ValueError(f"the module has {len(tensors)} float state_dict tensors, the descriptor walks {nt.value}")
        if soft is not None:
            n_layers = int(desc.n_layers)
            if tuple(soft.shape) != (n_layers, 17) or soft.device != x.device or soft.dtype != torch.float32:
                raise ValueError(f"soft must be fp32 [{n_layers}, 17] on {x.device}, got {soft.dtype} "
                                 f"{tuple(soft.shape)} on {soft.device}")
        sv, sc = ctypes.c_size_t(), ctypes.c_size_t()
        _check(lib.hn_nas_train_workspace_bytes(ctypes.byref(desc), b, ctypes.byref(sv), ctypes.byref(sc)),
               "hn_nas_train_workspace_bytes")
        saved = torch.empty(sv.value, device=x.device, dtype=torch.uint8)
        scratch = torch.empty(sc.value, device=x.device, dtype=torch.uint8)
        out = torch.empty((b, 128), device=x.device, dtype=torch.float32)
        soft_c = soft.detach().contiguous() if soft is not None else None
        stream = torch.cuda.current_stream(x.device).cuda_stream
        with torch.cuda.device(x.device):
            _check(lib.hn_nas_train_forward(ctypes.byref(desc), x.data_ptr(), b, _ptr_array(tensors), float(momentum),
                                            soft_c.data_ptr() if soft_c is not None else None, out.data_ptr(),
                                            saved.data_ptr(), saved.numel(), scratch.data_ptr(), scratch.numel(),
                                            stream), "hn_nas_train_forward")
        del scratch
        ctx.desc, ctx.tensors, ctx.b = desc, tensors, b
        # per slot: 1 = a parameter whose gradient is returned, 2 = a frozen parameter (the kernels still
        # write its gradient: it gets a throwaway buffer), 0 = a buffer (running statistics)
        ctx.slot = [1 if t.requires_grad else 2 if isinstance(t, torch.nn.Parameter) else 0 for t in tensors]
        ctx.has_soft = soft is not None
        ctx.save_for_backward(saved, x, soft_c if soft_c is not None else x.new_empty(0), *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = load_library()
        saved, x, soft_c, *params = ctx.saved_tensors
        # one allocation for every parameter's gradient (the supernet has ~2,000), handed out as views
        # (contiguous, the parameters' shapes: autograd stores them as .grad without a copy)
        flat = torch.empty(sum(p.numel() for p in params), device=dout.device, dtype=torch.float32)
        grads = [g.view(p.shape) for g, p in zip(flat.split([p.numel() for p in params]), params)]
        it = iter(grads)
        gptrs = [next(it) if k == 1 else torch.empty_like(t) if k == 2 else None
                 for k, t in zip(ctx.slot, ctx.tensors)]
        sv, sc = ctypes.c_size_t(), ctypes.c_size_t()
        _check(lib.hn_nas_train_workspace_bytes(ctypes.byref(ctx.desc), ctx.b, ctypes.byref(sv), ctypes.byref(sc)),
               "hn_nas_train_workspace_bytes")
        scratch = torch.empty(sc.value, device=dout.device, dtype=torch.uint8)
        dsoft = torch.empty_like(soft_c) if ctx.has_soft else None
        stream = torch.cuda.current_stream(dout.device).cuda_stream
        gp = (ctypes.c_void_p * len(gptrs))(*[g.data_ptr() if g is not None else None for g in gptrs])
        with torch.cuda.device(dout.device):
            _check(lib.hn_nas_train_backward(ctypes.byref(ctx.desc), dout.contiguous().data_ptr(), x.data_ptr(), ctx.b,
                                             _ptr_array(ctx.tensors),
                                             soft_c.data_ptr() if ctx.has_soft else None, gp,
                                             dsoft.data_ptr() if dsoft is not None else None, saved.data_ptr(),
                                             saved.numel(), scratch.data_ptr(), scratch.numel(), stream),
                   "hn_nas_train_backward")
        return (None, dsoft, None, None, None, *grads)
