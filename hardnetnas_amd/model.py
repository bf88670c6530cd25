"""Drop-in descriptor modules: ``HardNet`` and ``HardNetNAS``.

Both keep the reference's ``nn.Module`` surface and state_dict layout so that the
reference training / FPR95 loops and checkpoints work unchanged:

* ``HardNet`` mirrors hardnet/HardNet.py:275-315 -- ``.features`` is an
  ``nn.Sequential`` with the same 21 indices, ``.input_norm(x)`` and
  ``.forward(x) -> [B,128]`` (L2-normalised, hardnet/Utils.py:15-22).
* ``HardNetNAS(arch)`` is the sampled hardnetNAS descriptor: the supernet skeleton
  (hardnetNAS/supernet_functions/model_supernet.py:53-85) with every MixedOperation
  replaced by its arch op (fbnet_modeldef.py:30-95).  Sub-module names follow
  ``ConvBNRelu`` / ``IRFBlock`` / ``Identity`` (fbnet_building_blocks/fbnet_builder.py)
  so the keys of a supernet checkpoint map 1:1 (``load_supernet_state_dict``).

Eval-mode forward on a HIP tensor (fp32 ``[B,1,32,32]``) with no autograd graph to record
(under ``torch.no_grad()`` as in the reference eval loop, hardnet/HardNet.py:454, or with
parameters frozen) runs the hand-written gfx950 kernels through the registered op
``torch.ops.hardnet_mi355x.forward`` (C ABI, ``hardnetnas_amd._native``).  There is no silent
fallback for that case: if the native library is missing the call raises.  Train mode
(BatchNorm batch statistics, Dropout), autograd-recording calls and CPU tensors run the
module's own PyTorch layers, exactly like the reference module would; ``strict=True`` turns
an eval-mode HIP call that cannot take the native path into an error.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import arch as A


class L2Norm(nn.Module):
    """hardnet/Utils.py:15-22: x / sqrt(sum(x^2) + 1e-10)."""

    def __init__(self):
        super().__init__()
        self.eps = 1e-10

    def forward(self, x):
        norm = torch.sqrt(torch.sum(x * x, dim=1) + self.eps)
        return x / norm.unsqueeze(-1).expand_as(x)


class Flatten(nn.Module):
    """fbnet_builder.py:194-199."""

    def forward(self, x):
        return x.reshape(x.size(0), -1)


def _native_blocker(module: nn.Module, x: torch.Tensor):
    """None if this call can run on the HIP kernels, else why not.  The native forward is an
    inference kernel: it builds no autograd graph, so whenever the reference module would
    record one (grad mode on and the input or any parameter requiring grad -- e.g. an eval-mode
    fine-tune, or input gradients; hardnet/HardNet.py:392-423) the module's own layers run."""
    if module.training:
        return "module is in train mode"
    if not x.is_cuda:
        return "input is not a HIP tensor"
    if x.dtype != torch.float32 or x.dim() != 4 or tuple(x.shape[1:]) != (1, 32, 32):
        return f"input must be fp32 [B,1,32,32], got {x.dtype} {tuple(x.shape)}"
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in module.parameters())):
        return "autograd is recording (grad mode on and the input or a parameter requires grad)"
    return None


def _native_eligible(module: nn.Module, x: torch.Tensor) -> bool:
    return _native_blocker(module, x) is None


class _NativeMixin:
    """Owns the packed device model; re-packs when parameters/buffers change.

    ``native_strict`` (constructor keyword ``strict``): an eval-mode call on a HIP tensor that
    cannot take the native path raises instead of running the torch layers."""

    native_strict = False

    def _native_key(self):
        ts = list(self.parameters()) + list(self.buffers())
        return tuple((t.data_ptr(), t._version) for t in ts)

    @torch.compiler.disable
    def _native_handle(self, x: torch.Tensor) -> int:
        from . import _native
        key = (x.device.index, getattr(self, "input_norm_eps", None), getattr(self, "l2_eps", None),
               self._native_key())
        h = getattr(self, "_hn_handle", None)
        if h is None or self._hn_key != key:
            self._hn_handle = None  # release the old one first
            self._hn_handle = _native.NativeModel.from_module(self, x.device)
            self._hn_key = key
        return self._hn_handle.op_id

    def _native_forward(self, x: torch.Tensor) -> torch.Tensor:
        from . import _native  # noqa: F401  (registers torch.ops.hardnet_mi355x)
        return torch.ops.hardnet_mi355x.forward(x, self._native_handle(x))

    def _dispatch_native(self, x: torch.Tensor):
        """The native descriptor if this call takes the HIP path, else None (torch layers)."""
        why = _native_blocker(self, x)
        if why is None:
            return self._native_forward(x)
        if self.native_strict and not self.training and x.is_cuda:
            raise RuntimeError(f"{type(self).__name__}(strict=True): native forward not taken: {why}")
        return None

    def __getstate__(self):
        d = dict(self.__dict__)
        d.pop("_hn_handle", None)
        d.pop("_hn_key", None)
        return d


def _dropout_seed(device: torch.device) -> int:
    """A 64-bit dropout seed drawn from the CUDA generator of ``device`` -- where the reference's
    nn.Dropout draws its mask on a HIP tensor -- without a device synchronisation and without
    touching the CPU generator (so e.g. DataLoader shuffling sees the same CPU RNG stream as with
    the reference module).  ``torch.manual_seed`` / ``torch.cuda.manual_seed`` make it
    reproducible: the seed is a hash of the generator's seed and its Philox offset, which is then
    advanced as a kernel launch that consumed 4 values per thread would advance it."""
    g = torch.cuda.default_generators[device.index if device.index is not None else torch.cuda.current_device()]
    off = g.get_offset()
    g.set_offset(off + 4)
    z = (g.initial_seed() * 0x9E3779B97F4A7C15 + off + 1) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return (z ^ (z >> 31)) & 0x3FFFFFFFFFFFFFFF


class HardNet(_NativeMixin, nn.Module):
    """HardNet model definition (hardnet/HardNet.py:275-315)."""

    def __init__(self, strict: bool = False):
        super().__init__()
        self.native_strict = strict
        self.features = nn.Sequential(
            nn.Conv2d(1, 32, kernel_size=3, padding=1, bias=False),
            nn.BatchNorm2d(32, affine=False),
            nn.ReLU(),
            nn.Conv2d(32, 32, kernel_size=3, padding=1, bias=False),
            nn.BatchNorm2d(32, affine=False),
            nn.ReLU(),
            nn.Conv2d(32, 64, kernel_size=3, stride=2, padding=1, bias=False),
            nn.BatchNorm2d(64, affine=False),
            nn.ReLU(),
            nn.Conv2d(64, 64, kernel_size=3, padding=1, bias=False),
            nn.BatchNorm2d(64, affine=False),
            nn.ReLU(),
            nn.Conv2d(64, 128, kernel_size=3, stride=2, padding=1, bias=False),
            nn.BatchNorm2d(128, affine=False),
            nn.ReLU(),
            nn.Conv2d(128, 128, kernel_size=3, padding=1, bias=False),
            nn.BatchNorm2d(128, affine=False),
            nn.ReLU(),
            nn.Dropout(0.3),
            nn.Conv2d(128, 128, kernel_size=8, bias=False),
            nn.BatchNorm2d(128, affine=False),
        )
        self.features.apply(weights_init)
        # epsilons of this variant (HardNet.py:308, Utils.py:18); FDLNet clones use 1e-8 / none
        self.input_norm_eps = 1e-7
        self.l2_eps = 1e-10

    def input_norm(self, x):
        """HardNet.py:306-310: per-patch (x - mean) / (unbiased std + eps)."""
        flat = x.view(x.size(0), -1)
        mp = torch.mean(flat, dim=1)
        sp = torch.std(flat, dim=1) + self.input_norm_eps
        return (x - mp.detach().view(-1, 1, 1, 1)) / sp.detach().view(-1, 1, 1, 1)

    def _train_native_eligible(self, x) -> bool:
        """model.train() on a HIP fp32 [B>=2,1,32,32] batch with the reference's BatchNorm setup
        (one momentum for all seven layers, running statistics tracked, eps 1e-5) and every conv
        weight and BN running buffer fp32 on x's device runs hn_hardnet_train_* (SURVEY 8(f) row 4).
        Anything else runs the module's torch layers, which raise the reference module's own
        dtype / device errors."""
        if not (getattr(self, "native_train", True) and self.training and x.is_cuda
                and x.dtype == torch.float32 and x.dim() == 4
                and tuple(x.shape[1:]) == (1, 32, 32) and x.shape[0] >= 2):
            return False
        bns = [self.features[i] for i in (1, 4, 7, 10, 13, 16, 20)]
        ts = [self.features[i].weight for i in (0, 3, 6, 9, 12, 15, 19)]
        ts += [t for b in bns for t in (b.running_mean, b.running_var)]
        return (self.input_norm_eps == 1e-7 and self.l2_eps == 1e-10
                and all(b.training and b.momentum is not None and b.track_running_stats and b.eps == 1e-5
                        and not b.affine and b.momentum == bns[0].momentum for b in bns)
                and all(t is not None and t.dtype == torch.float32 and t.device == x.device for t in ts))

    def _train_native_forward(self, x):
        from . import _native as N
        bns = [self.features[i] for i in N.HARDNET_BN_IDX]
        ws = [self.features[i].weight for i in N.HARDNET_CONV_IDX]
        drop = self.features[18]
        p = drop.p if drop.training else 0.0
        seed = _dropout_seed(x.device) if p > 0 else 0
        return N.HardNetTrainFunction.apply(x.contiguous(), p, seed, bns, *ws)

    def forward(self, input):
        y = self._dispatch_native(input)
        if y is not None:
            return y
        if self._train_native_eligible(input):
            return self._train_native_forward(input)
        x_features = self.features(self.input_norm(input))
        x = x_features.view(x_features.size(0), -1)
        norm = torch.sqrt(torch.sum(x * x, dim=1) + self.l2_eps)
        return x / norm.unsqueeze(-1)


def weights_init(m):
    """HardNet.py:317-324 (orthogonal, gain 0.6)."""
    if isinstance(m, nn.Conv2d):
        nn.init.orthogonal_(m.weight.data, gain=0.6)
        if m.bias is not None:
            nn.init.constant_(m.bias.data, 0.01)


# ----------------------------------------------------------------------------------
# hardnetNAS building blocks (fbnet_building_blocks/fbnet_builder.py)
# ----------------------------------------------------------------------------------

class ConvBNRelu(nn.Sequential):
    """fbnet_builder.py:352-404 with bn_type="bn" (affine BN, eps 1e-5)."""

    def __init__(self, c_in, c_out, kernel, stride, pad, relu=True, group=1):
        super().__init__()
        conv = nn.Conv2d(c_in, c_out, kernel_size=kernel, stride=stride, padding=pad,
                         bias=False, groups=group)
        nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
        self.add_module("conv", conv)
        self.add_module("bn", nn.BatchNorm2d(c_out))
        if relu:
            self.add_module("relu", nn.ReLU(inplace=True))


class ChannelShuffle(nn.Module):
    """fbnet_builder.py:332-349."""

    def __init__(self, groups):
        super().__init__()
        self.groups = groups

    def forward(self, x):
        n, c, h, w = x.size()
        g = self.groups
        return x.view(n, g, c // g, h, w).permute(0, 2, 1, 3, 4).contiguous().view(n, c, h, w)


class SEModule(nn.Module):
    """fbnet_builder.py:407-421."""

    def __init__(self, c):
        super().__init__()
        mid = A.se_mid(c)
        self.op = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(c, mid, 1, 1, 0),
                                nn.ReLU(inplace=True), nn.Conv2d(mid, c, 1, 1, 0), nn.Sigmoid())

    def forward(self, x):
        return x * self.op(x)


class IRFBlock(nn.Module):
    """fbnet_builder.py:455-570 (kernel 3/5, no cdw, no upsample)."""

    def __init__(self, c_in, c_out, expansion, stride, kernel=3, pw_group=1,
                 shuffle=False, se=False):
        super().__init__()
        self.use_res_connect = stride == 1 and c_in == c_out
        mid = A.ir_mid(c_in, expansion)
        self.pw = ConvBNRelu(c_in, mid, 1, 1, 0, relu=True, group=pw_group)
        self.dw = ConvBNRelu(mid, mid, kernel, stride, kernel // 2, relu=True, group=mid)
        self.pwl = ConvBNRelu(mid, c_out, 1, 1, 0, relu=False, group=pw_group)
        self.shuffle_type = "mid" if shuffle else None
        if shuffle:
            self.shuffle = ChannelShuffle(pw_group)
        self.se4 = SEModule(c_out) if se else nn.Sequential()

    def forward(self, x):
        y = self.pw(x)
        if self.shuffle_type == "mid":
            y = self.shuffle(y)
        y = self.dw(y)
        y = self.pwl(y)
        if self.use_res_connect:
            y = y + x
        return self.se4(y)


class Identity(nn.Module):
    """The "skip" candidate, fbnet_builder.py:202-228."""

    def __init__(self, c_in, c_out, stride):
        super().__init__()
        if c_in != c_out:
            if stride == 1:
                self.conv = ConvBNRelu(c_in, c_out, 1, 1, 0, relu=True)
            else:
                self.conv = nn.Sequential(nn.MaxPool2d(3, 2, 1), ConvBNRelu(c_in, c_out, 1, 1, 0))
        else:
            self.conv = None if stride == 1 else nn.Sequential(nn.MaxPool2d(3, 2, 1))

    def forward(self, x):
        return self.conv(x) if self.conv is not None else x


def make_op(name: str, c_in: int, c_out: int, stride: int) -> nn.Module:
    spec = A.OP_SPECS[name]
    if spec.kind == "skip":
        return Identity(c_in, c_out, stride)
    return IRFBlock(c_in, c_out, spec.expansion, stride, kernel=spec.kernel,
                    pw_group=spec.pw_group, shuffle=spec.shuffle, se=spec.se)


class FDLIdentity(nn.Module):
    """FDLNet's ``Identity`` (latency/NASNet/model/operations.py, class Identity): a 1x1
    ConvBNRelu with the block's stride when C or the resolution changes, else nothing
    (unlike fbnet_builder's, no max-pool)."""

    def __init__(self, c_in, c_out, stride):
        super().__init__()
        self.conv = (ConvBNRelu(c_in, c_out, 1, stride, 0, relu=True)
                     if c_in != c_out or stride != 1 else None)

    def forward(self, x):
        return self.conv(x) if self.conv is not None else x


class HardNetNeiMask(_NativeMixin, nn.Module):
    """FDLNet's hand-instantiated NAS descriptor ``HardNetNeiMask``:
    ``variant="NASNet"`` = FDLNet-master/latency/NASNet/model/des.py:8-55,
    ``variant="NASNet_0.1"`` = latency/NASNet_0.1/model/des.py:10-55.  Same ``.features``
    indices / state_dict keys as the reference; input_norm eps 1e-8 (des.py:40-47); L2 by
    ``torch.norm`` without eps (des.py:49-53).  The neighbour-mask training loss is not
    part of the descriptor forward and is not restated here."""

    def __init__(self, MARGIN: float = 1.0, C: float = 1.0, variant: str = "NASNet",
                 strict: bool = False):
        super().__init__()
        self.native_strict = strict
        if variant not in A.FDL_VARIANTS:
            raise ValueError(f"variant must be one of {A.FDL_VARIANTS}")
        self.MARGIN, self.C, self.variant = MARGIN, C, variant
        if variant == "NASNet":
            front = [nn.Conv2d(1, 32, kernel_size=3, stride=1, padding=1),
                     nn.BatchNorm2d(32, affine=False),
                     nn.Conv2d(32, 32, kernel_size=1, stride=2, padding=0, bias=False),
                     nn.BatchNorm2d(32), nn.ReLU(inplace=True),
                     nn.Conv2d(32, 64, kernel_size=1, stride=2, padding=0, bias=False),
                     nn.BatchNorm2d(64), nn.ReLU(inplace=True)]
        else:
            front = [nn.Conv2d(1, 32, kernel_size=3, stride=1, padding=1),
                     nn.MaxPool2d(kernel_size=3, stride=2, padding=1),
                     FDLIdentity(32, 32, 1), FDLIdentity(32, 64, 2)]
        blocks = [make_op(op, ci, co, s) for op, (ci, co, s) in zip(A.FDL_OPS, A.FDL_LAYERS)]
        head = [nn.Conv2d(128, 128, kernel_size=4, bias=False), nn.BatchNorm2d(128, affine=False)]
        self.features = nn.Sequential(*front, *blocks, *head)
        self.input_norm_eps = A.FDL_INPUT_NORM_EPS

    def input_norm(self, x):
        flat = x.view(x.size(0), -1)
        mp = torch.mean(flat, dim=1)
        sp = torch.std(flat, dim=1) + self.input_norm_eps
        return (x - mp.detach().view(-1, 1, 1, 1)) / sp.detach().view(-1, 1, 1, 1)

    def forward(self, input):
        y = self._dispatch_native(input)
        if y is not None:
            return y
        walk = _nas_train_native_eligible(self, input, A.FDL_LAYERS, A.FDL_LAYERS)
        if walk is not None:
            return _nas_train_native_forward(self, input, None, walk)
        x_features = self.features(self.input_norm(input))
        x = x_features.view(x_features.size(0), -1)
        return x / torch.norm(x, p=2, dim=-1, keepdim=True)


class HardNetNAS(_NativeMixin, nn.Module):
    """Sampled hardnetNAS descriptor (model_supernet.py:53-85, argmax op per layer).

    ``arch`` is a MODEL_ARCH name ('wang2', 'wang3', 'wang4') or a list of six
    CANDIDATE_BLOCKS op names.  There is no input_norm: the NAS loaders normalise
    globally (general_functions/dataloader.py:118-122).  The final normalisation is
    ``y / torch.norm(y)`` with no epsilon (model_supernet.py:84).
    """

    def __init__(self, arch="wang2", layers: Sequence = None, strict: bool = False):
        super().__init__()
        self.native_strict = strict
        self.arch_ops: List[str] = A.arch_ops(arch)
        self.layers = list(layers) if layers is not None else list(A.SEARCH_SPACE2)
        self.first = ConvBNRelu(1, A.STEM_CHANNELS, 3, 1, 1, relu=True)
        self.stages = nn.ModuleList([make_op(op, ci, co, s)
                                     for op, (ci, co, s) in zip(self.arch_ops, self.layers)])
        self.last_stages = nn.Sequential(OrderedDict([
            ("conv_k1", nn.Conv2d(self.layers[-1][1], A.DESC_DIM, kernel_size=A.HEAD_KERNEL,
                                  bias=False)),
            ("batchnorm", nn.BatchNorm2d(A.DESC_DIM, affine=False)),
            ("flatten", Flatten()),
        ]))

    def forward(self, x):
        y = self._dispatch_native(x)
        if y is not None:
            return y
        walk = _nas_train_native_eligible(self, x, self.layers)
        if walk is not None:
            return _nas_train_native_forward(self, x, None, walk)
        y = self.first(x)
        for op in self.stages:
            y = op(y)
        y = self.last_stages(y)
        return y / torch.norm(y, p=2, dim=-1, keepdim=True)

    def load_supernet_state_dict(self, sd, strict: bool = True):
        """Load a FBNet_Stochastic_SuperNet checkpoint (optionally DataParallel
        ``module.``-prefixed, general_functions/utils.py:94-98): keys
        ``stages_to_search.{i}.ops.{j}.*`` with j = CANDIDATE_BLOCKS.index(op_i)
        become ``stages.{i}.*``; ``thetas`` and the other ops are dropped."""
        out = OrderedDict()
        want = {i: A.CANDIDATE_BLOCKS.index(op) for i, op in enumerate(self.arch_ops)}
        for k, v in sd.items():
            if k.startswith("module."):
                k = k[len("module."):]
            if k.startswith("stages_to_search."):
                parts = k.split(".")
                i = int(parts[1])
                if parts[2] != "ops" or int(parts[3]) != want[i]:
                    continue
                out[".".join(["stages", str(i)] + parts[4:])] = v
            elif k.startswith("first.") or k.startswith("last_stages."):
                out[k] = v
        return self.load_state_dict(out, strict=strict)


def _nas_train_native_eligible(module: nn.Module, x: torch.Tensor, layers, expect=A.SEARCH_SPACE2):
    """model.train() of HardNetNAS / HardNetNASSupernet / HardNetNeiMask on a HIP fp32
    [B>=2,1,32,32] batch that needs no input gradient, with the reference's BatchNorm setup (one
    momentum, running statistics tracked, eps 1e-5) and every parameter / buffer fp32 contiguous on
    x's device, runs hn_nas_train_* (SURVEY 8(f) row 4).  Anything else runs the module's torch
    layers (returns None).  Eligible: returns (bns, tensors) -- the BatchNorms, and the float state_dict
    tensors in state_dict order without num_batches_tracked and the supernet's thetas (the train
    ABI's tensor list, _native.train_tensors) -- gathered in the same single pass over the module tree
    that checks them (the supernet has ~1,400 modules: one walk instead of five per forward)."""
    if not (getattr(module, "native_train", True) and module.training and x.is_cuda
            and x.dtype == torch.float32 and x.dim() == 4 and tuple(x.shape[1:]) == (1, 32, 32)
            and x.shape[0] >= 2 and not (torch.is_grad_enabled() and x.requires_grad)
            and list(layers) == list(expect)):
        return None
    return _nas_train_walk(module, x.device)


def _nas_train_walk(module: nn.Module, dev: torch.device):
    """The single pass of _nas_train_native_eligible: None unless every parameter / float buffer is fp32
    contiguous on `dev` and every BatchNorm has the kernels' form (affine=False for the head's BN and
    FDLNet NASNet's BN after conv0, affine for every other; train mode, running statistics, one momentum,
    eps 1e-5); else (bns, tensors) with tensors in _native.train_tensors' order."""
    plain = {id(b) for b in _non_affine_bns(module)}
    bns, tensors = [], []
    for mod in module.modules():  # the DFS pre-order state_dict walks
        for name, t in mod._parameters.items():
            if t is None:
                continue
            if not (t.dtype == torch.float32 and t.device == dev and t.is_contiguous()):
                return None
            if name != "thetas":
                tensors.append(t)
        for name, t in mod._buffers.items():
            if t is None or t.dtype == torch.int64:
                continue
            if not (t.dtype == torch.float32 and t.device == dev and t.is_contiguous()):
                return None
            if name not in mod._non_persistent_buffers_set:
                tensors.append(t)
        if isinstance(mod, nn.BatchNorm2d):
            if not (mod.training and mod.momentum is not None and mod.track_running_stats and mod.eps == 1e-5
                    and (not bns or mod.momentum == bns[0].momentum) and mod.affine == (id(mod) not in plain)):
                return None
            bns.append(mod)
    return bns, tensors


def _non_affine_bns(module: nn.Module):
    if isinstance(module, HardNetNeiMask):
        f = module.features
        return [f[1], f[-1]] if module.variant == "NASNet" else [f[-1]]
    return [module.last_stages.batchnorm]


def _nas_train_native_forward(module: nn.Module, x: torch.Tensor, soft, walk):
    from . import _native as N
    bns, tensors = walk
    desc = N.supernet_desc() if soft is not None else N.desc_for_module(module)
    params = [t for t in tensors if t.requires_grad]
    y = N.NasTrainFunction.apply(x.contiguous(), soft, desc, tensors, bns[0].momentum, *params)
    # one multi-tensor launch for every BatchNorm's counter (the supernet has 584)
    torch._foreach_add_([b.num_batches_tracked for b in bns], 1)
    return y


class MixedOperation(nn.Module):
    """One searchable layer of the supernet (hardnetNAS/supernet_functions/model_supernet.py:10-50):
    all 17 CANDIDATE_BLOCKS on the same input, output sum_j m_j op_j(x) with m the Gumbel-softmax of
    ``thetas`` (initialised to 1/17), plus the latency bookkeeping of the reference."""

    def __init__(self, c_in, c_out, stride, latency=None):
        super().__init__()
        self.ops = nn.ModuleList([make_op(op, c_in, c_out, stride) for op in A.CANDIDATE_BLOCKS])
        self.latency = list(latency) if latency is not None else [1.0] * len(A.CANDIDATE_BLOCKS)
        self.thetas = nn.Parameter(torch.Tensor([1.0 / len(A.CANDIDATE_BLOCKS)] * len(A.CANDIDATE_BLOCKS)))

    def softnms(self, variables, ksize, strength):
        """model_supernet.py:38-50 (1-D soft NMS over the op probabilities)."""
        maxk = F.max_pool1d(variables, ksize, stride=1, padding=ksize // 2)
        max_all, _ = maxk.max(dim=-1, keepdim=True)
        exp_maps = torch.exp(strength * (variables - max_all))
        exp_maps_pad = F.pad(exp_maps, [ksize // 2, ksize // 2], mode="replicate")
        sum_exp = F.conv1d(exp_maps_pad, weight=self._const("ones", [1.0] * ksize, exp_maps).view(1, 1, ksize),
                           stride=1)
        return exp_maps / sum_exp

    def _const(self, name, values, like):
        """values as a tensor on like's device / dtype, kept between calls (no host copy per step)."""
        cache = self.__dict__.setdefault("_const_cache", {})
        key = (name, like.device, like.dtype, tuple(values))
        t = cache.get(key)
        if t is None:
            t = cache[key] = torch.tensor(values, device=like.device, dtype=like.dtype)
        return t

    def latency_terms(self, m, latency_to_accumulate, hard_idx=None):
        """model_supernet.py:27-35: the soft latency, its soft-NMS and hard-sample forms.  The two weighted
        sums are one product and one reduction each (the reference's Python sum over the 17 ops launches 34
        kernels per term; the fp32 sum order differs at the 1e-7 level).  hard_idx: argmax(m), when the
        caller already has it (HardNetNASSupernet reads all six layers' in one device sync)."""
        lat = self._const("latency", self.latency, m)
        latency = (m * lat).sum()
        nmsprobs = self.softnms(m.unsqueeze(0).unsqueeze(0), len(self.latency), 50)
        soft = (nmsprobs.squeeze() * lat).sum()
        hard = self.latency[torch.argmax(m).item() if hard_idx is None else hard_idx]
        return latency_to_accumulate + latency, soft, hard

    def forward(self, x, temperature, latency_to_accumulate, m=None):
        if m is None:
            m = F.gumbel_softmax(self.thetas, temperature)
        out = sum(mj * op(x) for mj, op in zip(m, self.ops))
        lat, soft, hard = self.latency_terms(m, latency_to_accumulate)
        return out, lat, soft, hard


class HardNetNASSupernet(nn.Module):
    """FBNet_Stochastic_SuperNet (hardnetNAS/supernet_functions/model_supernet.py:53-85) with the
    reference's module names (``first``, ``stages_to_search.{i}.ops.{j}`` / ``.thetas``,
    ``last_stages``), so its checkpoints load unchanged.  ``latency``: per layer, the 17 op
    latencies of the lookup table (default 1.0).

    ``forward(x, temperature, latency_to_accumulate, soft_weights=None)`` returns
    ``(y, latency_to_accumulate, soft, hard)`` like the reference.  ``soft_weights`` ([6, 17],
    may require grad) replaces the per-layer Gumbel-softmax draw of ``thetas`` -- a caller that
    wants thetas' gradient passes ``softmax((thetas + g) / tau)`` with its own Gumbel noise g.  In
    train() on a HIP batch the descriptor runs on hn_nas_train_* (every op of every layer, the
    weighted sum, train-mode BatchNorm, and the backward to every parameter and to the soft
    weights); otherwise the module's torch layers run."""

    def __init__(self, latency=None, layers: Sequence = None):
        super().__init__()
        self.layers = list(layers) if layers is not None else list(A.SEARCH_SPACE2)
        lat = latency if latency is not None else [None] * len(self.layers)
        self.first = ConvBNRelu(1, A.STEM_CHANNELS, 3, 1, 1, relu=True)
        self.stages_to_search = nn.ModuleList([MixedOperation(ci, co, s, lat[i])
                                               for i, (ci, co, s) in enumerate(self.layers)])
        self.last_stages = nn.Sequential(OrderedDict([
            ("conv_k1", nn.Conv2d(self.layers[-1][1], A.DESC_DIM, kernel_size=A.HEAD_KERNEL, bias=False)),
            ("batchnorm", nn.BatchNorm2d(A.DESC_DIM, affine=False)),
            ("flatten", Flatten()),
        ]))

    def forward(self, x, temperature, latency_to_accumulate, soft_weights=None):
        if soft_weights is None:
            soft_weights = torch.stack([F.gumbel_softmax(st.thetas, temperature) for st in self.stages_to_search])
        soft, hard = 0, 0
        hard_idx = torch.argmax(soft_weights, dim=1).tolist()  # (one device sync for the six layers)
        for i, st in enumerate(self.stages_to_search):
            latency_to_accumulate, s_i, h_i = st.latency_terms(soft_weights[i], latency_to_accumulate, hard_idx[i])
            soft, hard = soft + s_i, hard + h_i
        walk = _nas_train_native_eligible(self, x, self.layers)
        if walk is not None:
            y = _nas_train_native_forward(self, x, soft_weights.to(device=x.device, dtype=torch.float32), walk)
            return y, latency_to_accumulate, soft, hard
        y = self.first(x)
        for i, st in enumerate(self.stages_to_search):
            y = sum(mj * op(y) for mj, op in zip(soft_weights[i], st.ops))
        y = self.last_stages(y)
        return y / torch.norm(y, p=2, dim=-1, keepdim=True), latency_to_accumulate, soft, hard


FP16_SPLIT_LIMIT = 65504.0  # largest finite fp16: the hi half of an fp16x3 operand


@torch.no_grad()
def fp16_split_margin(module: nn.Module, x: torch.Tensor) -> dict:
    """Range check for the fp16x3 kernels of HardNetNAS / HardNetNeiMask.

    Those kernels split every operand of their 1x1 / grouped convs, stem and head into fp16
    hi + lo halves (csrc/hn_common.h ``split8_f16``), so an activation of magnitude >= 65520
    entering such a layer overflows the hi half.  ``hn_create`` rejects BN-folded *weights* out of
    that range; activations depend on the data, so this runs the module's own torch layers (a CPU
    copy, fp32) over a calibration batch ``x`` and reports the largest |input| reaching any
    non-depthwise conv.  ``margin = 65504 / peak`` must stay above 1 for the native forward to be
    valid on data like ``x``; the golden checkpoints sit at margins of order 10^3.  (Stock
    HardNet runs on bf16x3, whose range is fp32's: no limit applies.)

    Returns ``{"peak": float, "layer": str, "margin": float}``.
    """
    import copy
    m = copy.deepcopy(module).cpu().eval()
    peak = {"peak": 0.0, "layer": ""}
    hooks = []
    for name, mod in m.named_modules():
        if isinstance(mod, nn.Conv2d) and not (mod.groups == mod.in_channels and mod.in_channels > 1):
            def hook(_mod, inp, _out, name=name):
                v = float(inp[0].abs().max()) if inp[0].numel() else 0.0
                if v > peak["peak"]:
                    peak.update(peak=v, layer=name)
            hooks.append(mod.register_forward_hook(hook))
    try:
        m(x.detach().to("cpu", torch.float32))
    finally:
        for h in hooks:
            h.remove()
    peak["margin"] = FP16_SPLIT_LIMIT / peak["peak"] if peak["peak"] > 0 else float("inf")
    return peak
