"""Architecture registry for the NAS-searched descriptors.

Restates (does not import) the pieces of the reference that define the shape of a
sampled hardnetNAS descriptor:

* ``CANDIDATE_BLOCKS``  -- hardnetNAS/supernet_functions/lookup_table_builder.py:18-20
* ``SEARCH_SPACE2``     -- hardnetNAS/supernet_functions/lookup_table_builder.py:22-45,
  turned into per-layer ``(C_in, C_out, stride)`` exactly like
  ``LookUpTable._generate_layers_parameters`` (lookup_table_builder.py:96-110).
* ``MODEL_ARCH``        -- the op names of the searched archs wang2/3/4
  (hardnetNAS/fbnet_building_blocks/fbnet_modeldef.py:30-95).
* ``OP_SPECS``          -- the constructor arguments each candidate op passes to
  ``IRFBlock`` / ``Identity`` in ``PRIMITIVES``
  (hardnetNAS/fbnet_building_blocks/fbnet_builder.py:36-191).

The integer op ids used by the native library are the indices into
``CANDIDATE_BLOCKS`` -- the same index ``j`` as in the supernet state-dict key
``stages_to_search.{i}.ops.{j}`` (model_supernet.py:18-19).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple

# lookup_table_builder.py:18-20 (order matters: it is the MixedOperation op index)
CANDIDATE_BLOCKS: List[str] = [
    "skip", "ir_k3_e1", "ir_k3_e3", "ir_k3_s4", "ir_k5_e1", "ir_k5_e3", "ir_k5_s4",
    "ir_k3_e1_se", "ir_k3_e3_se", "ir_k3_s4_se", "ir_k5_e1_se", "ir_k5_e3_se",
    "ir_k5_s4_se", "ir_k3_s2", "ir_k5_s2", "ir_k3_s2_se", "ir_k5_s2_se",
]

# lookup_table_builder.py:22-45 -> (C_in, C_out, stride) per searched layer
SEARCH_SPACE2: List[Tuple[int, int, int]] = [
    (32, 32, 2),
    (32, 32, 1),
    (32, 64, 2),
    (64, 64, 1),
    (64, 128, 2),
    (128, 128, 1),
]

# fbnet_modeldef.py:30-95
MODEL_ARCH: Dict[str, List[str]] = {
    "wang2": ["ir_k3_e1", "ir_k5_e1", "ir_k5_s2", "ir_k3_s2", "ir_k5_e1", "skip"],
    "wang3": ["ir_k5_e1", "skip", "ir_k5_e1", "skip", "skip", "skip"],
    "wang4": ["skip", "skip", "ir_k5_s2", "ir_k3_s2", "ir_k5_e1", "ir_k5_e1"],
}

# stem: model_supernet.py:57-58  ConvBNRelu(1 -> 32, k3, s1, p1)
STEM_CHANNELS = 32
# head: model_supernet.py:64-68  Conv2d(C_last, 128, kernel_size=4, bias=False) + BN(affine=False)
HEAD_KERNEL = 4
DESC_DIM = 128


@dataclass(frozen=True)
class OpSpec:
    """Arguments a candidate passes to IRFBlock (fbnet_builder.py:455-490)."""
    kind: str          # "skip" or "ir"
    expansion: int = 1
    kernel: int = 3
    pw_group: int = 1
    shuffle: bool = False  # shuffle_type == "mid"
    se: bool = False


def _ir(e: int, k: int, g: int = 1, se: bool = False) -> OpSpec:
    return OpSpec("ir", expansion=e, kernel=k, pw_group=g, shuffle=g > 1, se=se)


# fbnet_builder.py:36-191, restricted to the ops reachable from CANDIDATE_BLOCKS
# (plus the e6 variants, which the same IRFBlock code covers).
OP_SPECS: Dict[str, OpSpec] = {
    "skip": OpSpec("skip"),
    "ir_k3_e1": _ir(1, 3), "ir_k3_e3": _ir(3, 3), "ir_k3_e6": _ir(6, 3),
    "ir_k3_s4": _ir(4, 3, 4),
    "ir_k5_e1": _ir(1, 5), "ir_k5_e3": _ir(3, 5), "ir_k5_e6": _ir(6, 5),
    "ir_k5_s4": _ir(4, 5, 4),
    "ir_k3_e1_se": _ir(1, 3, se=True), "ir_k3_e3_se": _ir(3, 3, se=True),
    "ir_k3_e6_se": _ir(6, 3, se=True), "ir_k3_s4_se": _ir(4, 3, 4, se=True),
    "ir_k5_e1_se": _ir(1, 5, se=True), "ir_k5_e3_se": _ir(3, 5, se=True),
    "ir_k5_e6_se": _ir(6, 5, se=True), "ir_k5_s4_se": _ir(4, 5, 4, se=True),
    "ir_k3_s2": _ir(1, 3, 2), "ir_k5_s2": _ir(1, 5, 2),
    "ir_k3_s2_se": _ir(1, 3, 2, se=True), "ir_k5_s2_se": _ir(1, 5, 2, se=True),
}


def se_mid(c: int) -> int:
    """SEModule hidden width, fbnet_builder.py:407-413 (reduction 4, floor 8)."""
    return max(c // 4, 8)


def ir_mid(c_in: int, expansion: int) -> int:
    """IRFBlock mid width, fbnet_builder.py:479-480 (width_divisor=1 -> int(C_in*e))."""
    return int(c_in * expansion)


def arch_ops(arch) -> List[str]:
    """Accept a registry name ('wang2') or an explicit list of 6 op names."""
    if isinstance(arch, str):
        if arch not in MODEL_ARCH:
            raise KeyError(f"unknown arch {arch!r}; known: {sorted(MODEL_ARCH)}")
        ops = MODEL_ARCH[arch]
    else:
        ops = list(arch)
    if len(ops) != len(SEARCH_SPACE2):
        raise ValueError(f"arch needs {len(SEARCH_SPACE2)} ops, got {len(ops)}")
    for o in ops:
        if o not in CANDIDATE_BLOCKS:
            raise ValueError(f"op {o!r} is not a CANDIDATE_BLOCKS entry")
    return list(ops)


def layer_macs(c_in: int, c_out: int, stride: int, op: str, hw_in: int) -> int:
    """Multiply-accumulates of one searched layer for one patch (documentation/bench)."""
    spec = OP_SPECS[op]
    hw_out = hw_in // stride
    if spec.kind == "skip":
        if c_in == c_out:
            return 0
        return c_in * c_out * hw_out * hw_out
    mid = ir_mid(c_in, spec.expansion)
    g = spec.pw_group
    macs = (c_in // g) * mid * hw_in * hw_in            # pw
    macs += spec.kernel * spec.kernel * mid * hw_out * hw_out  # dw
    macs += (mid // g) * c_out * hw_out * hw_out        # pwl
    if spec.se:
        m = se_mid(c_out)
        macs += 2 * c_out * m
    return macs


def nas_macs(arch) -> int:
    ops = arch_ops(arch)
    hw = 32
    total = 1 * STEM_CHANNELS * 9 * hw * hw
    for (ci, co, s), op in zip(SEARCH_SPACE2, ops):
        total += layer_macs(ci, co, s, op, hw)
        hw //= s
    total += SEARCH_SPACE2[-1][1] * DESC_DIM * HEAD_KERNEL * HEAD_KERNEL
    return total


# FDLNet's hand-instantiated NAS descriptors (HardNetNeiMask,
# FDLNet-master/latency/NASNet/model/des.py:8-55 and latency/NASNet_0.1/model/des.py:10-55):
# a fixed front on the 32x32 patch to 8x8x64, then three IRFBlocks from the same op vocabulary
# (latency/NASNet/model/operations.py:205-320 == fbnet_builder.IRFBlock), the 4x4 head and
# torch.norm L2.  The variants differ only in the front:
#   "NASNet":     Conv 3x3 (bias) -> BN(affine=False) -> [Conv 1x1 s2 -> BN -> ReLU] x 2 (32, 64)
#   "NASNet_0.1": Conv 3x3 (bias) -> MaxPool(3, 2, 1) -> Identity -> ConvBNRelu 1x1 s2 (64)
FDL_VARIANTS = ("NASNet", "NASNet_0.1")
FDL_LAYERS: List[Tuple[int, int, int]] = [(64, 64, 1), (64, 128, 2), (128, 128, 1)]
FDL_OPS: List[str] = ["ir_k5_e1", "ir_k3_e3", "ir_k5_s2"]  # IRFBlock(64,64,1,1,k5), (64,128,3,2,k3), (128,128,1,1,k5,mid,g2)
FDL_INPUT_NORM_EPS = 1e-8


def fdl_macs(variant: str) -> int:
    """MACs per patch of the FDLNet descriptor as the reference computes it (full 32x32 stem)."""
    total = 9 * 32 * 32 * 32                       # stem
    if variant == "NASNet":
        total += 32 * 32 * 16 * 16 + 32 * 64 * 8 * 8  # two 1x1 stride-2 convs
    else:
        total += 32 * 64 * 8 * 8                     # 1x1 stride-2 conv after the maxpool
    hw = 8
    for (ci, co, s), op in zip(FDL_LAYERS, FDL_OPS):
        total += layer_macs(ci, co, s, op, hw)
        hw //= s
    return total + 128 * DESC_DIM * HEAD_KERNEL * HEAD_KERNEL


# Stock HardNet conv stack (hardnet/HardNet.py:280-302): (C_in, C_out, k, stride, pad, relu)
HARDNET_CONVS: List[Tuple[int, int, int, int, int, bool]] = [
    (1, 32, 3, 1, 1, True),
    (32, 32, 3, 1, 1, True),
    (32, 64, 3, 2, 1, True),
    (64, 64, 3, 1, 1, True),
    (64, 128, 3, 2, 1, True),
    (128, 128, 3, 1, 1, True),
    (128, 128, 8, 1, 0, False),
]
# indices of the conv / BN modules inside HardNet.features (Dropout sits at 18)
HARDNET_CONV_IDX = [0, 3, 6, 9, 12, 15, 19]
HARDNET_BN_IDX = [1, 4, 7, 10, 13, 16, 20]


def hardnet_macs() -> int:
    hw = 32
    total = 0
    for ci, co, k, s, p, _ in HARDNET_CONVS:
        ho = (hw + 2 * p - k) // s + 1
        total += ci * co * k * k * ho * ho
        hw = ho
    return total
