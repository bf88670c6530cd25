#!/usr/bin/env python3
"""Throughput of the MI355X descriptor forward -- BASELINE.json metric
"Mpatches/s (32x32 -> 128-D)".

One step = one eval forward of B synthetic patches already resident in HBM (default:
stock HardNet, B = 262,144 per GPU = BASELINE config 2) through the hand-written
gfx950 kernels (C ABI), plus -- when N > 1 -- the RCCL all-gather of the [B,128]
descriptors that reassembles the descriptor matrix (BASELINE config 4).  Per-GPU work
is fixed (weak scaling); ``value`` = patches processed by all ranks / max-over-ranks
wall time of the K timed steps.

Extra objects on the JSON line:
  roofline      dominant kernel's algorithmic FLOP per launch / its average launch
                duration (hipEvents recorded by the library on the launch stream
                during the timed region), against the bf16x3 effective peak.
  cpu_baseline  the torch-CPU restatement of the same forward (oracle/), rank 0 at
                N = 1 only, on a bounded sample.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--model hardnet|wang2|...|fdl_NASNet|fdl_NASNet_01]
For N > 1 launch with torch.distributed.run (one process per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from hardnetnas_amd import arch as A  # noqa: E402
from hardnetnas_amd import synth  # noqa: E402
from hardnetnas_amd._native import NativeModel  # noqa: E402
from hardnetnas_amd.model import HardNet, HardNetNAS, HardNetNeiMask  # noqa: E402

METRIC = "Mpatches/s (32×32→128-D) at 1/2/4/8 MI355X; HPatches FPR95 parity"
PEAK_MFMA_BF16 = 2500.0           # TFLOP/s dense bf16 (MI355X_MICROARCH.md)
PEAK_BF16X3 = PEAK_MFMA_BF16 / 3  # fp32-equivalent: 3 bf16 MFMAs per fp32 product
PEAK_FP32 = 157.3                 # TFLOP/s f32 (vector == f32 MFMA)
PEAK_HBM = 8000.0                 # GB/s

# algorithmic work per patch of each HardNet stage
HARDNET_STAGE_MAC = {"stem": 294912, "conv1": 9437184, "stem+conv1": 294912 + 9437184,
                     "stem+conv1+conv2": 294912 + 9437184 + 4718592,
                     "conv2": 4718592, "conv3": 9437184, "conv4": 4718592, "conv5": 9437184,
                     "head": 1048576}
HARDNET_STAGE_BYTES = {"stem": 4096 + 131072, "conv1": 2 * 131072, "stem+conv1": 4096 + 131072,
                       "stem+conv1+conv2": 4096 + 65536,
                       "conv2": 131072 + 65536, "conv3": 2 * 65536, "conv4": 65536 + 32768,
                       "conv5": 2 * 32768, "head": 32768 + 512}


# hn_irf.hip HN_IRF2_SHAPES: (C_A, H, k_A, mid_A, C_B, k_B, mid_B) of the two-block fused kernel k_irf2
IRF2_SHAPES = {(32, 16, ka, 32, 64, kb, 32) for ka in (3, 5) for kb in (3, 5)} | \
              {(64, 8, ka, 64, 128, kb, 64) for ka in (3, 5) for kb in (3, 5)}


def irf2_pairs(ops) -> set:
    """First layers of the block pairs hn_api.hip::forward_nas runs as one k_irf2 (a stride-1 block
    without SE followed by a stride-2 block at the same resolution), unless HN_NO_IRF2 / HN_NO_IRF."""
    if os.environ.get("HN_NO_IRF2", "0") not in ("", "0") or os.environ.get("HN_NO_IRF", "0") not in ("", "0"):
        return set()
    ops = A.arch_ops(ops)
    out, hw, i = set(), 32, 0
    hws = []
    for (ci, co, s) in A.SEARCH_SPACE2:
        hws.append(hw)
        hw //= s
    i = 1
    while i + 1 < len(ops):
        a, b = A.OP_SPECS[ops[i]], A.OP_SPECS[ops[i + 1]]
        (ci, co, s), (cb_in, cb, sb) = A.SEARCH_SPACE2[i], A.SEARCH_SPACE2[i + 1]
        if (a.kind != "skip" and b.kind != "skip" and not a.se and s == 1 and ci == co and sb == 2 and
                (ci, hws[i], a.kernel, A.ir_mid(ci, a.expansion), cb, b.kernel,
                 A.ir_mid(cb_in, b.expansion)) in IRF2_SHAPES):
            out.add(i)
            i += 2
        else:
            i += 1
    return out


def irf3_triples(ops) -> set:
    """First layers i of the k_irf2 pairs that hn_api.hip::forward_nas extends to k_irf3: the 8x8 64-channel pair
    (i, i + 1), B without SE, then layer i + 2 a 4x4 stride-1 128 -> 128 block of mid 128 (e1 / s2 ops) without SE,
    kernels 3 / 5 -- only with HN_IRF3=1 on the experiments library (HN_LIB; measured slower)."""
    if os.environ.get("HN_IRF3", "0") in ("", "0") or "abl" not in os.environ.get("HN_LIB", ""):
        return set()
    ops = A.arch_ops(ops)
    out = set()
    for i in irf2_pairs(ops):
        if i + 2 >= len(ops) or A.SEARCH_SPACE2[i][0] != 64:
            continue
        b, c = A.OP_SPECS[ops[i + 1]], A.OP_SPECS[ops[i + 2]]
        ci, co, s = A.SEARCH_SPACE2[i + 2]
        if (not b.se and c.kind != "skip" and not c.se and s == 1 and ci == co == 128
                and A.ir_mid(ci, c.expansion) == 128 and c.kernel in (3, 5)):
            out.add(i)
    return out


def mpfront_irf(ops) -> bool:
    """True when hn_api.hip::forward_nas runs the max-pool front (layer 0 "skip" at stride 2), the identity layer 1
    and the 16x16 stride-2 32 -> 64 layer-2 block (no SE, mid 32 / 96 / 128) as one k_mpfront_irf, unless
    HN_NO_MPFRONT / HN_NO_FRONT (float input; the uint8 modes keep the two kernels)."""
    if any(os.environ.get(k, "0") not in ("", "0") for k in ("HN_NO_MPFRONT", "HN_NO_FRONT")):
        return False
    ops = A.arch_ops(ops)
    spec = A.OP_SPECS[ops[2]]
    return (ops[0] == "skip" and ops[1] == "skip" and spec.kind != "skip" and not spec.se
            and A.ir_mid(32, spec.expansion) in (32, 96, 128))


def irf_skip_layers(ops) -> dict:
    """{i: n}: the IRF layer i (16x16 stride 2, 32 -> 64, no SE, not in a k_irf2 pair) whose output goes
    -- past identity skips -- into the 8x8 64 -> 128 stride-2 skip of layer n, both in one k_irf_skip
    (hn_api.hip::forward_nas), unless HN_NO_IRFSKIP / HN_NO_SKIPFUSE / HN_NO_IRF."""
    if any(os.environ.get(k, "0") not in ("", "0") for k in ("HN_NO_IRFSKIP", "HN_NO_SKIPFUSE", "HN_NO_IRF")):
        return {}
    ops = A.arch_ops(ops)
    pairs = irf2_pairs(ops)
    out = {}
    mpf = mpfront_irf(ops)
    for i in range(1, len(ops)):
        spec, (ci, co, s) = A.OP_SPECS[ops[i]], A.SEARCH_SPACE2[i]
        if (spec.kind == "skip" or spec.se or i in pairs or i - 1 in pairs or (ci, co, s) != (32, 64, 2) or mpf
                or A.ir_mid(ci, spec.expansion) not in (32, 96, 128)):
            continue
        n = i + 1
        while n < len(ops) and A.OP_SPECS[ops[n]].kind == "skip" and A.SEARCH_SPACE2[n][2] == 1 and \
                A.SEARCH_SPACE2[n][0] == A.SEARCH_SPACE2[n][1]:
            n += 1
        if n < len(ops) and A.OP_SPECS[ops[n]].kind == "skip" and A.SEARCH_SPACE2[n] == (64, 128, 2):
            out[i] = n
    return out


def nas_stage_bytes(ops) -> dict:
    """Algorithmic HBM bytes per patch of each NAS stage class, summed over its launches in
    one forward (fp32 NHWC in + out (+ residual read)), mirroring hn_api.hip::forward_nas
    (stem + layer 0 run as one fused "front" kernel unless HN_NO_FRONT=1; IRF layers 1..5 as
    fused "irf" blocks unless HN_NO_IRF=1)."""
    front = os.environ.get("HN_NO_FRONT", "0") in ("", "0")
    irf = os.environ.get("HN_NO_IRF", "0") in ("", "0")
    out = {"stem": 0 if front else 4096 + 32 * 32 * 32 * 4, "front": 0, "irf": 0, "irf2": 0, "skip": 0, "pw": 0,
           "dw": 0, "pwl": 0, "maxpool": 0, "se": 0, "head": 0, "irf+skip": 0, "front+irf": 0, "irf3": 0}
    pairs = irf2_pairs(ops)
    triples = irf3_triples(ops)
    in3 = {j for i in triples for j in (i, i + 1, i + 2)}
    fused_skip = irf_skip_layers(ops)
    skipped = {n for n in fused_skip.values()}
    mpf = mpfront_irf(ops)
    hw = 32
    for i, (op, (ci, co, s)) in enumerate(zip(A.arch_ops(ops), A.SEARCH_SPACE2)):
        spec = A.OP_SPECS[op]
        ho = hw // s
        if mpf and i < 3:  # k_mpfront_irf: the patch in, layer 2's 8x8x64 out
            out["front+irf"] += 4096 + 4 * 64 * 8 * 8 if i == 0 else 0
            hw = ho
            continue
        if i in fused_skip:  # k_irf_skip: the block's input in, the skip's 4x4x128 output out
            out["irf+skip"] += 4 * ci * hw * hw + 4 * 128 * 4 * 4
            hw = ho
            continue
        if i in skipped:
            hw = ho
            continue
        if i in in3:  # k_irf3: the pair's input in, layer i + 2's 4x4x128 output out
            out["irf3"] += 4 * ci * hw * hw + 4 * 128 * 4 * 4 if i in triples else 0
            hw = ho
            continue
        if i in pairs:  # k_irf2: this block's input in, the next block's output out
            _, co2, s2 = A.SEARCH_SPACE2[i + 1]
            out["irf2"] += 4 * ci * hw * hw + 4 * co2 * (hw // s2) ** 2
            hw = ho
            continue
        if i - 1 in pairs:
            if spec.se:
                out["se"] += 4 * 2 * co * ho * ho
            hw = ho
            continue
        fused = front and i == 0
        if spec.kind == "skip":
            if fused:
                out["front"] += 4096 + 4 * ci * ho * ho
            elif s == 2 and ci != co and os.environ.get("HN_NO_SKIPFUSE", "0") in ("", "0"):
                out["skip"] += 4 * (ci * hw * hw + co * ho * ho)  # k_skip_s2: maxpool + 1x1 fused
                hw = ho
                continue
            elif s == 2:
                out["maxpool"] += 4 * (ci * hw * hw + ci * ho * ho)
            if ci != co:
                out["pw"] += 4 * (ci * ho * ho + co * ho * ho)
        else:
            mid = A.ir_mid(ci, spec.expansion)
            if fused or (irf and i > 0):
                # fused front (stem + layer 0) / fused block: x in + y out only (the residual
                # re-read of x is not counted)
                out["front" if fused else "irf"] += (4096 if fused else 4 * ci * hw * hw) + 4 * co * ho * ho
                if spec.se:
                    out["se"] += 4 * 2 * co * ho * ho
                hw = ho
                continue
            out["pw"] += 4 * (ci * hw * hw + mid * hw * hw)
            out["dw"] += 4 * (mid * hw * hw + mid * ho * ho)
            res = (s == 1 and ci == co)
            out["pwl"] += 4 * (mid * ho * ho + co * ho * ho + (co * ho * ho if res else 0))
            if spec.se:
                out["se"] += 4 * 2 * co * ho * ho
        hw = ho
    out["head"] = 4 * (A.SEARCH_SPACE2[-1][1] * 16 + 2 * 128)
    return out


# FDLNet HardNetNeiMask descriptors (bench --model fdl_NASNet | fdl_NASNet_01)
FDL_MODELS = {"fdl_NASNet": "NASNet", "fdl_NASNet_01": "NASNet_0.1"}


def fdl_stage_bytes(name: str) -> dict:
    """Algorithmic HBM bytes per patch of each FDL stage: the fused front (patch in, 8x8x64
    out), the three fused IRF blocks (x in + y out), the head (4x4x128 in, 128 out)."""
    irf, hw = 0, 8
    for ci, co, s in A.FDL_LAYERS:
        irf += 4 * (ci * hw * hw + co * (hw // s) ** 2)
        hw //= s
    return {"front": 4096 + 4 * 64 * 64, "irf": irf, "head": 4 * (128 * 16 + 128)}


def build_model(name: str):
    """Synthetic weights (splitmix64 seed 1234) + the calibrated BN statistics committed
    with the golden fixtures (tests/golden/*.npz, data only)."""
    if name in FDL_MODELS:
        m, fxname = HardNetNeiMask(variant=FDL_MODELS[name]), name
    else:
        m = HardNet() if name == "hardnet" else HardNetNAS(name)
        fxname = "hardnet" if name == "hardnet" else "nas_" + name
    fx = np.load(os.path.join(ROOT, "tests", "golden", fxname + ".npz"))
    sd = m.state_dict()
    tmpl = {k: tuple(v.shape) for k, v in sd.items()}
    w = synth.synth_state_dict(tmpl, 1234)
    for k in w:
        sd[k] = torch.from_numpy(fx["bn/" + k] if "running" in k else w[k])
    m.load_state_dict(sd)
    return m.eval()


# BASELINE config 4: 16,777,216 patches sharded over 8 ranks (weak scaling: fixed per rank)
CONFIG4_PER_RANK = 16_777_216 // 8


def synth_input_on_device(b: int, device, seed: int) -> torch.Tensor:
    g = torch.Generator(device=device).manual_seed(seed)
    q = torch.randint(0, 256, (b, 1, 32, 32), device=device, generator=g, dtype=torch.int32)
    x = q.float() / 255.0
    return (x - synth.MEAN_IMAGE) / synth.STD_IMAGE


def flop_per_patch(name: str) -> int:
    if name in FDL_MODELS:
        return 2 * A.fdl_macs(FDL_MODELS[name])
    return 2 * (A.hardnet_macs() if name == "hardnet" else A.nas_macs(name))


def _cpu_model_string() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _cpu_quota() -> float:
    """CPUs this cgroup may use (cpu.max quota / period), or 0 if unlimited / unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        return 0.0 if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return 0.0


def cpu_baseline(name: str, model, seconds: float = 12.0, x_timed=None, y_timed=None, check_rows=1024):
    """The oracle (torch fp32 CPU restatement of the reference forward) timed on
    the host's cores: torch.set_num_threads(nproc), plus a 1-thread figure and -- when the
    cgroup grants fewer CPUs than nproc shows -- the quota's thread count; ``value`` is the best
    of them (the strongest CPU number this host gives).  With the timed GPU input/output it
    also checks the GPU run at its own size: a strided ``check_rows``-row sample of the timed
    batch through the same oracle (the sample *is* the timed CPU workload)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import hardnet_oracle as O
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    b = 1024
    if x_timed is not None:
        idx = torch.arange(0, x_timed.shape[0], max(1, x_timed.shape[0] // check_rows))[:check_rows]
        idx = idx + min(255, x_timed.shape[0] - 1 - int(idx[-1]))  # also rows away from chunk starts
        x = x_timed[idx.to(x_timed.device)].cpu()
        b = x.shape[0]
    else:
        idx, x = None, torch.from_numpy(synth.synth_patches(b, seed=11))

    def run():
        with torch.no_grad():
            if name == "hardnet":
                return O.hardnet_forward(p, x)
            if name in FDL_MODELS:
                return O.fdl_forward(p, FDL_MODELS[name], x)
            return O.nas_forward(p, model.arch_ops, x)

    def timed(threads, secs, min_runs=3):
        torch.set_num_threads(threads)
        run()
        rates, t_start = [], time.perf_counter()
        while time.perf_counter() - t_start < secs or len(rates) < min_runs:
            t0 = time.perf_counter()
            run()
            rates.append(b / (time.perf_counter() - t0))
        return statistics.median(rates), len(rates)

    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = _cpu_quota()
    legs = {nproc: None}
    if 0 < quota < nproc:
        legs[max(1, int(quota))] = None
    legs[1] = None
    share = seconds / (len(legs) + 1)
    for t in sorted(legs, reverse=True):
        # nproc threads under a much smaller CPU quota are throttled: keep that leg short
        legs[t] = timed(t, 2 * share if t == nproc else share,
                        1 if (t == nproc and 0 < quota < nproc / 2) else 3)
    torch.set_num_threads(best_threads := max(legs, key=lambda t: legs[t][0]))
    best = best_threads
    out = {"value": round(legs[best][0], 1), "unit": "patches/s", "cores": best, "kind": "port",
           "nproc": nproc, "cgroup_cpu_quota": quota or None, "model": _cpu_model_string(),
           "value_nproc": round(legs[nproc][0], 1), "value_1t": round(legs[1][0], 1),
           "sample": f"oracle/hardnet_oracle.py {name} fp32 torch-CPU forward, batch {b} "
                     + ("(a strided sample of the timed GPU batch)" if idx is not None else "")
                     + f", ~{seconds:.0f} s over thread counts "
                     + ", ".join(f"{t}: {legs[t][0]:.0f}/s x{legs[t][1]}" for t in sorted(legs))
                     + f"; value = best ({best} threads), median per leg"}
    if 0 < quota < nproc:
        out["value_quota"] = round(legs[max(1, int(quota))][0], 1)
    if idx is not None and y_timed is not None:
        ref = run()
        got = y_timed[idx.to(y_timed.device)].cpu()
        tol = 1e-4 if name == "hardnet" else 2e-5
        err = float((got - ref).abs().max())
        dev_norm = float((y_timed.norm(dim=1) - 1).abs().max())
        out_check = {"rows": int(b), "of": int(x_timed.shape[0]), "max_abs_err_vs_oracle": err, "tol": tol,
                     "unit_norm_max_dev_all_rows": dev_norm, "ok": bool(err <= tol and dev_norm < 1e-5)}
        return out, out_check
    return out, None


def nas_stage_flop(name: str) -> dict:
    """Algorithmic FLOP per patch of each NAS / FDL stage class (summed over its launches in one
    forward), mirroring hn_api.hip::forward_nas (fused front = stem + layer 0; "irf" = every
    fused IRF block; "skip" = the fused maxpool + 1x1 ConvBNRelu; "irf+skip" = k_irf_skip; head = 4x4 conv)."""
    if name in FDL_MODELS:
        v = FDL_MODELS[name]
        front = 9 * 32 * 32 * 32 + (32 * 32 * 16 * 16 + 32 * 64 * 64 if v == "NASNet" else 32 * 64 * 64)
        irf, hw = 0, 8
        for (ci, co, st), op in zip(A.FDL_LAYERS, A.FDL_OPS):
            irf += A.layer_macs(ci, co, st, op, hw)
            hw //= st
        return {"front": 2 * front, "irf": 2 * irf, "head": 2 * 128 * 128 * 16}
    ops = A.arch_ops(name)
    out = {"front": 0, "irf": 0, "irf2": 0, "skip": 0, "irf+skip": 0, "front+irf": 0, "irf3": 0,
           "head": 2 * A.SEARCH_SPACE2[-1][1] * 128 * 16}
    pairs = irf2_pairs(ops)
    in3 = {j for i in irf3_triples(ops) for j in (i, i + 1, i + 2)}
    fused_skip = irf_skip_layers(ops)
    skipped = set(fused_skip.values())
    mpf = mpfront_irf(ops)
    hw = 32
    for i, (op, (ci, co, st)) in enumerate(zip(ops, A.SEARCH_SPACE2)):
        macs = A.layer_macs(ci, co, st, op, hw)
        if mpf and i < 3:
            out["front+irf"] += 2 * (macs + (9 * 32 * 32 * 32 if i == 0 else 0))
        elif i in fused_skip or i in skipped:
            out["irf+skip"] += 2 * macs
        elif i in in3:
            out["irf3"] += 2 * macs
        elif i in pairs or i - 1 in pairs:
            out["irf2"] += 2 * macs
        elif i == 0:
            out["front"] += 2 * (9 * 32 * 32 * 32 + macs)
        elif A.OP_SPECS[op].kind == "skip":
            out["skip"] += 2 * macs
        else:
            out["irf"] += 2 * macs
        hw //= st
    return out


def cpu_baseline_pairs(model, seconds: float = 8.0, pairs: int = 2048):
    """Config 5 on the host cores (rank 0, N = 1): the oracle's HardNet forward of `pairs` anchor /
    positive pairs (2 x `pairs` patches) followed by its loss_HardNet (Losses.py:87-154, anchor_swap,
    the B x B matrix materialised as the reference does), at the quota's thread count.  ``value`` is
    whole-step patches/s at that batch; the pair step alone is also timed at B = 4,096 pairs
    (SURVEY/BASELINE.md's CPU pair-step row)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import hardnet_oracle as O
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = _cpu_quota()
    threads = max(1, int(quota)) if 0 < quota < nproc else nproc
    torch.set_num_threads(threads)
    xa = torch.from_numpy(synth.synth_patches(pairs, seed=21))
    xp = xa + 0.3 * torch.from_numpy(synth.synth_patches(pairs, seed=22))
    g = torch.Generator().manual_seed(3)
    da = torch.nn.functional.normalize(torch.randn(4096, 128, generator=g), dim=1)
    dp = torch.nn.functional.normalize(da + 0.3 * torch.randn(4096, 128, generator=g), dim=1)

    def step():
        with torch.no_grad():
            ya, yp = O.hardnet_forward(p, xa), O.hardnet_forward(p, xp)
            return O.loss_hardnet(ya, yp, anchor_swap=True)

    def pair_only():
        with torch.no_grad():
            return O.loss_hardnet(da, dp, anchor_swap=True)

    step()
    pair_only()
    t_step, t_pair, t_start = [], [], time.perf_counter()
    while time.perf_counter() - t_start < seconds or len(t_step) < 2:
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        pair_only()
        t_step.append(t1 - t0)
        t_pair.append(time.perf_counter() - t1)
    ms, mp = statistics.median(t_step), statistics.median(t_pair)
    return {"value": round(2 * pairs / ms, 1), "unit": "patches/s", "cores": threads, "kind": "port",
            "nproc": nproc, "cgroup_cpu_quota": quota or None, "model": _cpu_model_string(),
            "pair_step_pairs_per_s_b4096": round(4096 / mp, 1), "pair_step_ms_b4096": round(mp * 1e3, 2),
            "step_ms": round(ms * 1e3, 1),
            "sample": f"oracle/hardnet_oracle.py: forward of {pairs} anchor + {pairs} positive patches then "
                      f"loss_hardnet (anchor_swap, B x B matrix) at {threads} threads, median of {len(t_step)} "
                      f"steps (~{seconds:.0f} s); the pair step alone (loss_hardnet over 4,096 random unit "
                      "descriptor pairs) timed beside it"}


def check_pairs(out, pairs, pos, min_neg, rows=1024):
    """The timed config-5 step at its own size: the oracle's hardest_negative_rows (fp64) on a
    strided row sample of the 65,536-pair batch against the GPU's pos / min_neg of those rows."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import hardnet_oracle as O
    idx = torch.arange(0, pairs, max(1, pairs // rows))[:rows]
    a = out[:pairs].detach().double().cpu()
    p_ = out[pairs:2 * pairs].detach().double().cpu()
    rp, rn = O.hardest_negative_rows(a, p_, idx, anchor_swap=True)
    gp, gn = pos[idx.to(pos.device)].double().cpu(), min_neg[idx.to(min_neg.device)].double().cpu()
    err = max(float((gp - rp).abs().max()), float((gn - rn).abs().max()))
    return {"rows": int(len(idx)), "of": int(pairs), "max_abs_err_vs_oracle_fp64": err, "tol": 1e-4,
            "what": "pos and min_neg (anchor_swap) of sampled rows vs oracle.hardest_negative_rows",
            "ok": bool(err <= 1e-4)}


def read_pmc(name: str):
    """profiles/pmc_<name>.json (tools/pmc_stage.py: per-stage HBM bytes and instruction counts
    per patch from rocprofv3 --pmc passes on the current build), or None."""
    f = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    if not os.path.exists(f):
        return None
    try:
        return json.load(open(f))
    except Exception:
        return None


CLOCK_GHZ = 2.4           # MI355X peak engine clock (MI355X_MICROARCH.md)
SIMDS = 256 * 4
VALU_ISSUE_CYC = 2        # cycles per wave64 VALU instruction on a SIMD-32 (MI355X_MICROARCH.md)


def run(opts, world, rank, local, dev, on_gpu, backend):
    """One measured configuration: W warmup steps, then K timed steps bracketed by a barrier and a
    device synchronisation on both sides; max over ranks.  Returns rank 0's result dict."""
    cfg5 = opts.config == 5
    model = build_model(opts.model)
    nm = NativeModel.from_module(model, dev) if on_gpu else None
    pairs = None
    if cfg5:
        pairs = opts.batch or 65536
        from hardnetnas_amd.distributed import shard_range, sharded_hardnet_loss
        s0, e0 = shard_range(pairs, world, rank) if world > 1 else (0, pairs)
        b = 2 * (e0 - s0)  # this rank's anchors and positives, one forward
    else:
        b = opts.batch
        if b is None:
            b = (CONFIG4_PER_RANK if (world > 1 and opts.model == "hardnet") else 262144) if on_gpu else 256
    u8_mode = opts.input[3:] if opts.input.startswith("u8-") else None
    x = synth_input_on_device(b, dev, seed=1000 + rank)
    if u8_mode:
        hw = 32 if u8_mode == "none" else 64
        x8 = torch.randint(0, 256, (b, hw, hw), device=dev, dtype=torch.uint8,
                           generator=torch.Generator(device=dev).manual_seed(1000 + rank))
    if cfg5:  # positives = anchors + noise (the same patch seen twice), as a real pair batch
        x[b // 2:] = x[: b // 2] + 0.3 * torch.randn(b // 2, 1, 32, 32, device=dev,
                                                     generator=torch.Generator(device=dev).manual_seed(7 + rank))
    out = torch.empty((b, 128), device=dev)
    ws = torch.empty(nm.workspace_bytes_u8(b) if u8_mode else nm.workspace_bytes(b), device=dev,
                     dtype=torch.uint8) if on_gpu else None
    gathered = torch.empty((b * world, 128), device=dev) if (world > 1 and not cfg5) else None
    last = {}

    def forward():
        if u8_mode:
            nm.forward_u8(x8, resize=u8_mode, out=out, workspace=ws)
        elif on_gpu:
            nm.forward(x, out=out, workspace=ws)
        else:
            with torch.no_grad():
                out.copy_(model(x))

    def collective_or_pairs():
        if cfg5:
            n = b // 2
            if world > 1:
                last["loss"], last["pos"], last["min_neg"] = sharded_hardnet_loss(out[:n], out[n:], pairs,
                                                                                  anchor_swap=True)
            else:
                from hardnetnas_amd._native import hardnet_loss, pairdist_rows
                pos, rmin, cmin = pairdist_rows(out[:n], 0, out[n:], col_min=True)
                last["loss"], last["min_neg"] = hardnet_loss(pos, rmin, cmin)
                last["pos"] = pos
        elif world > 1 and not opts.no_allgather:
            if backend == "gloo":
                dist.all_gather(list(gathered.chunk(world)), out)
            else:
                dist.all_gather_into_tensor(gathered, out)

    if on_gpu:
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(opts.steps)]
    cpu_phase = [0.0, 0.0]

    def step(k=None):
        if on_gpu and k is not None:
            evs[k][0].record()
        t0 = time.perf_counter()
        forward()
        if on_gpu and k is not None:
            evs[k][1].record()
        t1 = time.perf_counter()
        collective_or_pairs()
        if on_gpu and k is not None:
            evs[k][2].record()
        if not on_gpu and k is not None:
            cpu_phase[0] += t1 - t0
            cpu_phase[1] += time.perf_counter() - t1

    for _ in range(opts.warmup):
        step()
    if on_gpu:
        torch.cuda.synchronize()
        nm.stage_times()  # clear
        nm.set_profiling(True)
    if world > 1:
        dist.barrier()
    if on_gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(opts.steps):
        step(k)
    if on_gpu:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if on_gpu:
        nm.set_profiling(False)
        stages = nm.stage_times()
        phase = [sum(e[0].elapsed_time(e[1]) for e in evs), sum(e[1].elapsed_time(e[2]) for e in evs)]
    else:
        stages = {}
        phase = [1e3 * cpu_phase[0], 1e3 * cpu_phase[1]]
    ranks_seen = world
    if world > 1:
        t = torch.tensor([elapsed, phase[0], phase[1]], device=dev if backend == "nccl" else "cpu",
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, phase = t[0].item(), [t[1].item(), t[2].item()]
        cnt = torch.ones(1, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(cnt)
        ranks_seen = int(cnt.item())

    total = (pairs * 2 if cfg5 else b * world) * opts.steps
    value = total / elapsed / 1e6
    if rank != 0:
        return None
    roof = None
    if on_gpu:
        stages_ms = {k: round(v[0] / opts.steps, 3) for k, v in stages.items()}
        if cfg5:
            # the pair step's own roofline: distance FLOP (2 B^2 D) over its time
            pair_ms = phase[1] / opts.steps
            flop = 2.0 * pairs * pairs * 128 / world
            achieved = flop / (pair_ms * 1e-3) / 1e12
            pmc = read_pmc("c5") or {}
            tr = pmc.get("pairdist") if pmc.get("pairs") == pairs and world == 1 else None
            roof = {"bound": "mfma", "kernel": "pair step (k_pairdist_ring + k_split_planes/k_sq/k_pos/k_loss)",
                    "achieved": round(achieved, 2), "peak": round(PEAK_BF16X3, 1), "unit": "TFLOP/s",
                    "frac": round(achieved / PEAK_BF16X3, 4),
                    "traffic": int(tr["bytes_per_launch"]) if tr else None,
                    "traffic_source": "profiles/pmc_c5.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate "
                                      "passes, k_pairdist_ring at this batch)" if tr else None,
                    "avg_launch_ms": round(pair_ms, 4), "launches": opts.steps,
                    "pairs_per_launch": int(pairs),
                    "peak_basis": "bf16 MFMA dense 2.5 PFLOP/s / 3 (bf16x3 split-precision distance "
                                  "dots); algorithmic FLOP = 2 * B^2 * 128 per step",
                    "forward_stages_ms_per_step": stages_ms}
        else:
            # dominant kernel = stage with the largest summed device time
            dom = max(stages, key=lambda k: stages[k][0])
            dom_ms, dom_n = stages[dom]
            avg_ms = dom_ms / max(dom_n, 1)
            launches_per_step = dom_n / opts.steps
            patches_per_launch = b / launches_per_step
            pmc = read_pmc(opts.model) or {}
            pst = pmc.get("stages", {}).get(dom)
            traffic = int(pst["bytes_per_patch"] * patches_per_launch) if pst and "bytes_per_patch" in pst else None
            if opts.model == "hardnet":
                flop = 2 * HARDNET_STAGE_MAC[dom] * patches_per_launch
                achieved = flop / (avg_ms * 1e-3) / 1e12
                alg = HARDNET_STAGE_BYTES[dom] * patches_per_launch
                roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2),
                        "peak": round(PEAK_BF16X3, 1), "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16X3, 4)}
                peak_basis = ("bf16 MFMA dense 2.5 PFLOP/s / 3 (bf16x3 split-precision fp32 products); "
                              "algorithmic FLOP = 2*MAC")
            else:
                # A NAS / FDL stage class aggregates several layers' launches.  Its roofs: the fp16x3
                # MFMA (algorithmic FLOP / summed time), HBM (PMC bytes / time) and VALU issue (PMC
                # VALU instructions x 2 cycles / SIMD-cycles of the launch).  "bound" names whichever
                # of MFMA / HBM it is closer to, "frac" is that fraction; all three are reported.
                per_patch = nas_stage_flop(opts.model).get(dom, 0)
                mfma_tf = per_patch * b * opts.steps / (dom_ms * 1e-3) / 1e12
                alg = (fdl_stage_bytes(opts.model) if opts.model in FDL_MODELS
                       else nas_stage_bytes(opts.model)).get(dom, 0) * patches_per_launch
                hbm_gbps = (traffic if traffic else alg) / (avg_ms * 1e-3) / 1e9
                mfma_frac, hbm_frac = mfma_tf / PEAK_BF16X3, hbm_gbps / PEAK_HBM
                valu_frac = None
                if pst and pst.get("valu_insts_per_patch"):
                    valu_frac = (pst["valu_insts_per_patch"] * patches_per_launch * VALU_ISSUE_CYC
                                 / (avg_ms * 1e-3 * CLOCK_GHZ * 1e9 * SIMDS))
                if hbm_frac >= mfma_frac:
                    roof = {"bound": "hbm", "kernel": dom, "achieved": round(hbm_gbps, 1), "peak": PEAK_HBM,
                            "unit": "GB/s", "frac": round(hbm_frac, 4)}
                else:
                    roof = {"bound": "mfma", "kernel": dom, "achieved": round(mfma_tf, 2),
                            "peak": round(PEAK_BF16X3, 1), "unit": "TFLOP/s", "frac": round(mfma_frac, 4)}
                fracs = {"mfma": mfma_frac, "hbm": hbm_frac, "valu_issue": valu_frac or 0.0}
                top = max(fracs, key=fracs.get)
                # what binds the stage: the resource nearest its roof, or latency when none is at half of it;
                # "bound" then says latency too, and "frac_roof" names the roof achieved / peak / frac refer to
                roof["frac_roof"] = roof["bound"]
                if fracs[top] >= 0.5:
                    roof["binding_counter"] = top
                else:
                    roof["binding_counter"] = "latency (MFMA, HBM and VALU issue all < 0.5)"
                    roof["bound"] = "latency"
                roof.update({"mfma_tflops": round(mfma_tf, 2), "mfma_frac": round(mfma_frac, 4),
                             "hbm_gbps": round(hbm_gbps, 1), "hbm_frac": round(hbm_frac, 4),
                             "hbm_bytes_basis": "PMC" if traffic else "algorithmic",
                             "valu_issue_frac": round(valu_frac, 4) if valu_frac is not None else None,
                             "mfma_busy_pmc": pst.get("mfma_busy") if pst else None})
                peak_basis = ("fp16 MFMA dense 2.5 PFLOP/s / 3 (fp16x3 split-precision 1x1 convs; depthwise "
                              "on the VALU); HBM 8 TB/s; VALU issue = 1,024 SIMDs x 2.4 GHz / 2 cycles per "
                              "wave64 instruction; algorithmic FLOP = 2*MAC")
            roof.update({"traffic": traffic, "avg_launch_ms": round(avg_ms, 4), "launches": dom_n,
                         "patches_per_launch": int(patches_per_launch),
                         "algorithmic_bytes_per_launch": int(alg) if alg else None,
                         "hbm_gbps_algorithmic": round(alg / (avg_ms * 1e-3) / 1e9, 1) if alg else None,
                         "pmc_source": f"profiles/pmc_{opts.model}.json" if pst else None,
                         "peak_basis": peak_basis, "stages_ms_per_step": stages_ms})
    if cfg5:
        workload = (f"Stock HardNet forward of {pairs} anchor/positive pairs ({2 * pairs} patches) + "
                    "fused masked distance / hardest negative (anchor_swap) / triplet margin loss")
        if world > 1:
            workload += f", pairs sharded over {world} ranks (RCCL all-gather of positives, all-reduce MIN/SUM)"
    else:
        workload = (("Stock HardNet forward" if opts.model == "hardnet"
                     else f"FDLNet HardNetNeiMask {FDL_MODELS[opts.model]} forward"
                     if opts.model in FDL_MODELS else f"hardnetNAS {opts.model} forward")
                    + f", {b} synthetic 32x32 patches per GPU"
                    + (" (BASELINE config 4 per-rank shard)" if world > 1 and b == CONFIG4_PER_RANK else "")
                    + (", RCCL all-gather of descriptors" if world > 1 and not opts.no_allgather else ""))
    if not on_gpu:
        workload += " [CPU plumbing dry run: module torch layers, gloo; not a throughput figure]"
    if u8_mode:
        workload += (f" from uint8 {'32x32' if u8_mode == 'none' else '64x64'} patches, loader "
                     f"preprocessing ({u8_mode}) fused into the forward")
    result = {
        "metric": METRIC, "value": round(value, 4 if on_gpu else 6), "unit": "Mpatches/s", "n_gpus": world,
        "steps": opts.steps, "warmup": opts.warmup,
        "ms_per_step": round(elapsed / opts.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong" if (cfg5 and world > 1) else "weak", "vs_baseline": None,
        "dtype": ("bf16x3" if opts.model == "hardnet" else "fp16x3") if on_gpu else "f32",
        "data": "synthetic",
        "config": {"workload": workload, "model": opts.model,
                   "baseline_config": 5 if cfg5 else (4 if world > 1 and b == CONFIG4_PER_RANK
                                                      else (2 if opts.model == "hardnet" else 3)),
                   "global_batch": pairs * 2 if cfg5 else b * world, "per_gpu_batch": b,
                   "parallelism": f"dp{world}",
                   "precision": "fp32 torch CPU layers (dry run)" if not on_gpu else
                                ("bf16x3 split-precision MFMA (fp32-accurate: hi/lo bf16 operands, "
                                 "3 products, fp32 accumulate)" if opts.model == "hardnet"
                                 else "fp16x3 split-precision MFMA for 1x1 convs and head, fp32 VALU depthwise"
                                 + (" and front" if opts.model in FDL_MODELS else "")),
                   "flop_per_patch": flop_per_patch(opts.model)},
        "ranks_seen": ranks_seen,
        "compute_ms": round(phase[0] / opts.steps, 3),
        ("pair_step_ms" if cfg5 else "allgather_ms"): round(phase[1] / opts.steps, 3),
        "roofline": roof,
        "cpu_baseline": None,
    }
    if cfg5:
        result["pairs_per_s"] = round(pairs * opts.steps / elapsed, 1)
        result["loss"] = float(last["loss"].item()) if "loss" in last else None
    if world == 1 and on_gpu and not opts.no_cpu_baseline:
        if cfg5:
            cb, check = cpu_baseline_pairs(model, opts.cpu_seconds), check_pairs(out, pairs, last["pos"],
                                                                                   last["min_neg"])
        elif u8_mode:
            cb, check = cpu_baseline(opts.model, model, opts.cpu_seconds)
        else:
            cb, check = cpu_baseline(opts.model, model, opts.cpu_seconds, x_timed=x, y_timed=out)
        result["cpu_baseline"] = cb
        result["gpu_vs_cpu"] = round(value * 1e6 / cb["value"], 1)
        if check is not None:
            result["check"] = check
    del nm, ws, out, x
    return result


TRAIN_PAIRS = 512  # the reference training loop's --batch-size (hardnet/HardNet.py:98)
PEAK_F32 = 157.3   # TFLOP/s, the f32-input MFMA (= the f32 vector peak): the train kernels' exact fp32 products


def cpu_baseline_train(seconds: float = 10.0, pairs: int = TRAIN_PAIRS):
    """The oracle's train step on the host cores (the cgroup quota's thread count): hardnet_train_forward
    of anchors and positives (batch statistics, running-stat update), the oracle loss_hardnet
    (anchor_swap, triplet margin), autograd backward and the reference's SGD step, on a bounded batch of
    ``pairs`` pairs (default: the GPU leg's 512, so the two rates are like for like); patches/s =
    2 pairs / step time (median over the runs)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import hardnet_oracle as O
    torch.manual_seed(0)
    m = HardNet()
    p = {k: v.detach().clone().requires_grad_(k.endswith("weight")) for k, v in m.state_dict().items()}
    run = {k: v for k, v in p.items() if "running" in k}
    opt = torch.optim.SGD([v for k, v in p.items() if v.requires_grad], lr=1.0, momentum=0.9, dampening=0.9,
                          weight_decay=1e-4)
    xa = torch.from_numpy(synth.synth_patches(pairs, seed=21))
    xp = xa + 0.3 * torch.from_numpy(synth.synth_patches(pairs, seed=22))
    quota = _cpu_quota()
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = max(1, int(quota)) if 0 < quota < nproc else nproc
    torch.set_num_threads(threads)

    def step():
        out_a = O.hardnet_train_forward(p, xa, run)
        out_p = O.hardnet_train_forward(p, xp, run)
        loss = O.loss_hardnet(out_a, out_p, anchor_swap=True)
        opt.zero_grad()
        loss.backward()
        opt.step()

    step()
    rates, t_start = [], time.perf_counter()
    while time.perf_counter() - t_start < seconds or len(rates) < 3:
        t0 = time.perf_counter()
        step()
        rates.append(2 * pairs / (time.perf_counter() - t0))
    return {"value": round(statistics.median(rates), 1), "unit": "patches/s", "cores": threads, "kind": "port",
            "model": _cpu_model_string(),
            "sample": f"oracle/hardnet_oracle.py train step (hardnet_train_forward x2 + loss_hardnet + autograd "
                      f"backward + SGD) at {pairs} pairs, {len(rates)} steps over ~{seconds:.0f} s, median"}


def run_train(opts, dev, with_cpu: bool):
    """The reference training loop's step (hardnet/HardNet.py:379-441) on the HIP train path: model.train()
    forward of anchors and of positives (two calls, batch statistics), loss_HardNet (anchor_swap, triplet
    margin, batch_reduce min: the fused hn_loss.hip kernels), backward, SGD (lr 1, momentum 0.9, dampening
    0.9, weight decay 1e-4: create_optimizer, :492-504), at the reference's batch of 512 pairs."""
    from hardnetnas_amd.losses import loss_HardNet
    torch.manual_seed(0)
    m = HardNet().to(dev).train()
    opt = torch.optim.SGD(m.features.parameters(), lr=1.0, momentum=0.9, dampening=0.9, weight_decay=1e-4)
    b = TRAIN_PAIRS
    xa = synth_input_on_device(b, dev, seed=31)
    xp = xa + 0.3 * synth_input_on_device(b, dev, seed=32)
    last = {}

    def step():
        out_a = m(xa)
        out_p = m(xp)
        loss = loss_HardNet(out_a, out_p, anchor_swap=True)
        opt.zero_grad()
        loss.backward()
        opt.step()
        last["loss"] = loss

    steps, warmup = max(10, opts.steps), max(2, opts.warmup)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record()
    for _ in range(steps):
        step()
    ev[1].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms = elapsed / steps * 1e3
    # algorithmic work: forward + data gradient + weight gradient of every conv = 3 x the forward MACs
    flop = 3 * flop_per_patch("hardnet") * 2 * b
    achieved = flop / (ev[0].elapsed_time(ev[1]) / steps * 1e-3) / 1e12
    res = {"value": round(2 * b * steps / elapsed / 1e6, 4), "unit": "Mpatches/s", "ms_per_step": round(ms, 3),
           "steps": steps, "warmup": warmup, "dtype": "f32",
           "config": {"workload": f"Stock HardNet train step (HardNet.py:379-441): 2 x {b} patches, model.train() "
                                  "forward x2, fused loss_HardNet (anchor_swap, triplet margin, min), backward, "
                                  "SGD; orthogonal init (weights_init), synthetic pairs",
                      "model": "hardnet", "global_batch": 2 * b, "pairs": b, "parallelism": "dp1",
                      "precision": "forwards and weight gradients exact fp32 products (f32-input MFMA); stride-1 "
                                   "data gradients bf16x3 (HN_TRAIN_F32=17, the default); fp64 BatchNorm / split-K "
                                   "sums"},
           "loss": float(last["loss"].item()),
           "roofline": {"bound": "mfma", "kernel": "whole train step (forward, backward, BN, loss, SGD)",
                        "achieved": round(achieved, 2), "peak": PEAK_F32, "unit": "TFLOP/s",
                        "frac": round(achieved / PEAK_F32, 4), "traffic": None,
                        "peak_basis": "f32 MFMA 157.3 TFLOP/s (the train kernels' exact fp32 products); "
                                      "algorithmic FLOP = 3 x the forward's 2 x MAC per patch"},
           "cpu_baseline": None}
    if with_cpu:
        cb = cpu_baseline_train()
        res["cpu_baseline"] = cb
        res["gpu_vs_cpu"] = round(res["value"] * 1e6 / cb["value"], 1)
    del m, opt, xa, xp
    return res


SUPERNET_PAIRS = 128  # the supernet search's batch_size (hardnetNAS/supernet_functions/config_for_supernet.py:17)


def _supernet_step(m, opt, crit, xa, xp, lat_dev):
    """training_functions_supernet.py:93-104, one step of _training_step: outs_X with grad, outs_Y under no_grad
    (latency accumulated through both), SupernetLoss (target latency 15, config_for_supernet.py:42), backward,
    the optimizer's step; temperature 5.0 (the initial one, :39)."""
    opt.zero_grad()
    lat0 = torch.zeros(1, 1, device=lat_dev, requires_grad=True)
    ox, lacc, soft, _ = m(xa, 5.0, lat0)
    with torch.no_grad():
        oy, _, _, _ = m(xp, 5.0, lacc)
    loss = crit(ox, oy, lacc, soft, 15.0)[0]
    loss.backward()
    opt.step()
    return loss


def _supernet_setup(dev, pairs):
    from hardnetnas_amd.losses import SupernetLoss
    from hardnetnas_amd.model import HardNetNASSupernet
    torch.manual_seed(0)
    m = HardNetNASSupernet().to(dev).train()
    # the w_optimizer: SGD over the weights (not the thetas), lr 0.01, momentum 0.9, wd 1e-4 (config :22-24)
    opt = torch.optim.SGD([p for n, p in m.named_parameters() if not n.endswith("thetas")], lr=0.01,
                          momentum=0.9, weight_decay=1e-4)
    xa = torch.from_numpy(synth.synth_patches(pairs, seed=61)).to(dev)
    xp = xa + 0.3 * torch.from_numpy(synth.synth_patches(pairs, seed=62)).to(dev)
    return m, opt, SupernetLoss(), xa, xp


def supernet_flop_per_patch() -> int:
    """Forward FLOP (2 x MAC) of one patch through the supernet (every candidate op of every searched layer is
    evaluated and mixed, model_supernet.py:40-50), counted by torch's FlopCounterMode on the module's torch layers
    on the CPU at a batch of 2."""
    from torch.utils.flop_counter import FlopCounterMode
    from hardnetnas_amd.model import HardNetNASSupernet
    m = HardNetNASSupernet().eval()
    x = torch.from_numpy(synth.synth_patches(2, seed=63))
    with torch.no_grad(), FlopCounterMode(display=False) as fc:
        m(x, 5.0, torch.zeros(1, 1))
    return int(fc.get_total_flops()) // 2


def cpu_baseline_supernet(seconds: float = 8.0, pairs: int = SUPERNET_PAIRS):
    """The same supernet search step on the host cores (the cgroup quota's thread count): the module's torch
    layers (the reference's FBNet_Stochastic_SuperNet structure, model_supernet.py:53-85) in fp32 on the CPU,
    at the GPU leg's batch; patches/s = 2 x pairs / step time (median)."""
    quota = _cpu_quota()
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = max(1, int(quota)) if 0 < quota < nproc else nproc
    torch.set_num_threads(threads)
    m, opt, crit, xa, xp = _supernet_setup(torch.device("cpu"), pairs)
    _supernet_step(m, opt, crit, xa, xp, "cpu")
    rates, t_start = [], time.perf_counter()
    while time.perf_counter() - t_start < seconds or len(rates) < 3:
        t0 = time.perf_counter()
        _supernet_step(m, opt, crit, xa, xp, "cpu")
        rates.append(2 * pairs / (time.perf_counter() - t0))
    return {"value": round(statistics.median(rates), 1), "unit": "patches/s", "cores": threads, "kind": "port",
            "model": _cpu_model_string(),
            "sample": f"hardnetnas_amd.HardNetNASSupernet torch layers (fp32, CPU) supernet search step at {pairs} "
                      f"pairs (outs_X + no_grad outs_Y + SupernetLoss + backward + SGD), {len(rates)} steps over "
                      f"~{seconds:.0f} s, median"}


def run_train_supernet(opts, dev, with_cpu: bool):
    """The supernet search step (hardnetNAS/supernet_functions/training_functions_supernet.py:87-104) on the HIP
    NAS train path (NasTrainFunction: the supernet's mixed layers, backward to the weights and the thetas) at the
    reference's batch_size of 128 pairs, with the w_optimizer's SGD."""
    m, opt, crit, xa, xp = _supernet_setup(dev, SUPERNET_PAIRS)
    steps, warmup = max(10, opts.steps), max(2, opts.warmup)
    for _ in range(warmup):
        loss = _supernet_step(m, opt, crit, xa, xp, dev)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record()
    for _ in range(steps):
        loss = _supernet_step(m, opt, crit, xa, xp, dev)
    ev[1].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    b = SUPERNET_PAIRS
    # algorithmic work per step: outs_X forward + its data and weight gradients (3 x F) + outs_Y forward (F)
    flop = 4 * supernet_flop_per_patch() * b
    achieved = flop / (ev[0].elapsed_time(ev[1]) / steps * 1e-3) / 1e12
    res = {"value": round(2 * b * steps / elapsed / 1e6, 4), "unit": "Mpatches/s",
           "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps, "warmup": warmup, "dtype": "f32",
           "config": {"workload": f"hardnetNAS supernet search step (training_functions_supernet.py:93-104): "
                                  f"outs_X = model(X) with grad, outs_Y under no_grad, SupernetLoss (target "
                                  f"latency 15, temperature 5), backward, SGD on the weights; 2 x {b} patches, "
                                  "synthetic pairs",
                      "model": "hardnetnas_supernet", "global_batch": 2 * b, "pairs": b, "parallelism": "dp1"},
           "loss": float(loss.item()),
           "roofline": {"bound": "latency", "kernel": "whole supernet step (every candidate op, backward, loss, SGD)",
                        "achieved": round(achieved, 3), "peak": PEAK_F32, "unit": "TFLOP/s",
                        "frac": round(achieved / PEAK_F32, 4), "traffic": None,
                        "peak_basis": "f32 MFMA 157.3 TFLOP/s; algorithmic FLOP = 4 x the supernet forward's "
                                      "2 x MAC per patch (FlopCounterMode) x 128 pairs"},
           "cpu_baseline": None}
    if with_cpu:
        cb = cpu_baseline_supernet()
        res["cpu_baseline"] = cb
        res["gpu_vs_cpu"] = round(res["value"] * 1e6 / cb["value"], 1)
    del m, opt, xa, xp
    return res


EVAL_BATCH = 512  # the reference eval loop's --test-batch-size (hardnet/HardNet.py:100)


def cpu_baseline_eval(model, seconds: float = 6.0, b: int = EVAL_BATCH):
    """The eval batch on the host cores (the cgroup quota's thread count): the oracle's forward of b anchors
    and b positives and the per-pair distance of HardNet.py:456-458; pairs/s and patches/s (median)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import hardnet_oracle as O
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    xa = torch.from_numpy(synth.synth_patches(b, seed=41))
    xp = xa + 0.3 * torch.from_numpy(synth.synth_patches(b, seed=42))
    quota = _cpu_quota()
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = max(1, int(quota)) if 0 < quota < nproc else nproc
    torch.set_num_threads(threads)

    def batch():
        with torch.no_grad():
            oa, op = O.hardnet_forward(p, xa), O.hardnet_forward(p, xp)
            return torch.sqrt(torch.sum((oa - op) ** 2, 1))

    batch()
    times, t_start = [], time.perf_counter()
    while time.perf_counter() - t_start < seconds or len(times) < 3:
        t0 = time.perf_counter()
        batch()
        times.append(time.perf_counter() - t0)
    t = statistics.median(times)
    return {"value": round(2 * b / t, 1), "unit": "patches/s", "ms_per_batch": round(t * 1e3, 2), "cores": threads,
            "kind": "port", "model": _cpu_model_string(),
            "sample": f"oracle/hardnet_oracle.py hardnet_forward of {b} anchors + {b} positives and the pair "
                      f"distance, {len(times)} batches over ~{seconds:.0f} s, median"}


def run_eval512(opts, dev, with_cpu: bool):
    """The drop-in caller's own batch: the reference eval loop (hardnet/HardNet.py:443-459) runs, per batch,
    ``out_a = model(data_a); out_p = model(data_p)`` under torch.no_grad() at --test-batch-size 512 and
    ``dists = torch.sqrt(torch.sum((out_a - out_p) ** 2, 1))``.  Here the same three lines on the module
    (hardnetnas_amd.HardNet, eval mode: the native op through torch.ops.hardnet_mi355x.forward), over 64
    resident batch pairs in turn (inputs already in HBM; the loader's host->device copy is not timed).
    Reports hipEvent ms per batch (device time, launch stream = torch's current stream), wall ms per batch
    (includes the Python / ctypes / allocator path), caching-allocator allocations and device mallocs per
    batch, and the kernel launches of one 512-patch forward."""
    model = build_model("hardnet").to(dev)
    b, nb = EVAL_BATCH, 64
    g = torch.Generator(device=dev).manual_seed(51)
    xa = synth_input_on_device(b * nb, dev, seed=52).view(nb, b, 1, 32, 32)
    xp = xa + 0.3 * torch.randn(xa.shape, device=dev, generator=g)
    steps, warmup = max(200, 10 * opts.steps), 10
    with torch.no_grad():
        def batch(i):
            out_a = model(xa[i % nb])
            out_p = model(xp[i % nb])
            return torch.sqrt(torch.sum((out_a - out_p) ** 2, 1))
        for i in range(warmup):
            batch(i)
        torch.cuda.synchronize()
        m0 = torch.cuda.memory_stats(dev)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        t0 = time.perf_counter()
        for i in range(steps):
            evs[i][0].record()
            d = batch(i)
            evs[i][1].record()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        m1 = torch.cuda.memory_stats(dev)
        gpu_ms = sorted(e[0].elapsed_time(e[1]) for e in evs)
        # kernel launches and stage times of one 512-patch forward (the library's own hipEvent records)
        nm = NativeModel.from_module(model, dev)
        out = torch.empty((b, 128), device=dev)
        ws = torch.empty(nm.workspace_bytes(b), device=dev, dtype=torch.uint8)
        nm.forward(xa[0], out=out, workspace=ws)
        torch.cuda.synchronize()
        nm.stage_times()
        nm.set_profiling(True)
        nm.forward(xa[0], out=out, workspace=ws)
        torch.cuda.synchronize()
        nm.set_profiling(False)
        st = nm.stage_times()
        ref_d = None
        if with_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            from oracle import hardnet_oracle as O
            p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
            i = (steps - 1) % nb
            ref_d = torch.sqrt(torch.sum((O.hardnet_forward(p, xa[i].cpu()) - O.hardnet_forward(p, xp[i].cpu())) ** 2, 1))
    n_alloc = (m1["allocation.all.allocated"] - m0["allocation.all.allocated"]) / steps
    n_seg = m1["segment.all.allocated"] - m0["segment.all.allocated"]
    res = {"value": round(2 * b * steps / elapsed / 1e6, 4), "unit": "Mpatches/s",
           "ms_per_batch": round(elapsed / steps * 1e3, 4), "steps": steps, "warmup": warmup, "dtype": "bf16x3",
           "gpu_ms_per_batch": {"median": round(gpu_ms[len(gpu_ms) // 2], 4), "min": round(gpu_ms[0], 4),
                                "mean": round(sum(gpu_ms) / steps, 4)},
           "pairs_per_s": round(b * steps / elapsed, 1),
           "config": {"workload": f"reference eval loop batch (HardNet.py:454-458): model(data_a), model(data_p) "
                                  f"on {b}-patch batches under torch.no_grad() through the drop-in module, then "
                                  "the per-pair L2 distance; 64 resident synthetic batch pairs in turn",
                      "model": "hardnet", "batch": b, "parallelism": "dp1"},
           "module_path": {"allocator_allocations_per_batch": n_alloc,
                           "device_mallocs_during_timed_batches": int(n_seg),
                           "workspace_bytes_per_forward": int(nm.workspace_bytes(b)),
                           "kernel_launches_per_forward": int(sum(v[1] for v in st.values())),
                           "stage_ms_per_forward": {k: round(v[0], 4) for k, v in st.items()}},
           "cpu_baseline": None}
    if ref_d is not None:
        res["check"] = {"pairs": b, "max_abs_err_dist_vs_oracle": float((d.cpu() - ref_d).abs().max())}
        cb = cpu_baseline_eval(model)
        res["cpu_baseline"] = cb
        res["gpu_vs_cpu"] = round(res["value"] * 1e6 / cb["value"], 1)
    del model, xa, xp, nm, ws, out
    return res


# the other BASELINE configurations measured after the headline one on a default 1-GPU run
EXTRA_CONFIGS = [("3:wang2", "wang2", None), ("3:wang3", "wang3", None), ("3:wang4", "wang4", None),
                 ("5", "hardnet", 5)]
EXTRA_KEYS = ("value", "unit", "ms_per_step", "steps", "warmup", "dtype", "config", "compute_ms", "pair_step_ms",
              "pairs_per_s", "loss", "roofline", "cpu_baseline", "gpu_vs_cpu", "check")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="hardnet")
    ap.add_argument("--config", type=int, default=None, choices=[2, 3, 4, 5],
                    help="BASELINE config: 2/3/4 = descriptor forward (the default), 5 = HardNet forward "
                         "of 65,536 anchor/positive pairs + the fused distance / hardest-negative / "
                         "margin loss (Losses.py:87-154)")
    ap.add_argument("--batch", type=int, default=None,
                    help="patches per GPU per step (default: 262,144 = BASELINE config 2 at N=1; "
                         "2,097,152 per rank = config 4's 16.7M patches over 8 GPUs when N > 1); "
                         "config 5: pairs per step (default 65,536, split over the ranks)")
    ap.add_argument("--backend", default=None, choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (default nccl = RCCL on GPUs, gloo on CPU)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = plumbing dry run of the same step (module torch layers, gloo): no GPU")
    ap.add_argument("--input", default="f32", choices=["f32", "u8-cv2", "u8-pil", "u8-none"],
                    help="f32: normalised fp32 [B,1,32,32] patches (the reference's model input); u8-*: "
                         "raw uint8 patches (64x64, or 32x32 for u8-none) with the loader's resize / "
                         "ToTensor / Normalize fused into the forward (hn_forward_u8, SURVEY 8(f) row 3)")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="default 1-GPU runs of config 2 also measure configs 3 (wang2/3/4) and 5 after the "
                         "headline line and attach them under 'extra_configs'; this skips them")
    args = ap.parse_args()
    if args.config == 5 and args.model != "hardnet":
        ap.error("config 5 is the stock HardNet pair step")
    if args.input.startswith("u8-") and (args.device != "cuda" or args.config == 5):
        ap.error("--input u8-* is a GPU descriptor-forward mode")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    on_gpu = args.device == "cuda"
    if on_gpu:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
        torch.set_num_threads(max(1, min(4, (os.cpu_count() or 2) // max(world, 1))))
    backend = args.backend or ("nccl" if on_gpu else "gloo")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    result = run(args, world, rank, local, dev, on_gpu, backend)
    extras = (world == 1 and on_gpu and not args.no_extra_configs and args.model == "hardnet"
              and args.config in (None, 2) and args.batch is None and args.input == "f32")
    if extras:
        result["extra_configs"] = {}
        for key, model, cfg in EXTRA_CONFIGS:
            o = argparse.Namespace(**vars(args))
            o.model, o.config, o.batch = model, cfg, None
            o.steps, o.warmup = max(3, args.steps // 2), max(1, args.warmup)
            o.cpu_seconds = min(args.cpu_seconds, 5.0 if cfg is None else 8.0)
            torch.cuda.empty_cache()
            r = run(o, world, rank, local, dev, on_gpu, backend)
            result["extra_configs"][key] = {k: r[k] for k in EXTRA_KEYS if k in r}
        torch.cuda.empty_cache()
        result["extra_configs"]["train"] = run_train(args, dev, with_cpu=not args.no_cpu_baseline)
        torch.cuda.empty_cache()
        result["extra_configs"]["train_supernet"] = run_train_supernet(args, dev, with_cpu=not args.no_cpu_baseline)
        torch.cuda.empty_cache()
        result["extra_configs"]["eval512"] = run_eval512(args, dev, with_cpu=not args.no_cpu_baseline)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
