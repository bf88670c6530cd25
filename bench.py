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


def nas_stage_bytes(ops) -> dict:
    """Algorithmic HBM bytes per patch of each NAS stage class, summed over its launches in
    one forward (fp32 NHWC in + out (+ residual read)), mirroring hn_api.hip::forward_nas
    (stem + layer 0 run as one fused "front" kernel unless HN_NO_FRONT=1; IRF layers 1..5 as
    fused "irf" blocks unless HN_NO_IRF=1)."""
    front = os.environ.get("HN_NO_FRONT", "0") in ("", "0")
    irf = os.environ.get("HN_NO_IRF", "0") in ("", "0")
    out = {"stem": 0 if front else 4096 + 32 * 32 * 32 * 4, "front": 0, "irf": 0, "pw": 0,
           "dw": 0, "pwl": 0, "maxpool": 0, "se": 0, "head": 0}
    hw = 32
    for i, (op, (ci, co, s)) in enumerate(zip(A.arch_ops(ops), A.SEARCH_SPACE2)):
        spec = A.OP_SPECS[op]
        ho = hw // s
        fused = front and i == 0
        if spec.kind == "skip":
            if fused:
                out["front"] += 4096 + 4 * ci * ho * ho
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


def cpu_baseline(name: str, model, seconds: float = 12.0):
    """Time the oracle (torch fp32 CPU restatement of the reference forward) on host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import hardnet_oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    b = 1024
    x = torch.from_numpy(synth.synth_patches(b, seed=11))

    def run():
        with torch.no_grad():
            if name == "hardnet":
                O.hardnet_forward(p, x)
            elif name in FDL_MODELS:
                O.fdl_forward(p, FDL_MODELS[name], x)
            else:
                O.nas_forward(p, model.arch_ops, x)

    run()
    run()
    rates, t_start = [], time.perf_counter()
    while time.perf_counter() - t_start < seconds or len(rates) < 3:
        t0 = time.perf_counter()
        run()
        rates.append(b / (time.perf_counter() - t0))
    return {"value": round(statistics.median(rates), 1), "unit": "patches/s", "cores": threads,
            "kind": "port",
            "sample": f"oracle/hardnet_oracle.py {name} fp32 torch-CPU forward, batch {b} x "
                      f"{len(rates)} batches (~{seconds:.0f} s), {threads} threads, median"}


def read_traffic(name: str, stage: str, patches_per_launch: float):
    """PMC-measured HBM bytes per launch of `stage` (profiles/pmc_traffic_<name>.json holds
    bytes per patch from tools/pmc.sh + tools/pmc_traffic.py), or None."""
    f = os.path.join(ROOT, "profiles", f"pmc_traffic_{name}.json")
    if not os.path.exists(f):
        return None
    try:
        e = json.load(open(f)).get(stage)
        return int(e["bytes_per_patch"] * patches_per_launch) if e else None
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="hardnet")
    ap.add_argument("--batch", type=int, default=None,
                    help="patches per GPU per step (default: 262,144 = BASELINE config 2 at N=1; "
                         "2,097,152 per rank = config 4's 16.7M patches over 8 GPUs when N > 1)")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    model = build_model(args.model)
    nm = NativeModel.from_module(model, dev)
    b = args.batch
    if b is None:
        b = CONFIG4_PER_RANK if (world > 1 and args.model == "hardnet") else 262144
    x = synth_input_on_device(b, dev, seed=1000 + rank)
    out = torch.empty((b, 128), device=dev)
    ws = torch.empty(nm.workspace_bytes(b), device=dev, dtype=torch.uint8)
    gathered = torch.empty((b * world, 128), device=dev) if world > 1 else None

    def step():
        nm.forward(x, out=out, workspace=ws)
        if world > 1 and not args.no_allgather:
            dist.all_gather_into_tensor(gathered, out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    nm.stage_times()  # clear
    nm.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    nm.set_profiling(False)
    stages = nm.stage_times()
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    total = b * world * args.steps
    value = total / elapsed / 1e6
    result = None
    if rank == 0:
        # dominant kernel = stage with the largest summed device time
        dom = max(stages, key=lambda k: stages[k][0])
        dom_ms, dom_n = stages[dom]
        avg_ms = dom_ms / max(dom_n, 1)
        launches_per_step = dom_n / args.steps
        patches_per_launch = b / launches_per_step
        if args.model == "hardnet":
            flop = 2 * HARDNET_STAGE_MAC[dom] * patches_per_launch
            bound, peak = "mfma", PEAK_BF16X3
            achieved = flop / (avg_ms * 1e-3) / 1e12
            unit = "TFLOP/s"
            alg = HARDNET_STAGE_BYTES[dom] * patches_per_launch
        else:
            # NAS: HBM-bound fp32 kernels; a stage class aggregates its launches (e.g. every
            # pw of the 6 blocks), so use its summed algorithmic bytes / summed device time
            per_patch = (fdl_stage_bytes(args.model) if args.model in FDL_MODELS
                         else nas_stage_bytes(args.model)).get(dom, 0)
            alg = per_patch * b / launches_per_step
            bound, peak, unit = "hbm", PEAK_HBM, "GB/s"
            achieved = per_patch * b * args.steps / (dom_ms * 1e-3) / 1e9
        traffic = read_traffic(args.model, dom, b / launches_per_step)
        roof = {"bound": bound, "kernel": dom,
                "achieved": round(achieved, 2) if achieved is not None else None,
                "peak": round(peak, 1), "unit": unit,
                "frac": round(achieved / peak, 4) if achieved is not None else None,
                "traffic": traffic,
                "avg_launch_ms": round(avg_ms, 4), "launches": dom_n,
                "patches_per_launch": int(patches_per_launch),
                "algorithmic_bytes_per_launch": int(alg) if alg else None,
                "peak_basis": ("bf16 MFMA dense 2.5 PFLOP/s / 3 (bf16x3 split-precision fp32 "
                               "products); algorithmic fp32 FLOP = 2*MAC") if bound == "mfma"
                else "HBM3E 8 TB/s",
                "stages_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in stages.items()}}
        result = {
            "metric": METRIC, "value": round(value, 4), "unit": "Mpatches/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": ("Stock HardNet forward" if args.model == "hardnet"
                                    else f"FDLNet HardNetNeiMask {FDL_MODELS[args.model]} forward"
                                    if args.model in FDL_MODELS
                                    else f"hardnetNAS {args.model} forward")
                       + f", {b} synthetic 32x32 patches per GPU"
                       + (" (BASELINE config 4 per-rank shard)" if world > 1 and b == CONFIG4_PER_RANK else "")
                       + (", RCCL all-gather of descriptors" if world > 1 and not args.no_allgather else ""),
                       "model": args.model, "global_batch": b * world, "per_gpu_batch": b,
                       "parallelism": f"dp{world}",
                       "precision": "bf16x3 split-precision MFMA, fp32 accumulate" if args.model == "hardnet"
                       else "fp16x3 split-precision MFMA for 1x1 convs and head, fp32 VALU depthwise"
                       + (" and front" if args.model in FDL_MODELS else ""),
                       "flop_per_patch": flop_per_patch(args.model)},
            "roofline": roof,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args.model, model, args.cpu_seconds)
            cb = result["cpu_baseline"]["value"]
            result["gpu_vs_cpu"] = round(value * 1e6 / cb, 1)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
