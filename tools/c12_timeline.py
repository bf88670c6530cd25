"""k_c12 phase timeline from the HN_C12_ABL=64 timing build (s_memtime stamps per wave at the
band phase boundaries of each workgroup's third patch).  Prints the median cycles per phase.
usage (MI355X): python tools/c12_timeline.py"""
import os
import sys

os.environ["HN_C12_ABL"] = os.environ.get("HN_C12_ABL", "64")
os.environ.setdefault("HN_C12_CFG", "12")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from hardnetnas_amd._native import NativeModel  # noqa: E402

P = 16384  # one sub-chunk = one k_c12 launch
dev = torch.device("cuda:0")
nm = NativeModel.from_module(bench.build_model("hardnet"), dev)
x = bench.synth_input_on_device(P, dev, 5)
nwg, nw = 512, 4
if os.environ["HN_C12_CFG"] == "15":
    nwg, nw = 256, 8  # k_c12s: one 8-wave workgroup per CU
ws = torch.zeros(nm.workspace_bytes(P) + nwg * nw * 1024, dtype=torch.uint8, device=dev)
out = torch.empty((P, 128), device=dev)
for _ in range(2):
    nm.forward(x, out=out, workspace=ws)
torch.cuda.synchronize()
# the sub-chunked workspace: [a3: P x 16384][a2: P x 16384][a5: P x 8192] floats; k_c12's output is
# a2, and the stamps go past a5 (out + P * 24576 floats)
off = (16384 * P + 24576 * P) * 4
raw = ws[off: off + nwg * nw * 128 * 8].view(torch.int64).cpu().numpy().reshape(nwg, nw, 128)
if nw == 8:  # k_c12s: per step, A-waves (start, P2 end, past the barrier), B-waves (start, flush, P3, P1, norm, barrier)
    t = raw[:, :, :48].reshape(nwg, nw, 8, 6).astype(np.float64)
    ok = (t[:, :4, :, :3] > 0).all(axis=(1, 2, 3)) & (t[:, 4:] > 0).all(axis=(1, 2, 3))
    t = t[ok]
    a, b = t[:, :4], t[:, 4:]
    step = np.median(b[:, :, 1:, 0] - b[:, :, :-1, 0])
    print(f"{ok.sum()} workgroups; median cycles per step: {step:.0f}")
    rt = raw[:, :, 120:122].astype(np.float64) / 100.0  # 100 MHz -> microseconds
    st0, en = rt[..., 0].min(axis=1), rt[..., 1].max(axis=1)  # per workgroup
    t0 = st0.min()
    print(f"  workgroup start: {np.percentile(st0 - t0, 50):.1f} / max {np.max(st0 - t0):.1f} us after the first;"
          f" end: min {np.min(en - t0):.1f}, median {np.median(en - t0):.1f}, max {np.max(en - t0):.1f} us")
    da = np.diff(a[..., :3], axis=3)
    print(f"  A: P2 {np.median(da[..., 0]):.0f}  barrier wait {np.median(da[..., 1]):.0f}")
    db = np.diff(b, axis=3)
    for i, n in enumerate(["flush", "P3", "P1", "norm", "barrier wait"]):
        print(f"  B: {n:14s} {np.median(db[..., i]):8.0f}  (p90 {np.percentile(db[..., i], 90):8.0f})")
    sys.exit(0)
t = raw[:, :, :48].reshape(nwg, nw, 8, 6).astype(np.float64)
ok = (t > 0).all(axis=(1, 2, 3))
t = t[ok]
names = ["P1", "barrier 1", "P2 (+epilogue)", "conv2 frag loads + barrier 2", "P3 (+stores)"]
d = np.diff(t, axis=3)                           # [wg, wave, band, 5]
nxt = t[:, :, 1:, 0] - t[:, :, :-1, 5]           # P3 end -> next band start
print(f"{ok.sum()} workgroups; median cycles per band per wave (s_memtime):")
for i, n in enumerate(names):
    print(f"  {n:32s} {np.median(d[..., i]):8.0f}   (p90 {np.percentile(d[..., i], 90):8.0f})")
print(f"  {'band end -> next band':32s} {np.median(nxt):8.0f}")
band = t[:, :, 1:, 0] - t[:, :, :-1, 0]
print(f"  {'band total':32s} {np.median(band):8.0f}")
print("per band index (median over workgroups, wave 0):")
for b in range(8):
    print("  band", b, " ".join(f"{np.median(d[:, 0, b, i]):7.0f}" for i in range(5)))

if os.environ["HN_C12_ABL"] == "192":  # P1 sub-stamps: band start, a, b, c, P1 end
    raw2 = ws[off: off + nwg * nw * 128 * 8].view(torch.int64).cpu().numpy().reshape(nwg, nw, 128)
    sub = raw2[:, :, 48:80].reshape(nwg, nw, 8, 4)[ok][:, :, 1:, :3].astype(np.float64)
    t0 = t[:, :, 1:, 0]
    marks = np.concatenate([t0[..., None], sub], axis=3)
    dd = np.diff(marks, axis=3)
    for i, n in enumerate(["P1 operands read + split", "P1 MFMA chain", "P1 epilogue + stores"]):
        print(f"  {n:32s} {np.median(dd[..., i]):8.0f}")
