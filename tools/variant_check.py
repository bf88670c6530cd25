"""Max-abs difference of HardNet forwards under HN_VARIANT strings against the default tiling, on
the library HN_LIB names (the experiments library included): python tools/variant_check.py V1 V2 ..."""
import os
import sys

import numpy as np
import torch

_root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [_root, os.path.join(_root, "tests")]
from fixtures import build_module, golden_inputs  # noqa: E402
from hardnetnas_amd._native import NativeModel  # noqa: E402

m, fx, _ = build_module("hardnet")
x = torch.from_numpy(golden_inputs(fx)).cuda()
os.environ.pop("HN_VARIANT", None)
ref = NativeModel.from_module(m, "cuda")(x).cpu().numpy()
print("default vs reference vectors", float(np.abs(ref - fx["y"]).max()))
for v in sys.argv[1:]:
    os.environ["HN_VARIANT"] = v
    y = NativeModel.from_module(m, "cuda")(x[:255]).cpu().numpy()
    print(v, "max abs vs default", float(np.abs(y - ref[:255]).max()), "vs reference", float(np.abs(y - fx["y"][:255]).max()))
