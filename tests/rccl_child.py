"""Child process of tests/test_gpu_scale.py::test_rccl_world1_matches_single_calls (not a test module).

Initialises an ``nccl`` (= RCCL on ROCm) process group of world size 1 before anything touches the
GPU, then drives hardnetnas_amd.distributed's two collective paths on HIP tensors -- the
descriptor all-gather of BASELINE config 4 (``sharded_forward``: all_gather_into_tensor) and the
sharded config-5 loss (``sharded_hardnet_loss``: all-gather of the positives, all_reduce(MIN) of
the column minima, all_reduce(SUM) of the loss) -- and checks them bit for bit against the single
calls they reassemble (reference: hardnetNAS/supernet_main_file.py:60, hardnet/Losses.py:87-154).
Prints one line "RCCL_OK ..." and exits 0 on success."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main() -> int:
    import torch
    import torch.distributed as dist
    dist.init_process_group("nccl", init_method="env://", rank=0, world_size=1)
    from fixtures import build_module
    from hardnetnas_amd import _native, distributed as D
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    assert dist.get_backend() == "nccl"

    m, _, _ = build_module("hardnet")
    m = m.to(dev)
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randint(0, 256, (8192, 1, 32, 32), device=dev, generator=g, dtype=torch.int32).float() / 255.0
    x = (x - 0.443728476019) / 0.20197947209
    with torch.no_grad():
        single = m(x)
    gathered = D.sharded_forward(m, x)  # all_gather_into_tensor over RCCL
    torch.cuda.synchronize()
    assert gathered.is_cuda and gathered.shape == single.shape
    assert torch.equal(gathered, single), "all-gathered descriptors differ from the single call"

    n = 4096
    a, p = single[:n].contiguous(), single[n:].contiguous()
    for swap in (False, True):
        loss, pos, mn = D.sharded_hardnet_loss(a, p, n, anchor_swap=swap)
        pos1, mn1 = _native.pairdist_hardneg(a, p, anchor_swap=swap)
        loss1, _ = _native.hardnet_loss(pos1, mn1)
        torch.cuda.synchronize()
        assert torch.equal(pos, pos1), f"pos differs (anchor_swap={swap})"
        assert torch.equal(mn, mn1), f"min_neg differs (anchor_swap={swap})"
        assert torch.equal(loss, loss1), f"loss differs (anchor_swap={swap}): {loss.item()} vs {loss1.item()}"
        print(f"anchor_swap={swap}: loss {loss.item():.7f}")
    print(f"RCCL_OK backend={dist.get_backend()} rows={single.shape[0]} pairs={n}")
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
