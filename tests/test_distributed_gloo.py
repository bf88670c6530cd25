"""World-size-2 gloo tests of the patch-sharded path (CPU; the GPU run uses RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hardnetnas_amd.distributed import gather_descriptors, shard_range, sharded_forward


def test_shard_range_partitions():
    for n in (0, 1, 7, 8, 1000, 262144 * 8 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (s0, e0), (s1, e1) in zip(spans, spans[1:]):
                assert e0 == s1
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from fixtures import build_module, golden_inputs
        torch.set_num_threads(1)
        m, fx, _ = build_module(name)
        x = torch.from_numpy(golden_inputs(fx)[:n])
        y = sharded_forward(m, x, gather=True)
        # uneven gather path (n not divisible by world)
        local = torch.full((shard_range(5, world, rank)[1] - shard_range(5, world, rank)[0], 3),
                           float(rank))
        g = gather_descriptors(local, 5)
        if rank == 0:
            q.put((y.numpy(), g.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,n", [("hardnet", 64), ("wang2", 37)])
def test_sharded_forward_equals_single_process(name, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    y, g = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from fixtures import build_module, golden_inputs
    m, fx, _ = build_module(name)
    with torch.no_grad():
        ref = m(torch.from_numpy(golden_inputs(fx)[:n])).numpy()
    assert y.shape == (n, 128)
    assert np.abs(y - ref).max() <= 1e-6
    assert np.abs(y - fx["y"][:n]).max() <= 1e-5
    assert g[:, 0].tolist() == [0, 0, 0, 1, 1]


def _loss_worker(rank, world, port, n, swap, loss_type, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hardnetnas_amd.distributed import sharded_hardnet_loss
        g = torch.Generator().manual_seed(5)
        a = torch.nn.functional.normalize(torch.randn(n, 128, generator=g), dim=1)
        p = torch.nn.functional.normalize(a + 0.4 * torch.randn(n, 128, generator=g), dim=1)
        p[3] = a[7]  # a near-duplicate off the diagonal: exercises the < 0.008 mask
        s, e = shard_range(n, world, rank)
        loss, pos, mn = sharded_hardnet_loss(a[s:e], p[s:e], n, anchor_swap=swap, loss_type=loss_type)
        parts = [None] * world
        dist.all_gather_object(parts, (pos, mn))
        if rank == 0:
            q.put((float(loss), torch.cat([x[0] for x in parts]).numpy(),
                   torch.cat([x[1] for x in parts]).numpy(), a.numpy(), p.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,swap,loss_type", [(2, 64, True, "triplet_margin"),
                                                    (2, 37, False, "softmax"),
                                                    (3, 50, True, "contrastive")])
def test_sharded_hardnet_loss_equals_reference(world, n, swap, loss_type):
    """Config 5 at scale on gloo: row blocks + all-reduce(MIN) of the column minima + summed
    partial losses == loss_HardNet on the whole batch (oracle restatement of Losses.py:87-154)."""
    from oracle import hardnet_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loss_worker, args=(r, world, port, n, swap, loss_type, q))
             for r in range(world)]
    for p in procs:
        p.start()
    loss, pos, mn, a, pp = q.get(timeout=300)
    pos, mn, a, pp = (torch.from_numpy(v) for v in (pos, mn, a, pp))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rpos, rmn = O.hardest_negative(a.double(), pp.double(), swap)
    ref = O.loss_hardnet(a.double(), pp.double(), swap, loss_type=loss_type).item()
    assert (pos.double() - rpos).abs().max().item() < 1e-5
    assert (mn.double() - rmn).abs().max().item() < 1e-5
    assert abs(loss - ref) < 1e-5
