"""bench.py's multi-rank branch, driven for real on CPU (gloo, world size 2): the barrier +
per-rank timing + max-over-ranks reduction + the descriptor all-gather (BASELINE config 4)
and the sharded pair step (config 5).  The GPU run uses the same code with RCCL."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def test_allgather_branch_world2():
    d = _run(["--batch", "48"])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 96 and d["config"]["parallelism"] == "dp2"
    assert d["compute_ms"] > 0 and d["allgather_ms"] >= 0
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert "all-gather" in d["config"]["workload"]


def test_pair_step_branch_world2():
    d = _run(["--config", "5", "--batch", "40"])
    assert d["ranks_seen"] == 2 and d["config"]["baseline_config"] == 5
    assert d["config"]["global_batch"] == 80 and d["scaling"] == "strong"
    assert d["pair_step_ms"] > 0 and d["loss"] is not None and d["loss"] >= 0
