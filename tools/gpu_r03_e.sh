#!/bin/bash
# head ring-depth A/B (HN_HEAD 3 = A5/B3, 4 = 4/4, 5 = 5/4, 6 = 4/5)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "head_forms" > gpurun_out/r03e_pytest.log 2>&1 || { tail -20 gpurun_out/r03e_pytest.log; exit 1; }
ENVS="HN_HEAD=4;HN_HEAD=5;HN_HEAD=6;HN_HEAD=3" REPS=2 BENCH_ARGS="--steps 20 --warmup 5" bash tools/ab_bench.sh || exit 1
