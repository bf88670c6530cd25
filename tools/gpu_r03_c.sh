#!/bin/bash
# round-3 check: k_head3 parity (bit-identical to k_head2) and same-box A/B of the head forms
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -s -v --timeout 120 --timeout-method thread -k "head_forms or reference_vectors or ragged or timed_size or large_batch" > gpurun_out/r03c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r03c_pytest.log | tail -3; [ $rc -eq 0 ] || exit 1
ENVS="-;HN_HEAD=2" REPS=2 BENCH_ARGS="--steps 20 --warmup 5" bash tools/ab_bench.sh || exit 1
ENVS="-;HN_HEAD=2" REPS=2 BENCH_ARGS="--model wang2 --steps 20 --warmup 5" bash tools/ab_bench.sh || exit 1
