#!/bin/bash
# k_irf2 three-workgroups-per-CU form (IRF_BAND / IRF_WPAD): parity, then same-box A/B against abl/OCC3.so
# (the non-persistent two-workgroup form)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "two_block or reference_vectors or candidate or ragged or large_batch or persistent or timed_size or fdl or unfused or skip" > gpurun_out/r03h_pytest.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r03h_pytest.log | head -20; tail -5 gpurun_out/r03h_pytest.log; exit 1; }
tail -1 gpurun_out/r03h_pytest.log
LIBS="new abl/BAND.so" MODELS="wang2 wang4 fdl_NASNet" REPS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-extra-configs" bash tools/ab_lib.sh
