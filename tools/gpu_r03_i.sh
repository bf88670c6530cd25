#!/bin/bash
# paired stem rows in the k3 front: parity (front / u8 / candidate ops at layer 0), A/B against abl/PRE.so, then the PMC refresh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_preprocess.py -m gpu -q --timeout 120 --timeout-method thread -k "reference_vectors or front or layer0 or forward_u8 or ragged or timed_size or large_batch" > gpurun_out/r03i_pytest.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r03i_pytest.log | head -20; tail -5 gpurun_out/r03i_pytest.log; exit 1; }
tail -1 gpurun_out/r03i_pytest.log
LIBS="new abl/PRE.so" MODELS="wang2" REPS=3 BENCH_ARGS="--steps 20 --warmup 5 --no-extra-configs" bash tools/ab_lib.sh || exit 1
MODELS="${PMC_MODELS:-hardnet wang2 wang3 wang4}" timeout -k 10 900 bash tools/pmc_all.sh > gpurun_out/pmc.log 2>&1; rc=$?; tail -2 gpurun_out/pmc.log; exit $rc
