#!/bin/bash
# Winograd conv3 / conv5 with the outputs stored by the producer waves (digit r = ring 6 + PST): parity, A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k winograd > gpurun_out/ab9_pytest.log 2>&1 || { tail -30 gpurun_out/ab9_pytest.log; exit 1; }
tail -1 gpurun_out/ab9_pytest.log
REPS=2 ENVS="${ENVS:--;HN_VARIANT=605rir;HN_VARIANT=605qir;HN_VARIANT=605ril}" bash tools/ab_env.sh
