#!/bin/bash
# Winograd operand ring depth 3 (digits r = weight ring 6, s = 4) against the default (q / l): parity + A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k winograd > gpurun_out/ab8_pytest.log 2>&1 || { tail -30 gpurun_out/ab8_pytest.log; exit 1; }
tail -1 gpurun_out/ab8_pytest.log
REPS=2 ENVS="${ENVS:--;HN_VARIANT=605rir;HN_VARIANT=605sis;HN_VARIANT=605ris;HN_VARIANT=605qir}" bash tools/ab_env.sh
