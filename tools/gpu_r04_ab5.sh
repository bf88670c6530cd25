#!/bin/bash
# Winograd weight ring depth 8 (digit q) against the default 6 (l): parity, then same-box A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k winograd > gpurun_out/ab5_pytest.log 2>&1 || { tail -30 gpurun_out/ab5_pytest.log; exit 1; }
tail -1 gpurun_out/ab5_pytest.log
REPS=2 ENVS="${ENVS:--;HN_VARIANT=605qiq;HN_VARIANT=605liq;HN_VARIANT=605qil}" bash tools/ab_env.sh
