#!/bin/bash
# NAS front NF lane permutations (bank conflicts): parity, then same-box A/B against the previous commit's
# library (abl/prev) on wang2 / wang3 / wang4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab6_pytest.log 2>&1 || { tail -30 gpurun_out/ab6_pytest.log; exit 1; }
tail -1 gpurun_out/ab6_pytest.log
for m in ${MODELS:-wang2 wang3 wang4}; do
  MODEL=$m REPS=2 ENVS="HN_LIB=abl/prev/libhardnet_mi355x.so;-" bash tools/ab_env.sh || exit 1
done
