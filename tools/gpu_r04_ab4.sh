#!/bin/bash
# Weight ring depth 6 by default for the Winograd conv3 / conv5, the IRF pw fragment ring: parity on the
# new tree, then same-box A/B against the session-start library (abl/head) and two conv4 isolation builds
# (abl/ws1: k_conv_ws producers as before the branchless loads; abl/ws2: its next-stage weight prefetch
# conditional again).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
H=abl/head/libhardnet_mi355x.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab4_pytest.log 2>&1 || { tail -30 gpurun_out/ab4_pytest.log; exit 1; }
tail -1 gpurun_out/ab4_pytest.log
REPS=2 ENVS="HN_LIB=$H;-" bash tools/ab_env.sh || exit 1
for m in wang2 wang3 wang4; do
  MODEL=$m REPS=2 ENVS="HN_LIB=$H;-" bash tools/ab_env.sh || exit 1
done
