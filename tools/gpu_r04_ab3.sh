#!/bin/bash
# Branchless producer loads (buffer loads, unconditional stages) in k_conv_w1 / k_conv_ws and the NAS
# front's loop-invariant operands waited before the patch loop: parity subsets on the new tree, then
# same-box A/B against the HEAD library (abl/head, built from the previous commit).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=abl/libhardnet_mi355x.so
H=abl/head/libhardnet_mi355x.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab3_pytest.log 2>&1 || { tail -30 gpurun_out/ab3_pytest.log; exit 1; }
tail -1 gpurun_out/ab3_pytest.log
REPS=${REPS:-2} ENVS="${ENVS:-HN_LIB=$H;-;HN_VARIANT=605jik;HN_VARIANT=605kik;HN_VARIANT=605kil;HN_VARIANT=605lil}" bash tools/ab_env.sh || exit 1
for m in wang2 wang3; do
  MODEL=$m REPS=2 ENVS="HN_LIB=$H;-" bash tools/ab_env.sh || exit 1
done
