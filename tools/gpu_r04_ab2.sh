#!/bin/bash
# Round-4 check + Winograd ablations: the full GPU suite / smoke / default bench (final_check STEP=tests),
# then same-box A/B: default (605jij), conv5 weight ring 4 (605jik), and the timing-only ablations of the
# Winograd kernels from the experiments library (m idle producers, n no MFMAs, o no weight loads, p no stores).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEP=tests bash tools/final_check.sh || exit 1
L=abl/libhardnet_mi355x.so
REPS=${REPS:-1} ENVS="${ENVS:--;HN_VARIANT=605jik;HN_LIB=$L HN_VARIANT=605mim;HN_LIB=$L HN_VARIANT=605nin;HN_LIB=$L HN_VARIANT=605oio;HN_LIB=$L HN_VARIANT=605pip;-}" bash tools/ab_env.sh
