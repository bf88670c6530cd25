#!/bin/bash
# Round-4 kernel candidates: parity of the new forms (1-D Winograd conv3 / conv5, k_c12h, fused train
# loss, FDLNet uint8 fronts), then a same-box A/B of their HN_VARIANT / HN_C12_CFG sets.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pairs.py tests/test_preprocess.py -m gpu -q --timeout 120 --timeout-method thread -k "${PYK:-winograd or fused_train or forward_u8 or c12_variants}" -rf > gpurun_out/r04_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/r04_pytest.log; [ $rc -le 1 ] || exit $rc
REPS=${REPS:-2} ENVS="${ENVS:--;HN_VARIANT=605jij;HN_C12_CFG=13;HN_C12_CFG=13 HN_VARIANT=605jij}" bash tools/ab_env.sh
