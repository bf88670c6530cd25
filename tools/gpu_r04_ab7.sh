#!/bin/bash
# k3 NAS front in the channel-group dw form (HN_FRONT_XCH3=1, two workgroups per CU) against the default
# three-workgroup form: NAS parity with the knob set, then same-box A/B on wang2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
HN_FRONT_XCH3=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "nas or front or wang or fdl" > gpurun_out/ab7_pytest.log 2>&1 || { tail -30 gpurun_out/ab7_pytest.log; exit 1; }
tail -1 gpurun_out/ab7_pytest.log
MODEL=wang2 REPS=3 ENVS="-;HN_FRONT_XCH3=1" bash tools/ab_env.sh
