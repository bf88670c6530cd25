# A/B: the 4x4 128-channel k_irf at two waves per SIMD (202 VGPRs, no spill; abl/irf128) vs the
# in-tree three-wave form (168 VGPRs, 27 spilled), after the NAS parity tests on the variant
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
HN_LIB=$PWD/abl/irf128/libhardnet_mi355x.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "(wang or cov or candidate) and not demo" > gpurun_out/irf128_pytest.log 2>&1 || { tail -30 gpurun_out/irf128_pytest.log; exit 1; }
tail -n 1 gpurun_out/irf128_pytest.log
MODELS="wang4" LIBS="new abl/irf128/libhardnet_mi355x.so" REPS=3 bash tools/ab_lib.sh
