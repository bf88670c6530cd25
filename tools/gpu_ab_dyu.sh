# A/B: k_irf / k_irf2 depthwise dy loop unrolled (abl/dyu) vs the in-tree rolled loop, after the
# NAS / FDL parity tests on the variant
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
HN_LIB=$PWD/abl/dyu/libhardnet_mi355x.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "(wang or cov or candidate or fdl or irf) and not demo" > gpurun_out/dyu_pytest.log 2>&1 || { tail -30 gpurun_out/dyu_pytest.log; exit 1; }
tail -n 1 gpurun_out/dyu_pytest.log
MODELS="wang2 wang4 wang3 fdl_NASNet" LIBS="new abl/dyu/libhardnet_mi355x.so" REPS=2 bash tools/ab_lib.sh
