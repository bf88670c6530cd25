# k_c12 with P3's a2 tile stored through the LDS staging buffer (in-tree) vs the previous build
# (abl/c12old): HardNet parity first, then same-box bench A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_preprocess.py -m gpu -x -q --timeout 120 --timeout-method thread -k "hardnet or c12 or timed or chunk or u8 or demo or graph" > gpurun_out/c12x_pytest.log 2>&1 || { tail -30 gpurun_out/c12x_pytest.log; exit 1; }
tail -n 1 gpurun_out/c12x_pytest.log
MODELS="hardnet" LIBS="new abl/c12old/libhardnet_mi355x.so" REPS=3 bash tools/ab_lib.sh
