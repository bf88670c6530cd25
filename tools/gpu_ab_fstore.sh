# NAS front: whole-row stores after a DPP row rotation (in-tree) vs the half-row stores
# (abl/halves, -DHN_FRONT_STORE_HALVES): parity of the fronts first, then same-box bench A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_preprocess.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wang or cov or front or candidate or u8 or nas" > gpurun_out/fstore_pytest.log 2>&1 || { tail -30 gpurun_out/fstore_pytest.log; exit 1; }
tail -n 1 gpurun_out/fstore_pytest.log
MODELS="wang2 wang3" LIBS="new abl/halves/libhardnet_mi355x.so" REPS=2 bash tools/ab_lib.sh || exit 1
BENCH_ARGS="--input u8-cv2" MODELS="wang3" LIBS="new abl/halves/libhardnet_mi355x.so" REPS=1 bash tools/ab_lib.sh
