# A/B: fp16 split with v_fma_mix_f32 (abl/mix/libhardnet_mi355x.so, -DHN_SPLIT_MIX) vs the in-tree library, after the
# NAS parity tests on the variant; then k_head4 (HN_HEAD=4) vs k_head3 after its parity tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
HN_LIB=$PWD/abl/mix/libhardnet_mi355x.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "(nas or wang or candidate or fdl or irf or front) and not head4 and not demo" > gpurun_out/mix_pytest.log 2>&1 || { tail -30 gpurun_out/mix_pytest.log; exit 1; }
tail -1 gpurun_out/mix_pytest.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "head" > gpurun_out/head4_pytest.log 2>&1 || { tail -30 gpurun_out/head4_pytest.log; exit 1; }
tail -1 gpurun_out/head4_pytest.log
MODELS="wang2 wang4" LIBS="new abl/mix/libhardnet_mi355x.so" REPS=2 bash tools/ab_lib.sh || exit 1
ENVS="-;HN_HEAD=4" MODEL=hardnet REPS=2 bash tools/ab_env.sh || exit 1
ENVS="-;HN_HEAD=4" MODEL=wang2 REPS=1 bash tools/ab_env.sh || exit 1
bash tools/gpu_ab_k5.sh
