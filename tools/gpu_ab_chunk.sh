# k_head5 parity, then same-box A/Bs: HN_HEAD=5 (512-patch head, 131,072-patch chunks) and
# HN_CHUNK=131072 alone against the defaults (k_head4, 65,536-patch chunks)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "head" > gpurun_out/head5_pytest.log 2>&1 || { tail -30 gpurun_out/head5_pytest.log; exit 1; }
tail -n 1 gpurun_out/head5_pytest.log
for m in hardnet wang2; do
  echo "== $m"
  ENVS="-;HN_HEAD=5;HN_CHUNK=131072" MODEL=$m REPS=2 bash tools/ab_env.sh || exit 1
done
for m in wang3 wang4 fdl_NASNet; do
  echo "== $m"
  ENVS="-;HN_CHUNK=131072" MODEL=$m REPS=1 bash tools/ab_env.sh || exit 1
done
