# k5 NAS front with the paired stem rows (HN_FRONT_K5 bit 2): wang3 + coverage-arch parity under
# each form, then a same-box bench A/B (ENVS overrides the set)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${K5S:-4 5 6 7}; do
  HN_FRONT_K5=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wang3 or cov" > gpurun_out/k5_pytest_$v.log 2>&1 || { tail -30 gpurun_out/k5_pytest_$v.log; exit 1; }
  echo "k5=$v $(tail -1 gpurun_out/k5_pytest_$v.log)"
done
ENVS="${ENVS:--;HN_FRONT_K5=5;HN_FRONT_K5=6;HN_FRONT_K5=7}" MODEL=wang3 REPS=2 bash tools/ab_env.sh
