# k5 NAS front variants (HN_FRONT_K5 = 1 dy unrolled, 2 no fold, 3 both): wang3 parity under each,
# then a same-box bench A/B against the production form
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 1 2 3; do
  HN_FRONT_K5=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wang3 or cov" > gpurun_out/k5_pytest_$v.log 2>&1 || { tail -30 gpurun_out/k5_pytest_$v.log; exit 1; }
  echo "k5=$v $(tail -1 gpurun_out/k5_pytest_$v.log)"
done
ENVS="-;HN_FRONT_K5=1;HN_FRONT_K5=2;HN_FRONT_K5=3" MODEL=wang3 REPS=2 bash tools/ab_env.sh
