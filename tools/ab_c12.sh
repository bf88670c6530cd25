# A/B of k_c12 configurations (HN_C12_CFG) on one box: parity first, then bench.py per config
# (REPS alternations, to see the box's drift).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c12 or hardnet" > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pytest.log
for r in $(seq ${REPS:-1}); do
for c in ${CFGS:-0 2}; do HN_C12_CFG=$c timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_b$c.log 2>&1 || exit 1; python -c "import json;d=json.loads(open('gpurun_out/ab_b$c.log').read().strip().splitlines()[-1]);print($c,d['value'],d['roofline']['stages_ms_per_step'])"; done
done
