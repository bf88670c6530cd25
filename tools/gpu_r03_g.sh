#!/bin/bash
# pair kernel with -fno-honor-nans (no canonicalising max before every fminf): parity, then same-box A/B
# against abl/base.so (the previous build), and the wang2 / wang4 kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pairs.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03g_pytest.log 2>&1 || { tail -20 gpurun_out/r03g_pytest.log; exit 1; }
tail -1 gpurun_out/r03g_pytest.log
for r in 1 2; do
  for lib in abl/base.so new; do
    if [ $lib = new ]; then unset HN_LIB; else export HN_LIB=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra-configs --config 5 --steps 20 --warmup 5 > gpurun_out/ab_c5.log 2>&1 || { tail -5 gpurun_out/ab_c5.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_c5.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$lib', d['value'], d.get('pair_step_ms'), r.get('avg_launch_ms'), r.get('frac'))"
  done
done
unset HN_LIB
bash tools/prof_models.sh
