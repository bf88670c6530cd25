#!/bin/bash
# End-of-round evidence. STEP=tests: full GPU suite, smoke, default bench (the driver's command);
# STEP=prof: rocprofv3 kernel stats of the default bench and the PMC passes for MODELS (bench.py's roofline inputs)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${STEP:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_pytest.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/final_pytest.log | head -20; tail -5 gpurun_out/final_pytest.log; exit 1; }
  tail -1 gpurun_out/final_pytest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
  tail -1 gpurun_out/final_smoke.log
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench.log 2>&1 || { tail -5 gpurun_out/final_bench.log; exit 1; }
  grep '^{' gpurun_out/final_bench.log | tail -1 > gpurun_out/final_bench.json
  python -c "import json;d=json.load(open('gpurun_out/final_bench.json'));print(d['value'],d['ms_per_step'],{k:(v.get('value'),v.get('ms_per_step')) for k,v in d.get('extra_configs',{}).items()} if isinstance(d.get('extra_configs'),dict) else list(d.keys()))"
else
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/final_prof.log 2>&1 || { tail -5 gpurun_out/final_prof.log; exit 1; }
  find gpurun_out/final_prof -name "*kernel_stats.csv" | head -3
  MODELS="${MODELS:-hardnet c5}" timeout -k 10 900 bash tools/pmc_all.sh > gpurun_out/final_pmc.log 2>&1; rc=$?; tail -3 gpurun_out/final_pmc.log; exit $rc
fi
