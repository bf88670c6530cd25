#!/bin/bash
# Same-box A/B of the previous commit's library (abl/prev) against the tree's, per model, after the parity suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab9_pytest.log 2>&1 || { tail -30 gpurun_out/ab9_pytest.log; exit 1; }
tail -1 gpurun_out/ab9_pytest.log
for r in 1 2; do
  for m in ${MODELS:-hardnet wang2 wang3}; do
    for lib in abl/prev/libhardnet_mi355x.so -; do
      e=""; [ "$lib" != "-" ] && e="HN_LIB=$lib"
      env $e timeout -k 10 200 python bench.py --no-cpu-baseline --model $m > gpurun_out/ab9_$m.log 2>&1 || { tail -5 gpurun_out/ab9_$m.log; exit 1; }
      python -c "import json;d=json.loads(open('gpurun_out/ab9_$m.log').read().strip().splitlines()[-1]);print('$m [$e]',d['value'],d['roofline']['stages_ms_per_step'])"
    done
  done
done
