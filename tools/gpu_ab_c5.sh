#!/bin/bash
# same-box A/B of the config-5 pair step over LIBS (default "new abl/base.so")
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  for lib in ${LIBS:-new abl/base.so}; do
    if [ $lib = new ]; then unset HN_LIB; else export HN_LIB=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra-configs --config 5 --steps 20 --warmup 5 > gpurun_out/ab_c5.log 2>&1 || { tail -5 gpurun_out/ab_c5.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_c5.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$lib', d['value'], d.get('pair_step_ms'), r.get('frac'))"
  done
done
