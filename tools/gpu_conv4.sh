#!/bin/bash
# conv4 variants: parity, then same-box A/B over RUNS="lib:HN_VARIANT ..." (lib "new" = in-tree)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tiling_variants or producer_stores" > gpurun_out/c4_pytest.log 2>&1 || { tail -30 gpurun_out/c4_pytest.log; exit 1; }
  tail -1 gpurun_out/c4_pytest.log
fi
for r in 1 2; do
  for e in ${RUNS:-new:605gfg new:605gig}; do
    lib=${e%%:*}; v=${e##*:}
    if [ $lib = new ]; then unset HN_LIB; else export HN_LIB=$PWD/abl/$lib.so; fi
    HN_VARIANT=$v timeout -k 10 150 python bench.py --no-cpu-baseline --no-extra-configs --steps 10 --warmup 3 > gpurun_out/c4_$lib$v.log 2>&1 || { tail -5 gpurun_out/c4_$lib$v.log; exit 1; }
    echo "$lib $v $(grep '^{' gpurun_out/c4_$lib$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["roofline"]["stages_ms_per_step"]; print(d["value"], s["conv4"], s["conv3"])')"
  done
done
