#!/bin/bash
# HardNet: sweep HN_SUBCHUNK (conv stages per sub-chunk, head per chunk)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for c in ${SUBS:-2048 4096 8192 32768}; do
  HN_SUBCHUNK=$c timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/sub_$c.log 2>&1 || exit 1
  echo "sub=$c $(tail -1 gpurun_out/sub_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["stages_ms_per_step"])')"
done
