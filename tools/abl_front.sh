#!/bin/bash
# k_front phase ablations on wang2 (HN_FRONT_ABL bits: 1 stem, 2 pw, 4 dw, 8 pwl; 15 = all)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for a in ${ABLS:-0 1 2 4 8 15}; do
  HN_FRONT_ABL=$a timeout -k 10 200 python bench.py --model wang2 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/fabl_$a.log 2>&1 || exit 1
  echo "abl=$a $(tail -1 gpurun_out/fabl_$a.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["stages_ms_per_step"]["front"])')"
done
