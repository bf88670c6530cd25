cd "${GRAFT_REPO_ROOT:-/root/repo}"
for c in 2048 4096 8192 16384 32768 65536; do
  HN_CHUNK=$c timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/chunk_$c.log 2>&1 || exit 1
  echo "chunk=$c $(tail -1 gpurun_out/chunk_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["stages_ms_per_step"])')"
done
