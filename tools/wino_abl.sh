# Winograd conv3/conv5 timing ablations (HN_EXPERIMENTS library; results wrong by design)
export HN_LIB=abl/libhardnet_mi355x.so HN_VARIANT=${HN_VARIANT:-605hfh}
for d in 0 1 2 3 4 8 12 15; do
  HN_DEBUG=$d timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/wabl_$d.log 2>&1 || exit 1
  echo "dbg=$d $(grep '^{' gpurun_out/wabl_$d.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); s=d["roofline"]["stages_ms_per_step"]; print(s["conv3"], s["conv5"])')"
done
