#!/bin/bash
# Per-kernel profile of MODELS (default "hardnet"): rocprofv3 kernel stats of a short bench, then two PMC groups per
# model -- LDS (bank conflicts, LDS-issue stalls) and wait / VALU / MFMA issue -- at a 65,536-patch batch.
# Outputs gpurun_out/kprof_<model>/ and gpurun_out/kprof_pmc_<model>/.  (Was tools/gpu_r04_{hn,nas}prof.sh.)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
printf 'SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE\nSQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE\n' > /tmp/kprof_groups.txt
for m in ${MODELS:-hardnet}; do
  rm -rf gpurun_out/kprof_$m
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof_$m -o run --output-format csv -- python bench.py --no-cpu-baseline --model $m --steps 3 --warmup 1 > gpurun_out/kprof_$m.log 2>&1 || { tail -20 gpurun_out/kprof_$m.log; exit 1; }
  python tools/top_kernels.py "$(find gpurun_out/kprof_$m -name '*kernel_stats.csv' | head -1)" 6
  MODEL=$m PMC_GROUPS=/tmp/kprof_groups.txt PMC_BATCH=65536 bash tools/pmc.sh > gpurun_out/kprof_pmc_$m.log 2>&1 || { tail -20 gpurun_out/kprof_pmc_$m.log; exit 1; }
  rm -rf gpurun_out/kprof_pmc_$m; mv gpurun_out/pmc gpurun_out/kprof_pmc_$m
done
echo done
