#!/bin/bash
# conv4's clock / TLB / cache counters at the two launch-size configurations: the default
# (k_c12 groups and conv sub-chunks of 65,536 patches) against 16,384 / 16,384.  Two --pmc passes per
# configuration (each within the per-block limits), --kernel-trace only; the 262,144-patch step, 1 warmup + 1 step.
# Summary: python tools/pmc_conv4.py gpurun_out/pmc_conv4
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/pmc_conv4; mkdir -p gpurun_out/pmc_conv4
P1="GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_CYCLES TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
P2="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_TAG_STALL_sum SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for cfg in big small; do
  if [ $cfg = small ]; then export HN_C12_GROUP=16384 HN_SUBCHUNK=16384; else unset HN_C12_GROUP HN_SUBCHUNK; fi
  i=0
  for grp in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/pmc_conv4/${cfg}_p$i -o run --output-format csv -- \
      python bench.py --no-cpu-baseline --no-extra-configs --steps 1 --warmup 1 > gpurun_out/pmc_conv4/${cfg}_p$i.log 2>&1 || { tail -5 gpurun_out/pmc_conv4/${cfg}_p$i.log; exit 1; }
  done
done
echo done
