#!/bin/bash
# HardNet per-kernel PMC: LDS (bank conflicts, LDS-issue stalls) and wait / VALU / MFMA groups.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
printf 'SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE\nSQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE\n' > /tmp/hn_groups.txt
MODEL=hardnet PMC_GROUPS=/tmp/hn_groups.txt PMC_BATCH=65536 bash tools/pmc.sh > gpurun_out/hnprof_pmc.log 2>&1 || { tail -20 gpurun_out/hnprof_pmc.log; exit 1; }
rm -rf gpurun_out/hnprof_pmc; mv gpurun_out/pmc gpurun_out/hnprof_pmc
echo done
