#!/bin/bash
# Memory-pipeline PMC passes on the default kernel for configs C1 and C3 (one counter group per
# rocprofv3 run, kernel trace only): tools/pmc_mem.sh <outdir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1
for c in 1 3; do
  PMC_GROUPS="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY;TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum;TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum;TCC_HIT_sum TCC_MISS_sum TCC_BUSY_sum;TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum;SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU" \
    bash tools/pmc.sh $OUT/c$c --config $c --steps 10 --warmup 2 || exit $?
done
