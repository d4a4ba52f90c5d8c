#!/bin/bash
# tools/pmc_mem_v.sh <outdir> <variant> <config> : memory-pipeline PMC passes for one variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NFCS_VARIANT=$2 PMC_GROUPS="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE;TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum;SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU" \
  bash tools/pmc.sh $1 --config $3 --steps 10 --warmup 2
