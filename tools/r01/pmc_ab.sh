#!/bin/bash
# PMC A/B of kernel variants on one config: tools/pmc_ab.sh <outdir> <config> "<variants>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; CFG=$2; VARS=$3
for v in $VARS; do
  NFCS_VARIANT=$v PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD" \
    bash tools/pmc.sh $OUT/v$v --config $CFG --steps 10 --warmup 2 || exit $?
done
