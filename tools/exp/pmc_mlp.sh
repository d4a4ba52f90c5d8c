#!/bin/bash
# Measurement tool (not product): memory-pipeline PMC of the checksum read pass on C3 — the
# product (variant 0) against the two-group LDS-landing kernel (variant 6, 1.5x the packets in
# flight) — and on C1 (variant 0): TA busy, DRAM reads outstanding, VALU. One counter group per
# rocprofv3 run, kernel trace only. Output: gpurun_out/<out>/<work>_v<variant>_g<k>/.
#   bash tools/exp/pmc_mlp.sh <out>; python3 tools/exp/pmc_mlp_summary.py gpurun_out/<out>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=$PWD/gpurun_out/${1:-pmcmlp}
mkdir -p "$OUT"
export TMPDIR=/tmp
PG=("TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
        "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
        "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE")
for spec in "c3 0" "c3 6" "c1 0"; do
  set -- $spec
  for k in 0 1 2; do
    d="$OUT/${1}_v${2}_g$k"
    timeout -s KILL 150 rocprofv3 --pmc ${PG[$k]} --kernel-trace --output-format csv -d "$d" -o p -- \
        python3 tools/exp/ab.py --variants $2 --work $1 --iters 5 > "$d.log" 2>&1
    rc=$?; echo "$1 v$2 group $k rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
