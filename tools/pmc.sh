#!/bin/bash
# PMC counter passes for the checksum kernel (one counter group per rocprofv3 run, kernel-trace
# only, never combined with sys/runtime tracing). Usage: tools/pmc.sh <outdir> <bench args...>
# PMC_GROUPS="A B;C;D E" overrides the default groups (one rocprofv3 pass per group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 137 ] || [ "$1" -eq 139 ]; }
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $group --kernel-trace --output-format csv -d "$OUT/pmc$i" -o p -- \
      python3 bench.py "$@" --no-cpu > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($group) rc=$rc"
  if fatal $rc; then exit $rc; fi
done < <(if [ -n "${PMC_GROUPS:-}" ]; then echo "$PMC_GROUPS" | tr ';' '\n'; else cat <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
GROUPS
fi)
exit 0
