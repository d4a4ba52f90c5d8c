#!/bin/bash
# The round-6 GPU calls, one function per call (the exact command each ran through gpurun, from the repo
# root): `bash tools/r06/calls.sh <letter>`. Their results are in profiles/r06_*; the libraries they name
# are built here by tools/r05/build_lib.sh (git-ignored).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp

# one bench line per (library, spec), alternating within each round, on one box
ab_lines() {  # ab_lines OUTDIR ROUNDS "LIBS" "NAME ARGS" ... (LIB "cur" = the product library)
  local out=$1 rounds=$2 libs=$3; shift 3
  local specs=("$@") r lib spec name args path
  for r in $(seq 1 "$rounds"); do for lib in $libs; do
    path=tools/r06/lib$lib.so; [ "$lib" = cur ] && path=netflow_amd/libnfcs.so
    for spec in "${specs[@]}"; do
      read -r name args <<< "$spec"
      NFCS_LIB=$path timeout -k 10 200 python3 -u bench.py $args --no-cpu --no-host --no-c4 --no-replay --no-mix --no-ops \
        > "$out/${name}_${lib}_$r.json" 2>> "$out/bench.err" || return 1
    done
  done; done
}

call_a() {
  # round 6, GPU call a: packed C3 (16-byte frame starts) on the round-5 product, beside C3 at
  # 128-byte starts, alternating on one box; its rocprofv3 kernel stats; PMC traffic and instruction counts
  local o=gpurun_out/r6a; mkdir -p $o
  ab_lines $o 2 "cur" "c3p --config 3 --align 16 --steps 40" "c3 --config 3 --align 128 --steps 40" && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c3p -o p -- \
    python3 bench.py --config 3 --align 16 --steps 20 --no-cpu --no-host --no-c4 --no-replay > $o/prof_c3p.log 2>&1 && \
  PMC_GROUPS="FETCH_SIZE;WRITE_SIZE TCC_EA0_WRREQ_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
    bash tools/pmc.sh r6a/pmc_c3p --config 3 --align 16 --steps 10 --no-host --no-c4 --no-replay
}

"call_$1"
