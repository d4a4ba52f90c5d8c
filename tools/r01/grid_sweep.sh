#!/bin/bash
# Waves looping over several groups of packets (grid-stride, descriptors prefetched one
# iteration ahead): tools/grid_sweep.sh <outdir> (measurement build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
export NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so
for spec in "76 0 3" "76 524288 3" "76 262144 3" "76 131072 3" "75 0 1" "75 32768 1" "75 16384 1" "75 8192 1"; do
  set -- $spec
  NFCS_VARIANT=$1 NFCS_GRID=$2 timeout -k 10 180 python bench.py --config $3 --steps 30 --warmup 5 --no-cpu \
      > "$OUT/g_v$1_g$2_c$3.json" 2> "$OUT/g_v$1_g$2_c$3.err" || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], r['frac'], r['kernel_ms'], d['parity']['match'])" "$OUT/g_v$1_g$2_c$3.json" "v$1 grid=$2 C$3"
done
