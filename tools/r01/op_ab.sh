#!/bin/bash
# Variant A/B of one bench op (measurement build): tools/op_ab.sh <outdir> <op> "<variants>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; OP=$2
mkdir -p "$OUT"
for rep in 1 2; do
  for v in $3; do
    NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so NFCS_VARIANT=$v timeout -k 10 200 \
      python bench.py --op $OP --steps 20 --warmup 3 --no-cpu > "$OUT/${OP}_v${v}_$rep.json" 2> "$OUT/${OP}_v${v}_$rep.err" || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], r['frac'], r['kernel_ms'], d['parity']['match'])" "$OUT/${OP}_v${v}_$rep.json" "$OP v$v"
  done
done
