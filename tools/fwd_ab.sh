#!/bin/bash
# L3-forward ablations (measurement build): tools/fwd_ab.sh <outdir> "<variants>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
for rep in 1 2; do
  for v in $2; do
    NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so NFCS_VARIANT=$v timeout -k 10 200 \
      python bench.py --op l3fwd --steps 20 --warmup 3 --no-cpu > "$OUT/v${v}_$rep.json" 2> "$OUT/v${v}_$rep.err" || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], r['frac'], r['kernel_ms'], d['parity']['match'])" "$OUT/v${v}_$rep.json" "v$v"
  done
done
