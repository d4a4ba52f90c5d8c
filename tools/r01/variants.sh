#!/bin/bash
# A/B the kernel variants (NFCS_VARIANT) over configs; one JSON line per run.
# usage: tools/variants.sh <outdir> "<variants>" "<configs>" [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; VARS=$2; CFGS=$3; shift 3
mkdir -p "$OUT"
for v in $VARS; do for c in $CFGS; do
  NFCS_VARIANT=$v timeout -k 10 180 python bench.py --config $c --steps 30 --warmup 5 --no-cpu "$@" \
      > "$OUT/b_v${v}_c$c.json" 2> "$OUT/b_v${v}_c$c.err"
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v config $c rc=$rc"; exit $rc; }
  python3 - "$OUT/b_v${v}_c$c.json" "$v" "$c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"v{sys.argv[2]} C{sys.argv[3]} value={d['value']} GB/s kernel_ms={d['roofline']['kernel_ms']} frac={d['roofline']['frac']} parity={d['parity']['match']}")
PY
done; done
