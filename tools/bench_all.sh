#!/bin/bash
# All bench lines on one GPU: tools/bench_all.sh <outdir> [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  local rc=$?
  python3 - "$OUT/bench_$name.json" "$name" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"{sys.argv[2]:8s} value={d['value']} {d['unit']} ms/step={d['ms_per_step']} kernel_ms={r['kernel_ms']} frac={r['frac']} parity={d['parity']['match']} cpu={(d.get('cpu_baseline') or {}).get('value')}")
except Exception as e:
    print(sys.argv[2], "no result", e)
PY
  return $rc
}
run c1 --config 1 "$@" && run c2 --config 2 "$@" && run c3 --config 3 "$@" && \
run l3fwd --op l3fwd "$@" && run flowkey --op flowkey "$@" && run vlan --op vlan "$@"
