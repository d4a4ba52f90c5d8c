#!/bin/bash
# rocprofv3 kernel stats of tools/exp/ab.py runs: per-kernel average durations by variant.
# usage: tools/exp/prof_ab.sh <outdir> "<variants>" <work> [ab.py args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/$1; VARS=$2; WORK=$3; shift 3
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $VARS; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/v$v" -o p -- \
    python3 tools/exp/ab.py --variants "$v" --work "$WORK" "$@" > "$OUT/ab_v$v.json" 2> "$OUT/ab_v$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; tail -5 "$OUT/ab_v$v.err"; exit $rc; }
  cat "$OUT/ab_v$v.json"
  python3 - "$OUT/v$v/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("gen_config", "digest", "fill", "copyBuffer")):
        continue
    print(f"   {r['Name'][:90]:90s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1e3:.1f}")
PY
done
