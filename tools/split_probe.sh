#!/bin/bash
# Per-kernel durations (rocprofv3 --kernel-trace --stats) of store forms on the C4 shard
# (4M x 1500 B, 6.3 GB) and on C1: where does split mode's time go?
# usage: tools/split_probe.sh <outdir> "<variants>" [packets]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; VARS=$2; PK=${3:-4194304}
mkdir -p "$OUT"
export TMPDIR=/tmp NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so
for v in $VARS; do
  export NFCS_VARIANT=$v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/v$v" -o p -- \
    python3 bench.py --packets "$PK" --steps 20 --warmup 3 --no-cpu > "$OUT/b_v$v.json" 2> "$OUT/b_v$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; tail -5 "$OUT/b_v$v.err"; exit $rc; }
  python3 - "$OUT/b_v$v.json" "$v" "$OUT/v$v/p_kernel_stats.csv" <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"v{sys.argv[2]} value={d['value']} kernel_ms={d['roofline']['kernel_ms']} frac={d['roofline']['frac']} parity={d['parity']['match']}")
for r in csv.DictReader(open(sys.argv[3])):
    if "gen_config" in r["Name"] or "digest" in r["Name"] or "fill" in r["Name"]:
        continue
    print(f"   {r['Name'][:70]:70s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1e3:.1f}")
PY
done
