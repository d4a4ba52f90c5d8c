#!/bin/bash
# Per-wave timelines of the checksum kernel (measurement build): tools/timeline_run.sh <outdir>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-tl}
mkdir -p "$OUT"
export NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so
for a in "1 90" "1 92" "3 91" "3 93" "3 90"; do
  set -- $a
  timeout -k 10 120 python3 tools/wave_timeline.py --config $1 --variant $2 --out "$OUT/c$1_v$2.json" \
    > "$OUT/c$1_v$2.log" 2>&1 || { tail -5 "$OUT/c$1_v$2.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    print(f, d["shader_clock_GHz_est"], d["start_span_us"], d.get("resident_waves_est"))
    for k in ["desc", "first_slot", "all_slots", "to_stores", "store_ack", "life"]:
        print("   ", k, d[k])
PY
