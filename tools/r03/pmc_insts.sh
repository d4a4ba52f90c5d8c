#!/bin/bash
# Round 3: instructions per wave and per packet (rocprofv3 SQ counters, one pass each) of the
# checksum read pass and the fused forward on the C3 mix, and of the flow keys on C1.
set -o pipefail
out=gpurun_out/${1:-r03_pmc_insts}
mkdir -p $out
export TMPDIR=/tmp
for w in "update:--config 3:update_rows" "l3fwd:--op l3fwd --config 3:update_rows" "flowkey:--op flowkey:flow_keys"; do
  IFS=: read name args kern <<< "$w"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS --kernel-trace --output-format csv -d "$PWD/$out/$name" -o p -- \
    python3 bench.py $args --steps 3 --warmup 1 --warm-seconds 0 --no-cpu --no-fresh > $out/$name.log 2>&1 || exit 1
done
python3 - "$out" > $out/summary.json <<'PY'
import csv, glob, json, sys, statistics
from collections import defaultdict
res = {}
for name, kern, ppw in (("update", "update_rows", 4), ("l3fwd", "update_rows", 8), ("flowkey", "flow_keys", 64)):
    f = glob.glob(f"{sys.argv[1]}/{name}/**/*counter_collection.csv", recursive=True)[0]
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]: continue
        acc[r["Dispatch_Id"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    per = defaultdict(list)
    for d, c in acc.items():
        w = sum(c["SQ_WAVES"])
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM", "SQ_INSTS_LDS"):
            per[k].append(sum(c[k]) / w)
    res[name] = {"packets_per_wave": ppw, "per_wave": {k: round(statistics.median(v), 1) for k, v in per.items()},
                 "per_packet": {k: round(statistics.median(v) / ppw, 1) for k, v in per.items()}}
print(json.dumps(res, indent=1))
PY
