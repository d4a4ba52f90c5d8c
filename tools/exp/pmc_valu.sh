# VALU / SALU instructions per wave of the read pass: the update and the fused forward on C3.
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${1:-pmc_valu}; mkdir -p $O
export TMPDIR=/tmp
for op in update l3fwd; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM --kernel-trace --output-format csv -d "$PWD/$O/$op" -o p -- \
    python3 bench.py --op $op --config 3 --steps 3 --warmup 1 --warm-seconds 0 --no-cpu --no-fresh > $O/$op.log 2>&1 || exit 1
done
python3 - "$O" <<'PY'
import csv, glob, sys, statistics
from collections import defaultdict
for op in ("update", "l3fwd"):
    f = glob.glob(f"{sys.argv[1]}/{op}/**/*counter_collection.csv", recursive=True)[0]
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        if "update_rows" not in r["Kernel_Name"]: continue
        acc[r["Dispatch_Id"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    per = defaultdict(list)
    for d, c in acc.items():
        w = sum(c["SQ_WAVES"])
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM"):
            per[k].append(sum(c[k]) / w)
    print(op, {k: round(statistics.median(v), 1) for k, v in per.items()})
PY
