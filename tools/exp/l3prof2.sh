set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${1:-l3prof2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/p" -o l3 -- \
  python3 bench.py --op l3fwd --packets 4194304 --steps 20 --warmup 3 --no-cpu > $O/b.log 2>&1 || exit 1
python3 - "$O/p" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
