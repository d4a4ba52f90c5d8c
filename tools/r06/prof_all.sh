#!/bin/bash
# Round-6 evidence on one box (the product at the end of the round): rocprofv3 --kernel-trace --stats (csv)
# of the default bench line (the driver's command, the `more` children profiled alone below) and of each
# line alone, then PMC traffic per call (tools/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE / request
# passes, sub-batch launches counted from the trace), then the device-resident short-burst sweep.
# Output under gpurun_out/<out>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r6prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/$name" -o $name -- \
    python3 bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
}
run default --steps 20 --warmup 5 --no-cpu --no-ops
run c1 --steps 50 --no-cpu --no-replay --no-host --no-c4
run c2 --config 2 --steps 30 --no-cpu --no-replay --no-host --no-c4
run c3 --config 3 --steps 30 --no-cpu --no-replay --no-host --no-c4
run c3packed --config 3 --align 16 --steps 30 --no-cpu --no-replay --no-host --no-c4
run c4shard --packets 4194304 --steps 20 --no-cpu --no-replay --no-host --no-c4
run l3fwd_c1 --op l3fwd --steps 30 --no-cpu
run l3fwd_4m --op l3fwd --packets 4194304 --steps 20 --no-cpu
run l3fwd_c3 --op l3fwd --config 3 --steps 20 --no-cpu
run vlan --op vlan --steps 30 --no-cpu
run flowkey --op flowkey --steps 50 --no-cpu
cp profiles/traffic.json "$OUT/traffic_in.json"
timeout -k 10 900 python3 tools/pmc_traffic.py --out "$PWD/$OUT/pmc" --configs 1 2 3 --merge "$PWD/$OUT/traffic_in.json" \
  > "$OUT/pmc.log" 2>&1 || exit 1
timeout -k 10 600 python3 tools/pmc_traffic.py --out "$PWD/$OUT/pmc" --configs 1 --packets 4194304 \
  --merge "$PWD/$OUT/pmc/traffic.json" >> "$OUT/pmc.log" 2>&1 || exit 1
timeout -k 10 900 python3 tools/pmc_traffic.py --out "$PWD/$OUT/pmc" --configs 1 3 --ops l3fwd \
  --merge "$PWD/$OUT/pmc/traffic.json" >> "$OUT/pmc.log" 2>&1 || exit 1
timeout -k 10 900 python3 tools/pmc_traffic.py --out "$PWD/$OUT/pmc" --configs 1 --ops vlan flowkey \
  --merge "$PWD/$OUT/pmc/traffic.json" >> "$OUT/pmc.log" 2>&1 || exit 1
for n in 1024 4096 16384 65536 262144; do
  timeout -k 10 200 python3 bench.py --packets $n --steps 200 --warmup 20 --no-cpu --no-replay --no-host --no-c4 \
    > "$OUT/burst_dev_$n.json" 2>> "$OUT/burst_dev.err" || exit 1
done
cat "$OUT/pmc.log"
