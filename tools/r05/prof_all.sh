#!/bin/bash
# Round-5 evidence on one box (the product at the end of the round): rocprofv3 --kernel-trace --stats (csv)
# of the default bench line (the driver's command) and of each line alone, then PMC traffic per call
# (tools/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE / request passes; sub-batch launches counted
# from the trace). Output under gpurun_out/<out>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-r5prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/$name" -o $name -- \
    python3 bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
}
run default --steps 20 --warmup 5 --no-cpu --no-ops  # the `more` child lines are profiled alone below
run c1 --steps 50 --no-cpu --no-replay --no-host --no-c4
run c2 --config 2 --steps 30 --no-cpu --no-replay --no-host --no-c4
run c3 --config 3 --steps 30 --no-cpu --no-replay --no-host --no-c4
run c4shard --packets 4194304 --steps 20 --no-cpu --no-replay --no-host --no-c4
run l3fwd_c1 --op l3fwd --steps 30 --no-cpu
run l3fwd_4m --op l3fwd --packets 4194304 --steps 20 --no-cpu
run l3fwd_c3 --op l3fwd --config 3 --steps 20 --no-cpu
run vlan --op vlan --steps 30 --no-cpu
run flowkey --op flowkey --steps 50 --no-cpu
timeout -k 10 900 python3 tools/pmc_traffic.py --out "$PWD/$OUT/pmc" --configs 1 2 3 > "$OUT/pmc.log" 2>&1 || exit 1
timeout -k 10 600 python3 tools/pmc_traffic.py --out "$PWD/$OUT/pmc" --configs 1 --packets 4194304 \
  --merge "$PWD/$OUT/pmc/traffic.json" >> "$OUT/pmc.log" 2>&1 || exit 1
timeout -k 10 900 python3 tools/pmc_traffic.py --out "$PWD/$OUT/pmc" --configs 1 3 --ops l3fwd \
  --merge "$PWD/$OUT/pmc/traffic.json" >> "$OUT/pmc.log" 2>&1 || exit 1
timeout -k 10 900 python3 tools/pmc_traffic.py --out "$PWD/$OUT/pmc" --configs 1 --ops vlan flowkey \
  --merge "$PWD/$OUT/pmc/traffic.json" >> "$OUT/pmc.log" 2>&1 || exit 1
cat "$OUT/pmc.log"
