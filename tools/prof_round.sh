#!/bin/bash
# One profiling session: rocprofv3 kernel stats of the default bench line (C1, without the CPU and
# replay legs so the update kernels' average is over the timed rotation only) and of the other lines,
# then the PMC traffic per call (tools/pmc_traffic.py). Output under gpurun_out/<out>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/c1" -o c1 -- \
  python3 bench.py --no-cpu --no-replay --no-host > "$OUT/c1.json" 2> "$OUT/c1.err" || exit 1
bash tools/prof_ops.sh "${1:-prof}/ops" || exit 1
timeout -k 10 900 python3 tools/pmc_traffic.py --out "$PWD/$OUT/pmc" --configs 1 2 3 > "$OUT/pmc.log" 2>&1 || exit 1
timeout -k 10 600 python3 tools/pmc_traffic.py --out "$PWD/$OUT/pmc_ops" --configs 1 --ops l3fwd vlan flowkey \
  --merge "$PWD/$OUT/pmc/traffic.json" >> "$OUT/pmc.log" 2>&1 || exit 1
cat "$OUT/pmc.log"
