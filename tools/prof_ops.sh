#!/bin/bash
# rocprofv3 kernel stats of every bench line except C1 (which tools/gpu_check.sh profiles).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-profops}
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "c2 --config 2" "c3 --config 3" "l3fwd --op l3fwd" "flowkey --op flowkey" "vlan --op vlan"; do
  set -- $spec; name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/$name" -o $name -- \
    python3 bench.py "$@" --steps 20 --warmup 3 --no-cpu > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
done
