#!/bin/bash
# Round 3: the stream ceiling with the frames-read form on every config's arena (C1, C2, C3, the C4
# shard), and the ABI test of the new entry point.
set -o pipefail
out=gpurun_out/${1:-r03_ceiling}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_abi_errors.py -m gpu > $out/pytest.log 2>&1 || exit 1
for a in "c1:--no-cpu" "c2:--config 2 --no-cpu" "c3:--config 3 --no-cpu" "c4shard:--packets 4194304 --no-cpu"; do
  timeout -k 10 200 python3 bench.py ${a#*:} > $out/bench_${a%%:*}.json 2> $out/bench_${a%%:*}.err || exit 1
done
