#!/bin/bash
# Round 3: the whole GPU suite; PMC traffic of the 4M x 1500 B update and fused forward (record-only
# write pass); rocprofv3 kernel stats of the default line and of the 4M forward; forward lines on C1
# and the C3 mix.
set -o pipefail
out=gpurun_out/r03_check3
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $out/pytest.log 2>&1 || exit 1
timeout -k 10 600 python3 tools/pmc_traffic.py --out $out/pmc --configs 1 --packets 4194304 --ops update l3fwd --merge profiles/traffic.json > $out/pmc.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c1 -o c1 -- python3 bench.py --no-cpu > $out/bench_c1_under_rocprof.json 2> $out/prof_c1.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_l3 -o l3 -- python3 bench.py --op l3fwd --packets 4194304 --no-cpu > $out/bench_l3_4m_under_rocprof.json 2> $out/prof_l3.err || exit 1
for a in "--op l3fwd" "--op l3fwd --config 3"; do
  timeout -k 10 200 python3 bench.py $a --steps 20 --no-cpu >> $out/l3_lines.jsonl 2>> $out/l3_lines.err || exit 1
done
timeout -k 10 200 python3 tools/exp/slot_hint.py 64 256 512 > $out/slot_hint.jsonl 2> $out/slot_hint.err
