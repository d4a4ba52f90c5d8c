#!/bin/bash
# Round 3 final lines: the GPU tests touched since check3, every bench line of the product, and
# rocprofv3 kernel stats of the default line's main workload (C1 only: --no-fresh --no-c4, so the
# averages are C1's launches).
set -o pipefail
out=gpurun_out/${1:-r03_check4}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_slot_hint.py \
   tests/test_gpu_vlan.py tests/test_gpu_l3.py tests/test_gpu_abi_errors.py -m gpu -s > $out/pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err || exit 1
for a in "c2:--config 2 --no-cpu" "c3:--config 3 --no-cpu" "c4shard:--packets 4194304 --no-cpu" "l3fwd:--op l3fwd --no-cpu" \
         "l3fwd_c3:--op l3fwd --config 3 --no-cpu" "l3fwd_4m:--op l3fwd --packets 4194304 --no-cpu" "vlan:--op vlan --no-cpu" \
         "flowkey:--op flowkey --no-cpu"; do
  timeout -k 10 200 python3 bench.py ${a#*:} > $out/bench_${a%%:*}.json 2> $out/bench_${a%%:*}.err || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c1 -o c1 -- python3 bench.py --no-cpu --no-fresh --no-c4 > $out/bench_c1_under_rocprof.json 2> $out/prof_c1.err
