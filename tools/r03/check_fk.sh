#!/bin/bash
# Round 3: the lane-per-packet flow keys as the product — its GPU tests (C ABI, C++ API, 300k fuzz)
# and bench lines on C1 and C3 frames.
set -o pipefail
out=gpurun_out/${1:-r03_check_fk}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_flow_keys.py tests/test_gpu_fuzz_large.py tests/test_cpp_api.py -m gpu > $out/pytest.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --op flowkey > $out/bench_flowkey.json 2> $out/bench_flowkey.err || exit 1
timeout -k 10 200 python3 bench.py --op flowkey --config 3 --no-cpu > $out/bench_flowkey_c3.json 2> $out/bench_flowkey_c3.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o fk -- python3 bench.py --op flowkey --no-cpu > $out/bench_flowkey_under_rocprof.json 2> $out/prof.err
