#!/bin/bash
# Round 3, first check of the new bench fields: GPU tests of the bench lines and the reference's
# path scenario, the default bench line, rocprofv3 of C1 at 2048 / 2176-byte slots, the 8-rank
# rehearsal on one GPU.
set -o pipefail
out=gpurun_out/r03_check1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py \
   tests/test_netflow_adapter.py -m gpu > $out/pytest.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err &&
for a in 2048 2176; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_a$a -o run -- python3 bench.py --no-cpu --no-fresh --no-c4 --align $a --steps 30 > $out/bench_a$a.json 2> $out/prof_a$a.err || exit 1
done &&
NFCS_BENCH_DEVICE=0 timeout -k 10 400 python3 bench.py --gpus 8 --steps 3 --warmup 1 --no-cpu > $out/bench_gpus8_one_box.json 2> $out/bench_gpus8.err
