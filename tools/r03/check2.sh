#!/bin/bash
# Round 3: GPU tests of the new bench fields, the reference's path scenario and the record-only
# forward write pass; fused-forward A/B (4M x 1500 B) of the round-2 form (prev) against the record
# write pass (B) and B without MAC loads in deferring waves (C = product); the default bench line;
# rocprofv3 of C1 at 2048 / 2176-byte slots; the 8-rank rehearsal on one GPU.
set -o pipefail
out=gpurun_out/r03_check2
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 60 tools/r03/exit_probe > $out/exit_probe.jsonl 2>&1 || exit 1
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_l3.py \
   tests/test_gpu_dist.py tests/test_netflow_adapter.py -m gpu > $out/pytest.log 2>&1 || exit 1
for r in 1 2; do
for v in prev B C; do
  NFCS_LIB=tools/exp/libnfcs_$v.so timeout -k 10 200 python3 bench.py --op l3fwd --packets 4194304 --steps 20 --warmup 3 --no-cpu > $out/l3_$v.json 2> $out/l3_$v.err || exit 1
  python3 -c "import json;d=json.load(open('$out/l3_$v.json'));print('l3fwd 4M', '$v', d['roofline']['frac'], d['roofline']['kernel_ms'], d['parity']['match'])" >> $out/l3ab.txt
done
done
timeout -k 10 300 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err || exit 1
for a in 2048 2176; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_a$a -o run -- python3 bench.py --no-cpu --no-fresh --no-c4 --align $a --steps 30 > $out/bench_a$a.json 2> $out/prof_a$a.err || exit 1
done
NFCS_BENCH_DEVICE=0 timeout -k 10 400 python3 bench.py --gpus 8 --steps 3 --warmup 1 --no-cpu > $out/bench_gpus8_one_box.json 2> $out/bench_gpus8.err
