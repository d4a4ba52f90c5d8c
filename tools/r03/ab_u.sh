#!/bin/bash
# Round 3 A/B: the update's short shape (C3-like mixes) in 8-lane rows of 12 slots (U1) against the
# product's 16-lane one-wave rows (U0), now with preloaded arguments.
set -o pipefail
out=gpurun_out/${1:-r03_ab_u}
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for a in "--config 3 --no-fresh" "--config 3 --packets 1048576 --no-fresh"; do
for v in U0 U1; do
  NFCS_LIB=tools/exp/libnfcs_$v.so timeout -k 10 200 python3 bench.py $a --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "import json;d=json.load(open('$out/b.json'));print(json.dumps({'args': '$a', 'lib': '$v', 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': d['parity']['match']}))" >> $out/ab.jsonl
done
done
done
