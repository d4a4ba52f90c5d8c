#!/bin/bash
# Round 3 A/B: the fused forward on the C3 mix (and 1M x 64 B) in 8-lane rows with 12 / 8 / 10 slots
# (G / H / I: 8 packets per wave, so the forward's per-packet header work takes half the
# instructions) against the product's 16-lane rows (F).
set -o pipefail
out=gpurun_out/${1:-r03_ab_l3c3}
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for a in "--op l3fwd --config 3" "--op l3fwd --config 0 --packets 1048576"; do
for v in F G H I; do
  NFCS_LIB=tools/exp/libnfcs_$v.so timeout -k 10 200 python3 bench.py $a --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "import json;d=json.load(open('$out/b.json'));print(json.dumps({'args': '$a', 'lib': '$v', 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': d['parity']['match']}))" >> $out/ab.jsonl
done
done
done
