#!/bin/bash
# Round 3 A/B (alternating runs on one box): the round-2 product (prev), the record-only forward
# write pass without MAC loads in deferring waves (C), and C + next-hop-dependent work after the
# frame loads + the footprint sample (D), on the fused forward's three workloads and the update's
# C1 / C3 / C2.
set -o pipefail
out=gpurun_out/${1:-r03_ab_l3}
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for a in "--op l3fwd --config 3" "--op l3fwd" "--op l3fwd --packets 4194304" "--config 3 --no-fresh" "--no-fresh --no-c4" "--config 2 --no-fresh"; do
for v in prev C D; do
  NFCS_LIB=tools/exp/libnfcs_$v.so timeout -k 10 200 python3 bench.py $a --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "import json;d=json.load(open('$out/b.json'));print(json.dumps({'args': '$a', 'lib': '$v', 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': d['parity']['match'], 'ceiling': (d.get('stream_ceiling') or {}).get('read_only_GBps'), 'achieved': d['roofline']['achieved']}))" >> $out/ab.jsonl
done
done
done
