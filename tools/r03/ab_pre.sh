#!/bin/bash
# Round 3 A/B (alternating runs on one box): D (the footprint sample + next-hop work after the frame
# loads), E (D with kernel arguments preloaded into SGPRs) and F (E with the row kernel's arguments
# reordered so every argument a wave needs before its frame loads is preloaded, and the grid size
# passed explicitly instead of read from the hidden arguments).
set -o pipefail
out=gpurun_out/${1:-r03_ab_pre}
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for a in "--config 3 --no-fresh" "--op l3fwd --config 3" "--no-fresh --no-c4" "--op l3fwd" "--packets 4194304 --no-fresh" "--config 2 --no-fresh" "--config 0 --packets 1048576 --no-fresh" "--op vlan" "--op flowkey"; do
for v in D E F; do
  NFCS_LIB=tools/exp/libnfcs_$v.so timeout -k 10 200 python3 bench.py $a --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "import json;d=json.load(open('$out/b.json'));print(json.dumps({'args': '$a', 'lib': '$v', 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': d['parity']['match']}))" >> $out/ab.jsonl
done
done
done
