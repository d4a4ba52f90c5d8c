#!/bin/bash
# Round 3 probe: is the flow-key kernel bound by its instructions? The product (FKp) against the same
# loads and record / hash stores with the parse removed (FK0, timing only: the records are raw bytes).
set -o pipefail
out=gpurun_out/${1:-r03_ab_fk}
mkdir -p $out
for r in 1 2; do
for v in FKp FK0; do
  NFCS_LIB=tools/exp/libnfcs_$v.so timeout -k 10 200 python3 bench.py --op flowkey --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "import json;d=json.load(open('$out/b.json'));print(json.dumps({'args': 'flowkey C1', 'lib': '$v', 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': d['parity']['match']}))" >> $out/ab.jsonl
done
done
