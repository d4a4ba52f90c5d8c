#!/bin/bash
# Round 3 A/B on C3 (4M mixed frames): C0 product (short shape, one launch, stores inline);
# C1 512K sub-batches, stores inline; C2 512K sub-batches, every packet's stores deferred to the
# write pass; C3 as C2 with 256K sub-batches; C4 every packet deferred, one launch pair.
set -o pipefail
out=gpurun_out/${1:-r03_ab_c3d}
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for v in C0 C1 C2 C3 C4; do
  NFCS_LIB=tools/exp/libnfcs_$v.so timeout -k 10 200 python3 bench.py --config 3 --no-fresh --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "import json;d=json.load(open('$out/b.json'));print(json.dumps({'lib': '$v', 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': d['parity']['match']}))" >> $out/ab.jsonl
done
done
