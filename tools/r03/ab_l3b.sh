#!/bin/bash
# Round 3 A/B, the fused forward in 8-lane rows (8 packets per wave): G2 = the product (short mixes
# in 8-lane rows of 12 slots, one-wave workgroups), J = the same in 256-thread workgroups, K = 16
# slots at 5 waves/SIMD, M = G2 + long inline bursts (C1) in 8-lane rows of 12 slots, N = M + the
# deferred sub-batches (4M) in them too; F = round 3's previous product (16-lane rows).
set -o pipefail
out=gpurun_out/${1:-r03_ab_l3b}
mkdir -p $out
export TMPDIR=/tmp
run() {
  NFCS_LIB=tools/exp/libnfcs_$2.so timeout -k 10 200 python3 bench.py $1 --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "import json;d=json.load(open('$out/b.json'));print(json.dumps({'args': '$1', 'lib': '$2', 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': d['parity']['match']}))" >> $out/ab.jsonl
}
for r in 1 2; do
  for v in F G2 J K; do run "--op l3fwd --config 3" $v; done
  for v in F G2 M N; do run "--op l3fwd" $v; done
  for v in F G2 M N; do run "--op l3fwd --packets 4194304" $v; done
done
