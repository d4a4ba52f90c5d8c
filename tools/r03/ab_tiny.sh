#!/bin/bash
# Round 3 A/B: the update's tiny-frame shape (8-lane rows, 8 packets per wave) in one-wave
# workgroups (T0, the product) against 256-thread (T1) and 128-thread (T2) workgroups — a launch of
# one-wave workgroups dispatches ~4.6 workgroups per ns (profiles/r03_s1_exit_probe.jsonl), so 1M tiny
# frames = 131K workgroups cost >= 28 us of dispatch alone.
set -o pipefail
out=gpurun_out/${1:-r03_ab_tiny}
mkdir -p $out
export TMPDIR=/tmp
for r in 1 2; do
for v in T0 T1 T2; do
  NFCS_LIB=tools/exp/libnfcs_$v.so timeout -k 10 200 python3 bench.py --config 0 --packets 1048576 --steps 20 --warmup 3 --no-cpu --no-fresh > $out/b.json 2> $out/b.err || exit 1
  python3 -c "import json;d=json.load(open('$out/b.json'));print(json.dumps({'args': 'c0 1M', 'lib': '$v', 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': d['parity']['match']}))" >> $out/ab.jsonl
  NFCS_LIB=tools/exp/libnfcs_$v.so timeout -k 10 200 python3 tools/exp/slot_hint.py 64 256 512 > $out/sh_$v.jsonl 2> $out/sh.err || exit 1
  python3 -c "
import json
for l in open('$out/sh_$v.jsonl'):
    d=json.loads(l)
    if d['arena']=='exact': print(json.dumps({'args': 'exact %d B' % d['frame'], 'lib': '$v', 'update_us': d['update_us'], 'vlan_us': d['vlan_us'], 'digest': d['update_digest']}))" >> $out/ab.jsonl
done
done
