#!/bin/bash
# Round 3: frame layout A/B on one box — densely packed 16-byte-aligned frame starts (SURVEY.md §8d's
# synthetic layout) against 128-byte-aligned starts (the bench default so far) and 2176-byte slots
# (DPDK's mbuf); bench lines alternating, every line's digest checked against the reference's.
set -o pipefail
out=gpurun_out/${1:-r03_ab_align}
mkdir -p $out
for a in "c1:--config 1 --no-c4" "c3:--config 3" "c4shard:--packets 4194304 --no-fresh" "c2:--config 2 --no-fresh" \
         "l3c1:--op l3fwd" "l3c3:--op l3fwd --config 3" "fk:--op flowkey" "fkc3:--op flowkey --config 3"; do
for r in 1 2; do
for al in 128 16 2176; do
  timeout -k 10 200 python3 bench.py ${a#*:} --align $al --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "
import json;d=json.load(open('$out/b.json'));f=d.get('fresh') or {}
print(json.dumps({'work':'${a%%:*}','align':$al,'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],
 'fresh_frac':f.get('frac'),'parity':d['parity']['match'],'fresh_parity':f.get('parity'),
 'arena_GB':round(d['config']['frame_bytes_per_gpu']/1e9,3)}))" | tee -a $out/ab.jsonl
done
done
done
