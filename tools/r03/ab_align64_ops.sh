#!/bin/bash
# Round 3: the other ops at 64-byte frame starts (DPDK's mempool objects are 64-byte aligned):
# C1 in 1600-byte slots (frames alternate between line offsets 0 and 64) against 1536-byte slots
# (128-byte starts) — VLAN push/pop, flow keys, the fused forward, the update; digests checked.
set -o pipefail
out=gpurun_out/${1:-r03_ab_align64_ops}
mkdir -p $out
for a in "vlan:--op vlan" "fk:--op flowkey" "l3:--op l3fwd" "upd:--config 1 --no-c4 --no-fresh"; do
IFS=: read -r w args <<< "$a"
for r in 1 2; do
for al in 128 1600; do
  timeout -k 10 200 python3 bench.py $args --align $al --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'$w','align':$al,'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
