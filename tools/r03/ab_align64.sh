#!/bin/bash
# Round 3: 64-byte-aligned frame starts (x86 cache-line alignment, as DPDK mempools give) against
# 128-byte-aligned ones: C1 in 2112-byte slots (frames alternate between line offsets 0 and 64),
# C3 and C2 rounded to 64 bytes; bench lines alternating, digests checked.
set -o pipefail
out=gpurun_out/${1:-r03_ab_align64}
mkdir -p $out
for a in "c1:--config 1 --no-c4 --no-fresh:2176:2112" "c3:--config 3 --no-fresh:128:64" "c2:--config 2 --no-fresh:128:64"; do
IFS=: read -r w args a1 a2 <<< "$a"
for r in 1 2; do
for al in $a1 $a2; do
  timeout -k 10 200 python3 bench.py $args --align $al --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'$w','align':$al,'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
