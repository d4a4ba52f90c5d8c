#!/bin/bash
# Round 3: the fused forward's long shape with line-aligned windows in every wave (fwd1) against
# the product's per-wave choice (prev = the product build), at 128-byte, 64-byte (1600-byte slots)
# and 16-byte starts, C1 and the 4M burst; digests checked.
set -o pipefail
out=gpurun_out/${1:-r03_ab_fwd_lam}
mkdir -p $out
for a in "l3c1:--op l3fwd:128 1600 16" "l3_4m:--op l3fwd --packets 4194304:128 1600"; do
IFS=: read -r w args aligns <<< "$a"
for al in $aligns; do
for r in 1 2; do
for lib in tools/exp/libnfcs_prev.so tools/exp/libnfcs_fwd1.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py $args --align $al --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'$w','align':$al,'lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
done
