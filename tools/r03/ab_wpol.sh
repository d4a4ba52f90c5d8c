#!/bin/bash
# Round 3: the long shape's write-pass store policy on C1 (1M, replayed and fresh) and the C4 shard:
# `sc0 sc1 nt` (the product) against plain, `nt` and `sc1 nt` byte stores (round 2 measured plain
# and sc1 on the 4M shard only); tools/exp/patch_build.py builds, interleaved, 3 rounds.
set -o pipefail
out=gpurun_out/${1:-r03_ab_wpol}
mkdir -p $out
for r in 1 2 3; do
for l in prev wplain wnt wsc1nt; do
  NFCS_LIB=tools/exp/libnfcs_$l.so timeout -k 10 200 python3 bench.py --config 1 --no-cpu --steps 20 --warmup 3 > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'));f=d.get('fresh') or {};c=d.get('c4_shard') or {}
print(json.dumps({'work':'c1','lib':'$l','frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'fresh_frac':f.get('frac'),'c4':c.get('frac'),'parity':d['parity']['match'],'c4_parity':(c.get('parity') or {}).get('match')}))" | tee -a $out/ab.jsonl
done
done
