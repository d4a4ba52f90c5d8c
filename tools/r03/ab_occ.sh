#!/bin/bash
# Round 3: the long shape's workgroups per CU (kRowsLdsPad: 22528 B = 7 waves/SIMD, 24576 = 6 (the
# product), 32768 = 5) now that its line-aligned body holds 7 slots; C1, C4 shard, C2, interleaved.
set -o pipefail
out=gpurun_out/${1:-r03_ab_occ}
mkdir -p $out
for a in "c1:--config 1" "c2:--config 2 --no-fresh" ; do
IFS=: read -r w args <<< "$a"
for r in 1 2 3; do
for lib in tools/exp/libnfcs_prev.so tools/exp/libnfcs_occ7.so tools/exp/libnfcs_occ5.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py $args --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'));f=d.get('fresh') or {};c=d.get('c4_shard') or {}
print(json.dumps({'work':'$w','lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'fresh_frac':f.get('frac'),'c4':(c.get('roofline') or {}).get('frac', c.get('frac')),'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
