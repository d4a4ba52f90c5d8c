#!/bin/bash
# Round 3: the long shape's workgroups per CU (kRowsLdsPad: 22528 B = 7 waves/SIMD, 24576 = 6 (the
# product), 32768 = 5) now that its line-aligned body holds 7 slots, and the sub-batch size of
# batches above 1M long frames (kSubBatchPackets 384K / 512K (the product) / 768K / 1M; the C4
# shard sub-line); C1 with its C4-shard sub-line, C2, interleaved. Libraries from
# tools/exp/patch_build.py (libnfcs_prev.so = the product rebuilt the same way).
set -o pipefail
out=gpurun_out/${1:-r03_ab_occ}
mkdir -p $out
E=tools/exp
for a in "c1:--config 1:prev occ7 occ5 sb384 sb768 sb1m" "c2:--config 2 --no-fresh:prev occ7 occ5" ; do
IFS=: read -r w args libs <<< "$a"
for r in 1 2 3; do
for l in $libs; do
  lib=$E/libnfcs_$l.so
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py $args --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'));f=d.get('fresh') or {};c=d.get('c4_shard') or {}
print(json.dumps({'work':'$w','lib':'$l','frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'fresh_frac':f.get('frac'),'c4':c.get('frac'),'c4_parity':(c.get('parity') or {}).get('match'),'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
