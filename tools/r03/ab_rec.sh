#!/bin/bash
# Round 3: the read pass's 8-byte patch records stored write-through (sc1) or past the caches
# (sc0 sc1 nt) instead of write-back, so the kernel's end leaves no dirty L2 lines to write back
# before the write pass starts. Product vs the two measurement builds, alternating; digests checked.
set -o pipefail
out=gpurun_out/${1:-r03_ab_rec}
mkdir -p $out
for a in "c1:--config 1 --no-c4" "c4shard:--packets 4194304 --no-fresh" "c2:--config 2 --no-fresh"; do
IFS=: read -r w args <<< "$a"
for r in 1 2 3; do
for lib in netflow_amd/libnfcs.so tools/exp/libnfcs_recwt.so tools/exp/libnfcs_recnt.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py $args --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'));f=d.get('fresh') or {}
print(json.dumps({'work':'$w','lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'fresh_frac':f.get('frac'),'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
