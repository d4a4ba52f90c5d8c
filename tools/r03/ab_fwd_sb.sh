#!/bin/bash
# Round 3: the fused L3 forward's 4M-frame bursts (deferred stores, per sub-batch) at sub-batch sizes
# 512K (the product) / 768K / 1M; tools/exp/patch_build.py builds, interleaved, 3 rounds.
set -o pipefail
out=gpurun_out/${1:-r03_ab_fwd_sb}
mkdir -p $out
for r in 1 2 3; do
for l in prev sb768 sb1m; do
  NFCS_LIB=tools/exp/libnfcs_$l.so timeout -k 10 200 python3 bench.py --op l3fwd --packets 4194304 --no-cpu --steps 12 --warmup 3 > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'l3fwd_4m','lib':'$l','frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
