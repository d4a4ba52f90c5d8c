#!/bin/bash
# Round 3: C3 at packed / 64-byte / 128-byte frame starts — the product (short shape frame-relative)
# against two measurement builds: the short shape line-aligned per wave (c3la), and the same with
# every slot of a line-aligned wave loaded with the default policy (c3dp: lines shared by
# neighbouring frames then stay in L2 for the second reader). Bench lines alternating, digests checked.
set -o pipefail
out=gpurun_out/${1:-r03_ab_c3pol}
mkdir -p $out
for al in 16 64 128; do
for r in 1 2; do
for lib in netflow_amd/libnfcs.so tools/exp/libnfcs_c3la.so tools/exp/libnfcs_c3dp.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py --config 3 --no-fresh --align $al --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'c3','align':$al,'lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
