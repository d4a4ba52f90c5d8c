#!/bin/bash
# Round 3: what the per-call workspace event (release_ws: hipEventRecord after the write pass) costs
# between back-to-back calls — the product (prev) against a measurement build without it (noev,
# single-stream use only) and one whose event skips the system-scope fence (evdev); C1 and the C4 shard, then rocprofv3 kernel traces of both for the gaps.
set -o pipefail
out=gpurun_out/${1:-r03_ab_noev}
mkdir -p $out
for a in "c1:--config 1 --no-c4 --no-fresh" "c4shard:--packets 4194304 --no-fresh"; do
IFS=: read -r w args <<< "$a"
for r in 1 2 3; do
for lib in tools/exp/libnfcs_prev.so tools/exp/libnfcs_noev.so tools/exp/libnfcs_evdev.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py $args --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'$w','lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'ms_per_step':d['ms_per_step'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
export TMPDIR=/tmp
for lib in prev noev evdev; do
  NFCS_LIB=tools/exp/libnfcs_$lib.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/tr_$lib -o t -- python3 bench.py --no-cpu --no-fresh --no-c4 --steps 20 > $out/tr_$lib.json 2> $out/tr_$lib.err || exit 1
done
