#!/bin/bash
# Round 3: line-aligned row windows, per-wave form (update long shape: always, 7 slots; update
# short shape and the forward's long shape: only waves with a row starting mid-line, 6 / 7 slots;
# the forward's short-mix rows: always; 8-lane tiny rows: never). The GPU suite, then A/B of the
# build before line-aligned windows (tools/exp/libnfcs_prev.so) against the product on one box,
# bench lines alternating, for 128-byte-aligned (the default), densely packed and 64-byte-aligned
# frames; every digest checked against the reference's.
set -o pipefail
out=gpurun_out/${1:-r03_ab_lalign3}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu \
   -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for a in "c1:--config 1 --no-c4 --no-fresh:128 16 2112" "c4shard:--packets 4194304 --no-fresh:128 16" \
         "c3:--config 3 --no-fresh:128 16 64" "c2:--config 2 --no-fresh:128 16" "l3c1:--op l3fwd:128 16" \
         "l3c3:--op l3fwd --config 3:128 16" "l3_4m:--op l3fwd --packets 4194304:128 16" \
         "tiny:--config 0 --packets 1048576 --no-fresh:128 16"; do
IFS=: read -r w args aligns <<< "$a"
for al in $aligns; do
for r in 1 2; do
for lib in tools/exp/libnfcs_prev.so netflow_amd/libnfcs.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py $args --align $al --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'$w','align':$al,'lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
done
