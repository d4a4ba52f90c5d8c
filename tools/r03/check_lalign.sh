#!/bin/bash
# Round 3: the product with line-aligned windows (update long shape, the forward's long and short-mix
# shapes) — the whole GPU suite, then A/B against the build before them on the short/tiny shapes that
# stay frame-relative (C3 at 128 / 64-byte starts, 1M x 64 B) and the default C1 line.
set -o pipefail
out=gpurun_out/${1:-r03_check_lalign}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu \
   -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for a in "c3:--config 3 --no-fresh:128 64" "c1:--config 1 --no-c4 --no-fresh:128" "tiny:--config 0 --packets 1048576 --no-fresh:128"; do
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
