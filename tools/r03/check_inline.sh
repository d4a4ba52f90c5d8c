#!/bin/bash
# Round 3: short and tiny shapes store inline with no write pass — the whole GPU suite, A/B against
# the build before (tools/exp/libnfcs_prev.so) on C3, 1M x 64 B and C1, and C3's PMC traffic.
set -o pipefail
out=gpurun_out/${1:-r03_check_inline}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu \
   -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for a in "c3:--config 3" "tiny:--config 0 --packets 1048576 --no-fresh" "c1:--config 1 --no-c4 --no-fresh"; do
IFS=: read -r w args <<< "$a"
for r in 1 2; do
for lib in tools/exp/libnfcs_prev.so netflow_amd/libnfcs.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py $args --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'));f=d.get('fresh') or {}
print(json.dumps({'work':'$w','lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'fresh_frac':f.get('frac'),'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
timeout -k 10 600 python3 tools/pmc_traffic.py --out $out/pmc --configs 3 > $out/pmc.log 2>&1 || exit 1
grep "C3" $out/pmc.log
