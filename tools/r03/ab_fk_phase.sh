#!/bin/bash
# Round 3: flow keys loading header bytes 0..47 first and chunks 3..5 only for headers that reach
# past them (IPv6, IPv4 options) — the flow-key GPU tests, then A/B against the session's earlier
# build (tools/exp/libnfcs_prev.so) at 128-byte, 64-byte (1600-byte slots) and 16-byte starts.
set -o pipefail
out=gpurun_out/${1:-r03_ab_fk_phase}
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_flow_keys.py \
   tests/test_gpu_fuzz_large.py -m gpu -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for a in "fk:--op flowkey:128 1600 16" "fkc3:--op flowkey --config 3:128 16"; do
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
