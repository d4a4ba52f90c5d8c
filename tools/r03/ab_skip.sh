#!/bin/bash
# Round 3: the read pass issuing only the slots some row of the wave needs (wave-uniform branches on
# the longest frame) instead of every slot with lanes past the frame reading g_zero16; product (prev)
# vs the measurement build (skip): 1M x 64 B, IMIX-like C3, C1, C2; the parity tests on the variant.
set -o pipefail
out=gpurun_out/${1:-r03_ab_skip}
mkdir -p $out
NFCS_LIB=tools/exp/libnfcs_skip.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread \
   tests/test_gpu_parity.py tests/test_gpu_slot_hint.py tests/test_gpu_fuzz_large.py tests/test_gpu_l3.py -m gpu \
   -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for a in "tiny:--config 0 --packets 1048576 --no-fresh" "c3:--config 3 --no-fresh" "c1:--config 1 --no-c4 --no-fresh" \
         "c2:--config 2 --no-fresh" "l3c3:--op l3fwd --config 3"; do
IFS=: read -r w args <<< "$a"
for r in 1 2; do
for lib in tools/exp/libnfcs_prev.so tools/exp/libnfcs_skip.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py $args --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'$w','lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
