#!/bin/bash
# Round 3: the short and tiny shapes storing every wave inline (no write pass launched) against the
# product (a deferral decision per group of 4 and a write pass for the <1% of C3 waves that defer);
# C3 (replayed and fresh), 1M x 64 B; the parity tests on the variant first.
set -o pipefail
out=gpurun_out/${1:-r03_ab_c3inl}
mkdir -p $out
NFCS_LIB=tools/exp/libnfcs_c3inl.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread \
   tests/test_gpu_parity.py tests/test_gpu_slot_hint.py tests/test_gpu_fuzz_large.py -m gpu \
   -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for a in "c3:--config 3" "c3a64:--config 3 --align 64 --no-fresh" "tiny:--config 0 --packets 1048576 --no-fresh"; do
IFS=: read -r w args <<< "$a"
for r in 1 2 3; do
for lib in tools/exp/libnfcs_prev.so tools/exp/libnfcs_c3inl.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py $args --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'));f=d.get('fresh') or {}
print(json.dumps({'work':'$w','lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'fresh_frac':f.get('frac'),'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
