#!/bin/bash
# Round 3: the update's short shape with line-aligned windows per wave, each row line-aligned only
# where its window still fits the 6 slots of one row pass (c3fit), against the product (frame-relative
# short shape): C3 at 128-, 64- and 16-byte starts; the parity tests on the variant first.
set -o pipefail
out=gpurun_out/${1:-r03_ab_c3fit}
mkdir -p $out
NFCS_LIB=tools/exp/libnfcs_c3fit.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread \
   tests/test_gpu_parity.py tests/test_gpu_slot_hint.py tests/test_gpu_fuzz_large.py tests/test_gpu_line_windows.py -m gpu \
   -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for al in 128 64 16; do
for r in 1 2; do
for lib in tools/exp/libnfcs_prev.so tools/exp/libnfcs_c3fit.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py --config 3 --no-fresh --align $al --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'c3','align':$al,'lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
