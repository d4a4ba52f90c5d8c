#!/bin/bash
# Round 3 A/B: flow keys lane-per-packet (FK2: 64 packets per wave, header bytes through LDS, one
# VALU instruction per 64 packets) against the product's 8-lane rows (FKp); parity first.
set -o pipefail
out=gpurun_out/${1:-r03_ab_fk2}
mkdir -p $out
NFCS_LIB=tools/exp/libnfcs_FK2.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_flow_keys.py tests/test_gpu_fuzz_large.py -m gpu > $out/pytest.log 2>&1 || exit 1
for r in 1 2; do
for a in "--op flowkey" "--op flowkey --config 3"; do
for v in FKp FK2; do
  NFCS_LIB=tools/exp/libnfcs_$v.so timeout -k 10 200 python3 bench.py $a --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "import json;d=json.load(open('$out/b.json'));print(json.dumps({'args': '$a', 'lib': '$v', 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'value': d['value'], 'parity': d['parity']['match']}))" >> $out/ab.jsonl
done
done
done
