#!/bin/bash
# Round 3: descriptor prefetch in the checksum read pass (kDescAhead packets ahead) — A/B of the
# build before it (tools/exp/libnfcs_prev.so), the product (8192 ahead) and 4096 / 16384 ahead, on
# one box, bench lines alternating (replay frac by HIP events, fresh frac by wall clock); the GPU
# parity tests of the read pass first.
set -o pipefail
out=gpurun_out/${1:-r03_ab_desc}
mkdir -p $out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py \
   tests/test_gpu_edges.py tests/test_gpu_fuzz_large.py tests/test_gpu_l3.py tests/test_gpu_strides.py -m gpu \
   -p no:cacheprovider > $out/pytest.log 2>&1 || exit 1
tail -1 $out/pytest.log
for a in "c1:--config 1 --no-c4" "c3:--config 3" "c4shard:--packets 4194304 --no-fresh" "c2:--config 2 --no-fresh" \
         "l3c3:--op l3fwd --config 3 --no-fresh" "tiny:--config 0 --packets 1048576 --no-fresh"; do
for r in 1 2; do
for lib in tools/exp/libnfcs_prev.so netflow_amd/libnfcs.so tools/exp/libnfcs_d4k.so tools/exp/libnfcs_d16k.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py ${a#*:} --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || exit 1
  python3 -c "
import json;d=json.load(open('$out/b.json'));f=d.get('fresh') or {}
print(json.dumps({'work':'${a%%:*}','lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],
 'fresh_frac':f.get('frac'),'fresh_ms':f.get('ms_per_step'),'parity':d['parity']['match'],'fresh_parity':f.get('parity')}))" | tee -a $out/ab.jsonl
done
done
done
