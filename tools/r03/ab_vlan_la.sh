#!/bin/bash
# Round 3: VLAN push/pop with line-aligned windows (long shape) — the VLAN and line-offset GPU tests,
# then A/B against the build before (tools/exp/libnfcs_prev.so) at 128-byte starts (1536-byte
# slots), 64-byte starts (1600-byte slots) and 2176-byte slots; digests checked.
set -o pipefail
out=gpurun_out/${1:-r03_ab_vlan_la}
mkdir -p $out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_vlan.py \
   tests/test_gpu_line_windows.py tests/test_gpu_slot_hint.py tests/test_gpu_fuzz_large.py tests/test_gpu_edges.py \
   tests/test_netflow_adapter.py -m gpu -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for al in 128 1600 2176; do
for r in 1 2; do
for lib in tools/exp/libnfcs_prev.so netflow_amd/libnfcs.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py --op vlan --align $al --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'vlan','align':$al,'lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
