# L3 forward segment-store policy A/B (measurement; see tools/exp/patch_build.py): 64-byte frames
# (8-lane rows) and the C3 mix (16-lane rows), product vs nt in 8-lane rows vs nt everywhere.
set -u
mkdir -p gpurun_out/poll3
P=netflow_amd/libnfcs.so
run() { NFCS_LIB=$1 timeout -k 10 200 python bench.py --no-cpu --no-fresh --op l3fwd $2 > /tmp/o.json || exit 1; python3 -c "
import json,sys; d=json.load(open('/tmp/o.json')); print(json.dumps({'lib': '$1'.split('/')[-1], 'args': '$2', 'value': d['value'], 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'digest': d['parity']['digest'], 'parity': d['parity']['match']}))" >> gpurun_out/poll3/r.jsonl; }
for L in $P tools/exp/libnfcs_l3nt8.so tools/exp/libnfcs_l3ntall.so $P tools/exp/libnfcs_l3nt8.so tools/exp/libnfcs_l3ntall.so; do
  run $L "--config 0 --packets 1048576"; run $L "--config 3"; done
