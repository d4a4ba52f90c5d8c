# L3 forward on the C3 mix: the product's 256-thread workgroups vs one-wave workgroups (measurement)
set -u
mkdir -p gpurun_out/poll3d
P=netflow_amd/libnfcs.so
run() { NFCS_LIB=$1 timeout -k 10 200 python bench.py --no-cpu --no-fresh --op l3fwd $2 > /tmp/o.json || exit 1; python3 -c "
import json,sys; d=json.load(open('/tmp/o.json')); print(json.dumps({'lib': '$1'.split('/')[-1], 'args': '$2', 'value': d['value'], 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'digest': d['parity']['digest'], 'parity': d['parity']['match']}))" >> gpurun_out/poll3d/r.jsonl; }
for L in $P $P; do run $L "--config 3"; run $L "--config 1"; run $L "--config 0 --packets 1048576"; done
