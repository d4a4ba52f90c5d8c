set -u
mkdir -p gpurun_out/pol2
P=netflow_amd/libnfcs.so
run() { NFCS_LIB=$1 timeout -k 10 200 python bench.py --no-cpu --no-fresh $2 > /tmp/o.json || exit 1; python3 -c "
import json,sys; d=json.load(open('/tmp/o.json')); print(json.dumps({'lib': '$1'.split('/')[-1], 'args': '$2', 'value': d['value'], 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms'], 'parity': d['parity']['match']}))" >> gpurun_out/pol2/r.jsonl; }
for L in $P tools/exp/libnfcs_ld_allnt.so tools/exp/libnfcs_ld_alldef.so $P; do run $L "--config 1"; run $L "--config 3"; done
for L in $P tools/exp/libnfcs_vl_ldnt.so $P tools/exp/libnfcs_vl_ldnt.so; do run $L "--op vlan"; done
for L in $P tools/exp/libnfcs_fk_ldnt.so tools/exp/libnfcs_fk_stsys.so $P; do run $L "--op flowkey"; done
