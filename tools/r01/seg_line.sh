mkdir -p gpurun_out/s4g && O=gpurun_out/s4g
for v in 84 89 174 175 176; do for p in 1048576 4194304; do
  NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so NFCS_VARIANT=$v timeout -k 10 150 python bench.py --packets $p --steps 20 --warmup 3 --no-cpu > $O/b_${v}_$p.json 2> $O/b_${v}_$p.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/b_${v}_$p.json').read().strip().splitlines()[-1]); print('v$v n=$p frac', d['roofline']['frac'], 'ms', d['roofline']['kernel_ms'], 'parity', d['parity']['match'])"
done; done
