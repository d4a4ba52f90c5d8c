#!/bin/bash
# Store-form / occupancy / block-order variants of the write-back kernel on the C4 shard (4M x
# 1500 B) and the C1 batch, each a bench line with its parity digest. Session 4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-wbf}; mkdir -p "$O"
for v in ${2:-84 177 178 179}; do for p in 4194304 1048576; do
  NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so NFCS_VARIANT=$v timeout -k 10 150 python bench.py --packets $p \
      --steps 20 --warmup 3 --no-cpu > "$O/b_${v}_$p.json" 2> "$O/b_${v}_$p.err" || exit 1
  python3 -c "import json; d=json.loads(open('$O/b_${v}_$p.json').read().strip().splitlines()[-1]); print('v$v n=$p frac', d['roofline']['frac'], 'ms', d['roofline']['kernel_ms'], 'parity', d['parity']['match'])"
done; done
