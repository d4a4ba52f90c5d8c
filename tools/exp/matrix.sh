#!/bin/bash
# Same-box matrix: inline (1) vs deferred (4) stores in 256-thread workgroups, at 8 (lds 0) and
# 6 (lds 24576) waves/SIMD, on C1 replayed, C1 over 4 fresh batches and the C4 shard; 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-matrix}; mkdir -p $OUT
for r in 1 2 3; do
  for l in 0 24576; do
    timeout -k 10 200 python tools/exp/ab.py --variants 1,4 --work c1,c4shard --lds $l >> $OUT/ab.jsonl 2>&1 || exit 1
    timeout -k 10 200 python tools/exp/ab.py --variants 1,4 --work c1 --fresh 4 --lds $l >> $OUT/ab.jsonl 2>&1 || exit 1
  done
done
python3 - $OUT/ab.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith("{"):
        j = json.loads(l); d[(j["work"], j["fresh"], j["variant"], j["lds"])].append(j["frac"])
for k in sorted(d):
    v = d[k]; print(k, [round(x, 4) for x in v], "mean", round(sum(v) / len(v), 4))
PY
