mkdir -p gpurun_out/occ
for l in 0 20992 24576 32768; do
  timeout -k 10 200 python tools/exp/ab.py --variants 4,5 --work c1,c4shard --lds $l >> gpurun_out/occ/ab.jsonl 2>&1 || exit 1
done
for l in 0 6656 8192; do
  timeout -k 10 200 python tools/exp/ab.py --variants 2,3 --work c3 --lds $l >> gpurun_out/occ/ab.jsonl 2>&1 || exit 1
done
for l in 0 24576; do
  timeout -k 10 200 python tools/exp/ab.py --variants 4 --work c2 --lds $l >> gpurun_out/occ/ab.jsonl 2>&1 || exit 1
  timeout -k 10 200 python tools/exp/ab.py --variants 4 --work c1 --fresh 4 --lds $l >> gpurun_out/occ/ab.jsonl 2>&1 || exit 1
done
cat gpurun_out/occ/ab.jsonl
