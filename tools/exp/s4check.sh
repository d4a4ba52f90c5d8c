set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${1:-s4}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_abi_errors.py -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in 1 3 2; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu > $O/c$c.json 2> $O/c$c.err || exit 1
  python -c "import json;d=json.load(open('$O/c$c.json'));print($c, d['roofline']['frac'], d['stream_ceiling'])"
done
NFCS_BENCH_DEVICE=0 timeout -k 10 400 python bench.py --gpus 4 --steps 10 --warmup 2 > $O/g4.json 2> $O/g4.err || { tail -20 $O/g4.err; exit 1; }
python -c "import json;d=json.load(open('$O/g4.json'));print(d['n_gpus'], d['value'], d['per_gpu_GBps'], d['parity'], d['config']['workload'])"
