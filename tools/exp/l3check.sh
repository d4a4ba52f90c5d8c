set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/l3d1; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_l3.py tests/test_gpu_fuzz_large.py tests/test_gpu_slot_hint.py tests/test_gpu_high_offsets.py -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -8 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in 0 4194304 2097152; do
  timeout -k 10 200 python bench.py --op l3fwd --packets $p --steps 20 --warmup 3 --no-cpu > $O/l3_$p.json 2>&1 || exit 1
  python -c "import json;d=json.load(open('$O/l3_$p.json'));print($p, d['roofline']['frac'], d['roofline']['kernel_ms'], d['parity'])"
done
