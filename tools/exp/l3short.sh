set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${1:-l3short}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_slot_hint.py tests/test_gpu_l3.py -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for lib in tools/exp/libnfcs_prev.so netflow_amd/libnfcs.so; do
  NFCS_LIB=$lib timeout -k 10 200 python bench.py --op l3fwd --config 3 --steps 20 --warmup 3 --no-cpu > $O/l3c3.json 2> $O/l3c3.err || exit 1
  python -c "import json;d=json.load(open('$O/l3c3.json'));print('$lib', d['roofline']['frac'], d['roofline']['kernel_ms'], d['value'], d['parity']['match'])"
done
done
