# A/B of tools/exp/libnfcs_prev.so (the build before a change) against netflow_amd/libnfcs.so on
# one box, bench lines alternating; args: <out> "<bench args 1>" "<bench args 2>" ...
set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_slot_hint.py tests/test_gpu_l3.py tests/test_gpu_vlan.py tests/test_gpu_fuzz_large.py tests/test_gpu_edges.py -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for a in "$@"; do
for r in 1 2; do
for lib in tools/exp/libnfcs_prev.so netflow_amd/libnfcs.so; do
  NFCS_LIB=$lib timeout -k 10 200 python bench.py $a --steps 20 --warmup 3 --no-cpu --no-fresh > $O/b.json 2> $O/b.err || exit 1
  python -c "import json;d=json.load(open('$O/b.json'));print('$a', '$lib'.split('/')[-1], d['roofline']['frac'], d['roofline']['kernel_ms'], d['parity']['match'])"
done
done
done
