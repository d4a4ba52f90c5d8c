set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${1:-full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
shift
for a in "$@"; do
for lib in tools/exp/libnfcs_prev.so netflow_amd/libnfcs.so; do
  NFCS_LIB=$lib timeout -k 10 200 python bench.py $a --steps 20 --warmup 3 --no-cpu --no-fresh > $O/b.json 2> $O/b.err || exit 1
  python -c "import json;d=json.load(open('$O/b.json'));print('$a', '$lib'.split('/')[-1], d['roofline']['frac'], d['roofline']['kernel_ms'], d['parity']['match'])"
done
done
