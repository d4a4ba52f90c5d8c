#!/bin/bash
# One-segment write-through stores (variants 94/95/117) vs the defaults: parity, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-seg}
mkdir -p "$OUT"
export NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so
for v in 94 95; do
  NFCS_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_v$v.log 2>&1
  rc=$?; echo "pytest v$v rc=$rc"; tail -1 $OUT/pytest_v$v.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
NFCS_VARIANT=117 timeout -k 10 300 python -u -m pytest tests/test_gpu_l3.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_v117.log 2>&1
rc=$?; echo "pytest v117 rc=$rc"; tail -1 $OUT/pytest_v117.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/variants.sh $1 "0 94" "1" && bash tools/variants.sh $1 "0 95" "3" && bash tools/op_ab.sh $1 l3fwd "0 117 118" && \
bash tools/variants.sh ${1}b "94 0" "1" && bash tools/variants.sh ${1}b "95 0" "3"
