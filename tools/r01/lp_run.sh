set -u
OUT=${1:-lp}
mkdir -p gpurun_out/$OUT
for v in ${PARITY_VARIANTS:-20 21}; do
  NFCS_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_api.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$OUT/pytest_v$v.log 2>&1
  rc=$?; echo "pytest v$v rc=$rc"; tail -3 gpurun_out/$OUT/pytest_v$v.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so bash tools/variants.sh $OUT "${SWEEP_VARIANTS:-0 20 21}" "${SWEEP_CONFIGS:-1 3}"
