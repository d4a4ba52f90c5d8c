set -u
mkdir -p gpurun_out/wt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wt/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/wt/pytest.log; [ $rc -eq 0 ] || exit $rc
export NFCS_LIB=$PWD/netflow_amd/libnfcs_exp.so
bash tools/variants.sh wt "0 84" "1" && bash tools/variants.sh wt "0 83" "3" && bash tools/variants.sh wt "0 9" "2" && \
bash tools/variants.sh wt2 "84 0" "1" && bash tools/variants.sh wt2 "83 0" "3" && bash tools/variants.sh wt2 "9 0" "2" && \
bash tools/op_ab.sh wt vlan "0 32" && bash tools/op_ab.sh wt l3fwd "0"
