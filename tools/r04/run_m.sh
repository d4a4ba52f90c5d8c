# round 4 session 2, GPU call m: lanes past a frame with no load request at all — raw buffer loads whose
# out-of-range offset returns zeros (libnfcs_prod_buf, arenas up to 4 GB; timing build) — against the
# product (g_zero16 at page offset 0x5c0), the zero chunk at 0x900 and a 16-line zero pool; bit-exactness
# of the buffer build on the parity / edge / fuzz / line-window tests first (arenas below 4 GB: C2's 9.5 GB
# arena is outside this build's range)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4m && \
NFCS_LIB=tools/r04/libnfcs_prod_buf.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_fuzz_large.py tests/test_gpu_line_windows.py -x -q --deselect 'tests/test_gpu_parity.py::test_full_size_digest_matches_reference[2]' --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4m/pytest_buf.log 2>&1 && \
for r in 1 2 3; do for lib in prod_s2b prod_buf prod_z2304 prod_zp16; do
  for spec in "c3 --config 3" "c1 --config 1"; do
    set -- $spec; name=$1; shift
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4m/${name}_${lib}_$r.json 2>> gpurun_out/r4m/bench.err || exit 1
  done
done; done
