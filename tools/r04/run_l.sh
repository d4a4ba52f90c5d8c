# round 4 session 2, GPU call l: as call k (does the address of g_zero16 (the target of the loads of lanes past a
# frame) move C1 / C3? The product build (g_zero16 at page offset 0x5c0) against the same build with
# it at offsets 0x000 / 0x600 / 0x900 (tools/patch_build.py), bench lines alternating on one box
# ... ) plus spread targets: the zero chunk of packet p at line p % 32 / 16 of a 4 KB pool (prod_zp32 / prod_zp16)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4l && \
for r in 1 2 3; do for lib in prod_s2b prod_z2304 prod_zp32 prod_zp16; do
  for spec in "c3 --config 3" "c1 --config 1"; do
    set -- $spec; name=$1; shift
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4l/${name}_${lib}_$r.json 2>> gpurun_out/r4l/bench.err || exit 1
  done
done; done
