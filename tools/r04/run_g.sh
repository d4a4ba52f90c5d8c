# round 4 session 2, GPU call g: why the bench's C3 line (0.691 ms) and fresh_forms' (0.652) disagree on the
# same kernels: the bench line at 2 and 4 rotated batches, fresh_forms at 2 and 4, alternating; the
# shape-independent read + in-place-write bounds (variants 24-27) on C3 and C1; the long shape's inline stores past the caches (libnfcs_r4_inlnt, variant 9) against the product on C1
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4g && \
for r in 1 2; do
  timeout -k 10 200 python3 -u bench.py --config 3 --no-cpu --no-host --no-c4 > gpurun_out/r4g/bench_c3_b2_$r.json 2> gpurun_out/r4g/bench.err && \
  timeout -k 10 200 python3 -u bench.py --config 3 --batches 4 --no-cpu --no-host --no-c4 > gpurun_out/r4g/bench_c3_b4_$r.json 2>> gpurun_out/r4g/bench.err && \
  NFCS_LIB=tools/r04/libnfcs_r4_new.so timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 0 --work c3 --batches 2 --rounds 1 --modes rotate,replay > gpurun_out/r4g/ff_c3_b2_$r.jsonl 2>&1 && \
  NFCS_LIB=tools/r04/libnfcs_r4_new.so timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 0 --work c3 --batches 4 --rounds 1 --modes rotate,replay > gpurun_out/r4g/ff_c3_b4_$r.jsonl 2>&1 || exit 1
done && \
NFCS_LIB=tools/r04/libnfcs_r4_new.so timeout -k 10 300 python3 -u tools/r04/fresh_forms.py --variants 0,15,24,25,26,27 --work c3,c1 --rounds 2 --modes rotate,replay > gpurun_out/r4g/rw_bounds.jsonl 2>&1 && \
NFCS_LIB=tools/r04/libnfcs_r4_inlnt.so timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 0,9 --work c1 --rounds 2 --modes rotate,replay > gpurun_out/r4g/inlnt_c1.jsonl 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4g/prof_c3" -o c3 -- python3 bench.py --config 3 --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4g/prof_c3.json 2> gpurun_out/r4g/prof_c3.err
