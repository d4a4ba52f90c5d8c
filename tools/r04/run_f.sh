# round 4 session 2, GPU call f: C3 ablations of the short shape (timing only): the header plan replaced by a
# fixed IPv4/UDP plan, the last-chunk correction removed, both; product short shape (14) and records-only (15);
# then the base build against the session's new plan / last-chunk code (C3 short shape, C1 product)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4f && \
for lib in r4_base abl_noparse abl_noown abl_both r4_new; do
  NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 14,15 --work c3 --rounds 2 --modes rotate > gpurun_out/r4f/abl_$lib.jsonl 2>&1 || exit 1
done && \
for r in 1 2; do for lib in r4_base r4_new; do
  NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 0,14,16 --work c3,c1 --rounds 1 --modes rotate,replay > gpurun_out/r4f/ab${r}_$lib.jsonl 2>&1 || exit 1
done; done
