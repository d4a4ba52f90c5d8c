#!/bin/bash
# The round-4 GPU calls, one function per call (the exact command each ran through gpurun, from the repo
# root): `bash tools/r04/calls.sh <letter>`. Session 1: a-e (store forms under rotation, bounds, pipelined
# and slot-count short shapes, every bench line); session 2: f-r (ablations and A/Bs of the short shape's
# plan, zero-chunk targets and buffer loads, the forward's deferral threshold). Their results are in
# profiles/r04_s1_* and profiles/r04_s2_*; the libraries they name are built by tools/r04/build.sh,
# tools/r04/exp_build.py and tools/patch_build.py (git-ignored).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"

call_a() {
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4a && timeout -k 10 240 python3 -u tools/r04/fresh_forms.py --variants 0,1,2,3,4,5,6,7,8,9,10 --work c1 --rounds 2 > gpurun_out/r4a/forms_c1.jsonl 2>&1 && timeout -k 10 240 python3 -u tools/r04/fresh_forms.py --variants 0,1,11,12,13,14 --work c3 --rounds 2 > gpurun_out/r4a/forms_c3.jsonl 2>&1 && timeout -k 10 240 python3 -u tools/r04/fresh_forms.py --variants 0,1,4,7,10 --work c4shard --rounds 1 > gpurun_out/r4a/forms_c4.jsonl 2>&1 && timeout -k 10 240 python3 -u tools/r04/fresh_forms.py --variants 20,21,22,23 --work c1,c3 --rounds 2 > gpurun_out/r4a/bounds.jsonl 2>&1 && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r4a/prof -o rot -- python3 -u tools/r04/fresh_forms.py --variants 0 --modes rotate,replay --rounds 1 --iters 100 > gpurun_out/r4a/prof.log 2>&1
}

call_b() {
  # round 4, GPU call b: 64-byte-record deferral forms (C1, C3, C4 shard), then the bench default line
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4b && \
  timeout -k 10 240 python3 -u tools/r04/fresh_forms.py --variants 0,1,30,31,32,40,41,42 --work c1 --rounds 2 > gpurun_out/r4b/forms_c1.jsonl 2>&1 && \
  timeout -k 10 240 python3 -u tools/r04/fresh_forms.py --variants 0,15,33,34,14 --work c3 --rounds 2 > gpurun_out/r4b/forms_c3.jsonl 2>&1 && \
  timeout -k 10 240 python3 -u tools/r04/fresh_forms.py --variants 0,30,31 --work c4shard --rounds 1 > gpurun_out/r4b/forms_c4.jsonl 2>&1 && \
  timeout -k 10 300 python3 -u bench.py > gpurun_out/r4b/bench.json 2> gpurun_out/r4b/bench.err && \
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/pytest.log 2>&1
}

call_c() {
  # round 4, GPU call c: the software-pipelined short shape on C3
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4c && \
  timeout -k 10 300 python3 -u tools/r04/fresh_forms.py --variants 0,15,50,51,52,53,54,55,56,57 --work c3 --rounds 2 --modes rotate > gpurun_out/r4c/pipe_c3.jsonl 2>&1
}

call_d() {
  # round 4, GPU call d: short-shape slot counts on C3, then the round-4 profiles of every line
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4d && \
  timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 0,17,18,19 --work c3 --rounds 2 --modes rotate > gpurun_out/r4d/slots_c3.jsonl 2>&1 && \
  bash tools/r04/prof_all.sh r4d/prof
}

call_e() {
  # round 4, GPU call e: every bench line with the rotation (update, forward, VLAN, flow keys; C1-C3, 4M)
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4e && \
  for spec in "l3fwd_c1 --op l3fwd" "l3fwd_4m --op l3fwd --packets 4194304" "l3fwd_c3 --op l3fwd --config 3" "vlan --op vlan" "flowkey --op flowkey" "flowkey_c3 --op flowkey --config 3" "c2 --config 2" "c3 --config 3" "c4shard --packets 4194304"; do
    set -- $spec; name=$1; shift
    timeout -k 10 240 python3 -u bench.py "$@" --no-cpu > gpurun_out/r4e/$name.json 2> gpurun_out/r4e/$name.err || exit 1
  done
}

call_f() {
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
}

call_g() {
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
}

call_h() {
  # round 4 session 2, GPU call h: the GPU suite on the product, then the product bench lines with the
  # session's kernels against the session-start kernels (NFCS_LIB: libnfcs_r4_base = session start,
  # libnfcs_r4_s2a = + branch-free plan and last-chunk correction, libnfcs_r4_new = + forward deferral
  # above 64K packets = the product), alternating on one box; then the read-only bounds 24 / 26 (fixed)
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4h && \
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4h/pytest_gpu.log 2>&1 && \
  for r in 1 2 3; do for lib in r4_base r4_s2a r4_new; do
    for spec in "c3 --config 3" "c1 --config 1" "fwdc1 --op l3fwd --config 1" "fwdc3 --op l3fwd --config 3"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4h/${name}_${lib}_$r.json 2>> gpurun_out/r4h/bench.err || exit 1
    done
  done; done && \
  NFCS_LIB=tools/r04/libnfcs_r4_new.so timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 24,26,25,27,0 --work c3 --rounds 1 --modes rotate,replay > gpurun_out/r4h/rw_c3.jsonl 2>&1 && \
  NFCS_LIB=tools/r04/libnfcs_r4_new.so timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 24,26,25,27,0 --work c1 --rounds 1 --modes rotate,replay > gpurun_out/r4h/rw_c1.jsonl 2>&1
}

call_i() {
  # round 4 session 2, GPU call i: C1 in one launch pair against 512K sub-batches (variant 10) under rotation,
  # alternating; rocprofv3 kernel stats of the C1 line; the 8-rank path rehearsed on this one GPU
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4i && \
  NFCS_LIB=tools/r04/libnfcs_r4_new.so timeout -k 10 300 python3 -u tools/r04/fresh_forms.py --torch --variants 0,10 --work c1 --rounds 4 --modes rotate,replay > gpurun_out/r4i/sub_c1.jsonl 2>&1 && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4i/prof_c1" -o c1 -- python3 bench.py --no-cpu --no-host --no-c4 --no-replay --steps 50 > gpurun_out/r4i/prof_c1.json 2> gpurun_out/r4i/prof_c1.err && \
  NFCS_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --gpus 8 --steps 3 --warmup 1 > gpurun_out/r4i/bench_gpus8_one_box.json 2> gpurun_out/r4i/bench_gpus8.err
}

call_j() {
  # round 4 session 2, GPU call j: the GPU suite on the product (lanes past a frame load its first chunk),
  # then bench C3 / C1 alternating over four libraries on one box: the product build before / after that
  # change (libnfcs_prod_s2b / libnfcs_prod_zs) and the measurement builds of the same two sources
  # (libnfcs_r4_new / libnfcs_r4_zs) — the product build measured 3-5% slower on C3 than the measurement
  # build of the same kernel source in calls f, g and the profiling pass
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4j && \
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4j/pytest_gpu.log 2>&1 && \
  for r in 1 2 3; do for lib in prod_s2b r4_new prod_zs r4_zs; do
    for spec in "c3 --config 3" "c1 --config 1"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4j/${name}_${lib}_$r.json 2>> gpurun_out/r4j/bench.err || exit 1
    done
  done; done
}

call_k() {
  # round 4 session 2, GPU call k: does the address of g_zero16 (the target of the loads of lanes past a
  # frame) move C1 / C3? The product build (g_zero16 at page offset 0x5c0) against the same build with
  # it at offsets 0x000 / 0x600 / 0x900 (tools/patch_build.py), bench lines alternating on one box
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4k && \
  for r in 1 2 3; do for lib in prod_s2b prod_z4k prod_z1536 prod_z2304; do
    for spec in "c3 --config 3" "c1 --config 1"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4k/${name}_${lib}_$r.json 2>> gpurun_out/r4k/bench.err || exit 1
    done
  done; done
}

call_l() {
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
}

call_m() {
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
}

call_n() {
  # round 4 session 2, GPU call n: the product with per-wave buffer loads (lanes past a frame read zeros
  # with no request): the whole GPU suite, then bench lines alternating against the session's previous
  # product (libnfcs_prod_s2b: lanes past a frame load g_zero16) on one box: C3, C1, C2, the C4 shard;
  # then flow keys with their zero lanes as out-of-range buffer loads (libnfcs_prod_fkbuf, timing build,
  # arenas up to 4 GB) against the product
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4n && \
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4n/pytest_gpu.log 2>&1 && \
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4n/smoke.log 2>&1 && \
  for r in 1 2 3; do for lib in prod_s2b prod_wbuf; do
    for spec in "c3 --config 3" "c1 --config 1" "c2 --config 2" "c4 --packets 4194304" "fwdc3 --op l3fwd --config 3"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4n/${name}_${lib}_$r.json 2>> gpurun_out/r4n/bench.err || exit 1
    done
  done; done && \
  for r in 1 2 3; do for lib in prod_wbuf prod_fkbuf; do
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py --op flowkey --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4n/fk_${lib}_$r.json 2>> gpurun_out/r4n/bench.err || exit 1
  done; done
}

call_o() {
  # round 4 session 2, GPU call o: buffer loads only in the plain update's one-wave shapes (short: C3; tiny:
  # 1M x 64-byte frames in 128-byte slots) — libnfcs_prod_wbuf2 — against libnfcs_prod_s2b, alternating on one
  # box; C1, the C4 shard and the forward's C3 mix should be unchanged (they keep global loads)
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4o && \
  for r in 1 2 3; do for lib in prod_s2b prod_wbuf2; do
    for spec in "c3 --config 3" "tiny --config 0 --packets 1048576" "c1 --config 1" "c4 --packets 4194304" "fwdc3 --op l3fwd --config 3"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4o/${name}_${lib}_$r.json 2>> gpurun_out/r4o/bench.err || exit 1
    done
  done; done
}

call_p() {
  # round 4 session 2, GPU call p: the product (buffer loads in the plain update's short shape): the whole GPU
  # suite, smoke(), the default bench line (CPU baseline, replay / C4-shard / host sub-lines), C3, then
  # rocprofv3 kernel stats of C3
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4p && \
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4p/pytest_gpu.log 2>&1 && \
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4p/smoke.log 2>&1 && \
  timeout -k 10 400 python3 -u bench.py > gpurun_out/r4p/bench_default.json 2> gpurun_out/r4p/bench_default.err && \
  timeout -k 10 200 python3 -u bench.py --config 3 --no-cpu --no-host --no-c4 > gpurun_out/r4p/bench_c3.json 2> gpurun_out/r4p/bench_c3.err && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4p/prof_c3" -o c3 -- python3 bench.py --config 3 --no-cpu --no-host --no-c4 --no-replay --steps 30 > gpurun_out/r4p/prof_c3.json 2> gpurun_out/r4p/prof_c3.err
}

call_q() {
  # round 4 session 2, GPU call q: buffer loads in every shape of the plain update with no global-load path
  # in the kernel (a wave whose frames span more than 4 GB sends its rows to the cold path) —
  # libnfcs_prod_wbuf3 = the product — the whole GPU suite, then bench lines alternating against the previous
  # product (libnfcs_prod_s2c: buffer loads in the short shape only, global-load fallback in the kernel)
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4q && \
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4q/pytest_gpu.log 2>&1 && \
  for r in 1 2 3; do for lib in prod_s2c prod_wbuf3; do
    for spec in "c1 --config 1" "c3 --config 3" "tiny --config 0 --packets 1048576" "c4 --packets 4194304" "c2 --config 2"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4q/${name}_${lib}_$r.json 2>> gpurun_out/r4q/bench.err || exit 1
    done
  done; done
}

call_r() {
  # round 4 session 2, GPU call r: is the fused forward's short-mix shape (C3 mix) and the tiny shape sensitive
  # to g_zero16's address as C3's short shape was? The product (g_zero16 at page offset 0x5c0) against builds
  # with it at 0x900 / 0x600, alternating on one box
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4r && \
  for r in 1 2 3; do for lib in prod_s2c prod_z2304 prod_z1536; do
    for spec in "fwdc3 --op l3fwd --config 3" "tiny --config 0 --packets 1048576" "vlan --op vlan"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4r/${name}_${lib}_$r.json 2>> gpurun_out/r4r/bench.err || exit 1
    done
  done; done
}

call_s() {
  # round 4 session 2, GPU call s: instructions per wave of the C3 short shape (the update) and the forward's
  # C3 mix after the session's plan rewrite: SQ counters, one rocprofv3 pass each (kernel trace only)
  mkdir -p gpurun_out/r4s && export TMPDIR=/tmp && \
  for spec in "c3 --config 3" "fwdc3 --op l3fwd --config 3"; do
    set -- $spec; name=$1; shift
    timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-trace --output-format csv -d "$PWD/gpurun_out/r4s/$name" -o p -- python3 bench.py "$@" --no-cpu --no-host --no-c4 --no-replay --steps 10 --warmup 1 > gpurun_out/r4s/$name.json 2> gpurun_out/r4s/$name.err || return 1
  done
}

call_t() {
  # round 4 session 2, GPU call t: the fused forward's deferred read pass (bursts above 64K long frames) at 7
  # waves/SIMD (the product) against 6 and 5 (unused dynamic LDS caps the workgroups per CU, as the update's
  # long shape is held at 6): forward C1 and 4M, alternating on one box
  mkdir -p gpurun_out/r4t && export TMPDIR=/tmp && \
  for r in 1 2 3; do for lib in prod_s2c prod_fwd6 prod_fwd5; do
    for spec in "fwdc1 --op l3fwd --config 1" "fwd4m --op l3fwd --packets 4194304"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4t/${name}_${lib}_$r.json 2>> gpurun_out/r4t/bench.err || return 1
    done
  done; done
}

call_u() {
  # round 4 session 2, GPU call u: the update's long shape at 7 waves/SIMD (21 KB of unused LDS per
  # workgroup) against the product's 6, now that the steady state (rotation) is the measure — round 3's
  # sweep chose 6 on the replayed form and noted fresh batches +1.5% at 7 — C1 and the C4 shard, alternating
  mkdir -p gpurun_out/r4u && export TMPDIR=/tmp && \
  for r in 1 2 3; do for lib in prod_s2c prod_occ7; do
    for spec in "c1 --config 1" "c4 --packets 4194304" "c2 --config 2"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4u/${name}_${lib}_$r.json 2>> gpurun_out/r4u/bench.err || return 1
    done
  done; done
}

call_v() {
  # round 4 session 2, GPU call v: the final product (the forward's deferred read pass at 6 waves/SIMD):
  # the whole GPU suite, smoke(), the default bench line, the forward lines (C1, 4M, C3 mix) and C3
  mkdir -p gpurun_out/r4v && export TMPDIR=/tmp && \
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4v/pytest_gpu.log 2>&1 && \
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v/smoke.log 2>&1 && \
  timeout -k 10 400 python3 -u bench.py > gpurun_out/r4v/bench_default.json 2> gpurun_out/r4v/bench_default.err && \
  for spec in "fwdc1 --op l3fwd --config 1" "fwd4m --op l3fwd --packets 4194304" "fwdc3 --op l3fwd --config 3" "c3 --config 3"; do
    set -- $spec; name=$1; shift
    timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 > gpurun_out/r4v/bench_$name.json 2>> gpurun_out/r4v/bench.err || return 1
  done
}

call_w() {
  # round 4 session 2, GPU call w: C1 as one read + write pass pair (the product) against two 512K sub-batches
  # (kSubBatchAbovePackets 512K, libnfcs_prod_sb512): on some boxes C1 ran 2-3% below the C4 shard's 512K
  # sub-batches in the same run; bench C1 alternating, then rocprofv3 kernel stats of both
  mkdir -p gpurun_out/r4w && export TMPDIR=/tmp && \
  for r in 1 2 3; do for lib in prod_s2e prod_sb512; do
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py --no-cpu --no-host --no-replay > gpurun_out/r4w/c1_${lib}_$r.json 2>> gpurun_out/r4w/bench.err || return 1
  done; done && \
  for lib in prod_s2e prod_sb512; do
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4w/prof_$lib" -o c1 -- python3 bench.py --no-cpu --no-host --no-replay --no-c4 --steps 40 > gpurun_out/r4w/prof_$lib.json 2> gpurun_out/r4w/prof_$lib.err || return 1
  done
}

call_x() {
  # round 4 session 2, GPU call x: the product with long-frame batches split above 512K packets (C1 = two
  # sub-batches): the whole GPU suite, smoke(), the default bench line, rocprofv3 kernel stats of C1
  mkdir -p gpurun_out/r4x && export TMPDIR=/tmp && \
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4x/pytest_gpu.log 2>&1 && \
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4x/smoke.log 2>&1 && \
  timeout -k 10 400 python3 -u bench.py > gpurun_out/r4x/bench_default.json 2> gpurun_out/r4x/bench_default.err && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4x/prof_c1" -o c1 -- python3 bench.py --no-cpu --no-host --no-replay --no-c4 --steps 40 > gpurun_out/r4x/prof_c1.json 2> gpurun_out/r4x/prof_c1.err
}

call_y() {
  # round 4 session 2, GPU call y: PMC traffic per call of C1 and C2 now that C1 runs as two 512K
  # sub-batches (tools/pmc_traffic.py counts the sub-batches per call), merged into the committed record
  mkdir -p gpurun_out/r4y && export TMPDIR=/tmp && \
  timeout -k 10 600 python3 tools/pmc_traffic.py --out "$PWD/gpurun_out/r4y/pmc" --configs 1 --merge "$PWD/profiles/traffic.json" > gpurun_out/r4y/pmc.log 2>&1
}

call_z() {
  # round 4 session 2, GPU call z: jumbo frames' continuation batches double-buffered (batch b+1's loads in
  # flight while b is summed; libnfcs_prod_dbuf, timing build: the long shape's registers rise to 85 VGPRs)
  # against the product (libnfcs_prod_s2f): C2 and C1, alternating
  mkdir -p gpurun_out/r4z && export TMPDIR=/tmp && \
  for r in 1 2 3; do for lib in prod_s2f prod_dbuf; do
    for spec in "c2 --config 2" "c1 --config 1"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4z/${name}_${lib}_$r.json 2>> gpurun_out/r4z/bench.err || return 1
    done
  done; done
}

call_aa() {
  # round 4 session 2, GPU call aa: why the double-buffered build (85 VGPRs in the long shape) ran C1 1.2%
  # faster although C1 never enters the continuation loop: the product (6 waves/SIMD, LDS cap), the dbuf
  # build and the product held at 5 waves/SIMD by LDS (libnfcs_prod_occ5): C1, the C4 shard, C2, alternating
  mkdir -p gpurun_out/r4aa && export TMPDIR=/tmp && \
  for r in 1 2 3; do for lib in prod_s2f prod_dbuf prod_occ5; do
    for spec in "c1 --config 1" "c4 --packets 4194304" "c2 --config 2"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4aa/${name}_${lib}_$r.json 2>> gpurun_out/r4aa/bench.err || return 1
    done
  done; done
}

call_ab() {
  # round 4 session 2, GPU call ab: the product with the long shape at 5 waves/SIMD (forward's deferred
  # read pass kept at 6): the whole GPU suite, smoke(), the default bench line, C2/C3/C4 shard and the
  # forward lines, rocprofv3 kernel stats of C1
  mkdir -p gpurun_out/r4ab && export TMPDIR=/tmp && \
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4ab/pytest_gpu.log 2>&1 && \
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ab/smoke.log 2>&1 && \
  timeout -k 10 400 python3 -u bench.py > gpurun_out/r4ab/bench_default.json 2> gpurun_out/r4ab/bench_default.err && \
  for spec in "c2 --config 2" "c3 --config 3" "c4shard --packets 4194304" "l3fwd_c1 --op l3fwd" "l3fwd_4m --op l3fwd --packets 4194304"; do
    set -- $spec; name=$1; shift
    timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4ab/$name.json 2>> gpurun_out/r4ab/bench.err || return 1
  done && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4ab/prof_c1" -o c1 -- python3 bench.py --no-cpu --no-host --no-replay --no-c4 --steps 40 > gpurun_out/r4ab/prof_c1.json 2> gpurun_out/r4ab/prof_c1.err
}

call_ac() {
  # round 4 session 2, GPU call ac: each sub-batch's write pass on a second stream (event-ordered after its
  # read pass), so it runs beside the next sub-batch's read pass; only the last write pass stays on the
  # caller's stream. ovl512 / ovl256: 512K / 256K sub-batches, device-scope events; ovl512s: default
  # (system-scope) events. Against the product (prod_f4): C1 and the C4 shard, alternating
  mkdir -p gpurun_out/r4ac && export TMPDIR=/tmp && \
  for r in 1 2 3; do for lib in prod_f4 ovl512 ovl256 ovl512s; do
    for spec in "c1 --config 1" "c4 --packets 4194304"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4ac/${name}_${lib}_$r.json 2>> gpurun_out/r4ac/bench.err || return 1
    done
  done; done
}

call_ad() {
  # round 4 session 2, GPU call ad: VLAN's long shape (127 VGPRs = 4 waves/SIMD) under __launch_bounds__
  # 5 / 6 waves (96 / 80 VGPRs, 60 / 120 spilled to scratch; libnfcs_vlanw5 / w6) against the product:
  # the VLAN bench line (C1 push/pop), alternating
  mkdir -p gpurun_out/r4ad && export TMPDIR=/tmp && \
  for r in 1 2 3; do for lib in prod_f4 vlanw5 vlanw6; do
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py --op vlan --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4ad/vlan_${lib}_$r.json 2>> gpurun_out/r4ad/bench.err || return 1
  done; done
}

call_ae() {
  # round 4 session 2, GPU call ae: VLAN's long shape with fewer continuation slots per batch (K2 = 2 / 3;
  # C1's 1500-byte frames rarely continue) so that __launch_bounds__(256, 5) gives 5 waves/SIMD with few
  # spills (K2 = 2: 96 VGPRs, 6 spilled; K2 = 3: 21 spilled), and K2 = 3 alone (112 VGPRs, 4 waves):
  # against the product, the VLAN bench line, alternating
  mkdir -p gpurun_out/r4ae && export TMPDIR=/tmp && \
  for r in 1 2 3; do for lib in prod_f4 vlan_k2lb5 vlan_k3lb5 vlan_k3; do
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py --op vlan --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4ae/vlan_${lib}_$r.json 2>> gpurun_out/r4ae/bench.err || return 1
  done; done
}

call_af() {
  # round 4 session 2, GPU call af: is the flow-key kernel occupancy-limited? Header rows of 80 instead of 96
  # LDS bytes per packet (20 KiB per workgroup: 8 waves/SIMD instead of 6; timing probe only, headers
  # past byte 79 are not staged: C1's untagged IPv4 frames need 38), against the product: flowkey, alternating
  mkdir -p gpurun_out/r4af && export TMPDIR=/tmp && \
  for r in 1 2 3; do for lib in prod_f4 fk80; do
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py --op flowkey --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4af/fk_${lib}_$r.json 2>> gpurun_out/r4af/bench.err || return 1
  done; done
}

call_ag() {
  # round 4 session 2, GPU call ag: the final tree: smoke(), the default bench line, the 8-rank path
  # rehearsed on this one GPU (every rank's C4 shard digest checked)
  mkdir -p gpurun_out/r4ag && export TMPDIR=/tmp && \
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ag/smoke.log 2>&1 && \
  timeout -k 10 400 python3 -u bench.py > gpurun_out/r4ag/bench_default.json 2> gpurun_out/r4ag/bench_default.err && \
  NFCS_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --gpus 8 --steps 3 --warmup 1 > gpurun_out/r4ag/bench_gpus8_one_box.json 2> gpurun_out/r4ag/bench_gpus8.err
}

call_ah() {
  # round 4 session 2, GPU call ah: the long shape at 4 waves/SIMD (LDS pad 40960; libnfcs_occ4) against the
  # product at 5 (libnfcs_prod_f5): C1, the C4 shard, C2, alternating
  mkdir -p gpurun_out/r4ah && export TMPDIR=/tmp && \
  for r in 1 2 3; do for lib in prod_f5 occ4; do
    for spec in "c1 --config 1" "c4 --packets 4194304" "c2 --config 2"; do
      set -- $spec; name=$1; shift
      NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4ah/${name}_${lib}_$r.json 2>> gpurun_out/r4ah/bench.err || return 1
    done
  done; done
}

call_ai() {
  # round 4 session 2, GPU call ai: the whole GPU suite on the final tree
  mkdir -p gpurun_out/r4ai && export TMPDIR=/tmp && \
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4ai/pytest_gpu.log 2>&1
}

"call_${1:?usage: calls.sh <letter>}"
