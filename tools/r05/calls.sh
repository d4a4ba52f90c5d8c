#!/bin/bash
# The round-5 GPU calls, one function per call (the exact command each ran through gpurun, from the repo
# root): `bash tools/r05/calls.sh <letter>`. Their results are in profiles/r05_*; the libraries they name
# are built here by tools/r05/build_lib.sh (git-ignored).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"

# one bench line per library, alternating libraries within each round, on one box
ab_lines() {  # ab_lines OUTDIR ROUNDS "LIBS" "NAME ARGS" ... (LIB "cur" = the product library)
  local out=$1 rounds=$2 libs=$3; shift 3
  local specs=("$@") r lib spec name path
  for r in $(seq 1 "$rounds"); do for lib in $libs; do
    path=tools/r05/lib$lib.so; [ "$lib" = cur ] && path=netflow_amd/libnfcs.so
    for spec in "${specs[@]}"; do
      read -r name args <<< "$spec"
      NFCS_LIB=$path timeout -k 10 200 python3 -u bench.py $args --no-cpu --no-host --no-c4 --no-replay --no-mix \
        > "$out/${name}_${lib}_$r.json" 2>> "$out/bench.err" || return 1
    done
  done; done
}

call_a() {
  # round 5, GPU call a: the GPU tests on the product with per-slot zero lines (g_zero_pool), ring-wrapping
  # host bursts, scattered host frames (nfcs_update_host_frames) and tagged footprint samples; the new
  # default bench line (c3 / l3fwd_c3 / host_adapter sub-lines), then the zero-target A/B: round 4's
  # product (one 16-byte g_zero16),
  # per-slot lines at 128 B / 256 B / 4 KB strides, the 128-B form in three libraries whose data sections
  # differ (pads of 0 / 1536 / 2304 bytes move the pool by a page), and one aligned shared chunk; then
  # C3's write schedules of tools/r05/c3_exp.hip (write workgroups of sub-batch j-1 inside j's read pass).
  # (As it ran, ab_lines reset "$@" inside its loop: after the first library the A/B ran C1 lines under
  # wrong names; call b repeats the A/B. The tests, the bench line and the C3 forms are as listed.)
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5a && \
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5a/pytest.log 2>&1
  local rc=$?; [ $rc -le 1 ] || return $rc  # failed tests (1) still let the measurements run; nothing else does
  timeout -k 10 300 python3 -u bench.py > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err && \
  ab_lines gpurun_out/r5a 3 "nfcs_r4final z_s8 z_s8_p1536 z_s8_p2304 z_s16 z_s256 z_single" \
    "fwdc3 --op l3fwd --config 3 --steps 40" "c3 --config 3 --steps 40" && \
  timeout -k 10 200 python3 -u tools/r05/c3_forms.py --variants 0,1,2,3,4,5 --rounds 3 > gpurun_out/r5a/c3_forms.jsonl 2>&1
}


call_b() {
  # round 5, GPU call b: call a's zero-target A/B again (its loop had a shell bug): round 4's product
  # (one 16-byte g_zero16) against the product (per-slot zero lines), the product in two libraries whose
  # data sections differ (pads of 1536 / 2304 bytes move the pool by a page), per-slot lines at a 4 KB
  # stride and one page-aligned shared chunk; C1, C3 and the forward's C3 mix, alternating on one box.
  # Then the host paths with 8 and 16 copy threads (NFCS_HOST_THREADS)
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5b && \
  ab_lines gpurun_out/r5b 3 "nfcs_r4final cur cur_p1536 cur_p2304 z_s256 z_single" \
    "c1 --steps 50" "c3 --config 3 --steps 40" "fwdc3 --op l3fwd --config 3 --steps 40" && \
  for t in 8 16; do
    NFCS_HOST_THREADS=$t timeout -k 10 200 tests/cpp/_ref/netflow_adapter_test adapterbench 1048576 3 16 81cc3905092d7f44 \
      > gpurun_out/r5b/adapter_t$t.json 2> gpurun_out/r5b/adapter_t$t.err || exit 1
    NFCS_HOST_THREADS=$t timeout -k 10 300 python3 -u bench.py --no-cpu --no-replay --no-mix --steps 10 \
      > gpurun_out/r5b/bench_host_t$t.json 2>> gpurun_out/r5b/bench.err || exit 1
  done
}

call_c() {
  # round 5, GPU call c: the GPU tests on the product (past-frame lanes read the chunk of the same
  # instruction's first in-frame lane: no extra request), then the A/B: round 4's product (one 16-byte
  # g_zero16), the product, the product with its data section moved (2304-byte pad), past-frame lanes
  # aimed at the wave's row-0 frame start (NFCS_PAST=1) and at one page-aligned zero chunk (call b's
  # z_single); C1, C3, the forward's C3 mix and the C4 shard, alternating on one box; then the default line
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5c && \
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5c/pytest.log 2>&1
  local rc=$?; [ $rc -le 1 ] || return $rc
  ab_lines gpurun_out/r5c 3 "nfcs_r4final cur cur_p2304 past_row0 z_single" \
    "c1 --steps 50" "c3 --config 3 --steps 40" "fwdc3 --op l3fwd --config 3 --steps 40" "c4shard --packets 4194304 --steps 12" && \
  timeout -k 10 300 python3 -u bench.py > gpurun_out/r5c/bench.json 2> gpurun_out/r5c/bench.err
}

call_d() {
  # round 5, GPU call d: the GPU tests on the product (one 4 KB-aligned zero line, call c's outcome); where
  # the forward's C3-mix spread comes from (tools/r05/fwd_var.py: timing windows within one allocation
  # against fresh allocations, the update beside it), the product and its inline segment stores past the
  # caches (libfwd_nt); then the default bench line
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5d && \
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5d/pytest.log 2>&1
  local rc=$?; [ $rc -le 1 ] || return $rc
  timeout -k 10 300 python3 -u tools/r05/fwd_var.py --allocs 4 --windows 3 > gpurun_out/r5d/fwd_var_prod.jsonl 2> gpurun_out/r5d/fwd_var.err && \
  NFCS_LIB=tools/r05/libfwd_nt.so timeout -k 10 300 python3 -u tools/r05/fwd_var.py --allocs 4 --windows 3 > gpurun_out/r5d/fwd_var_nt.jsonl 2>> gpurun_out/r5d/fwd_var.err && \
  timeout -k 10 300 python3 -u tools/r05/fwd_var.py --allocs 3 --windows 3 --op update > gpurun_out/r5d/upd_var_prod.jsonl 2>> gpurun_out/r5d/fwd_var.err && \
  timeout -k 10 300 python3 -u bench.py > gpurun_out/r5d/bench.json 2> gpurun_out/r5d/bench.err
}

call_e() {
  # round 5, GPU call e: the GPU tests on the product (the forward's 8-lane rows store their segments past
  # the caches, call d's outcome); the product against the same with write-through segments (libfwd_wt)
  # on the forward's C3 mix and on 1M x 64-byte frames (its tiny shape), alternating; the default line
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5e && \
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5e/pytest.log 2>&1
  local rc=$?; [ $rc -le 1 ] || return $rc
  ab_lines gpurun_out/r5e 3 "cur fwd_wt" "fwdc3 --op l3fwd --config 3 --steps 40" \
    "fwdtiny --op l3fwd --config 0 --packets 1048576 --steps 40" && \
  timeout -k 10 300 python3 -u bench.py > gpurun_out/r5e/bench.json 2> gpurun_out/r5e/bench.err
}

call_f() {
  # round 5, GPU call f: the update's tiny shape (8-lane rows) storing past the caches instead of
  # write-through (libtiny_nt) on 1M x 64-byte frames, alternating; then rocprofv3 kernel stats of the
  # default line and of each line alone, PMC traffic per call (tools/r05/prof_all.sh) on the product
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5f && \
  ab_lines gpurun_out/r5f 3 "cur tiny_nt" "tiny --config 0 --packets 1048576 --steps 40" && \
  bash tools/r05/prof_all.sh r5f
}

call_g() {
  # round 5, GPU call g (run inline, not from this file): the GPU tests, smoke() and the default bench
  # line on the final product of session 2 (profiles/r05_g_*)
  cd /root/repo && mkdir -p gpurun_out/r5g && \
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5g/pytest.log 2>&1 && \
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5g/smoke.log 2>&1 && \
  timeout -k 10 240 python bench.py > gpurun_out/r5g/bench.json 2> gpurun_out/r5g/bench.err
}

call_h() {
  # round 5, GPU call h: the host path's staging copies with non-temporal stores (the product: the
  # scattered-frame gather and the pageable arena's staging copy) against plain memcpy (hostbase: the
  # sources before that change, built by build_lib.sh into tools/r05/hostbase/libnfcs.so); the host
  # GPU tests on the product first; then 3 alternating rounds of the adapter bench (1M C1 frames in
  # separate PacketBuffers, the adapter / BufferPool paths) and of bench.py's host sub-line
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5h && \
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    -k "host or adapter or pool or frames or ring" > gpurun_out/r5h/pytest.log 2>&1 || return 1
  local r lib dir
  for r in 1 2 3; do for lib in cur hostbase; do
    dir=netflow_amd; [ "$lib" = cur ] || dir=tools/r05/$lib
    LD_LIBRARY_PATH=$dir timeout -k 10 200 tests/cpp/_ref/netflow_adapter_test adapterbench 1048576 3 16 81cc3905092d7f44 \
      > gpurun_out/r5h/adapter_${lib}_$r.json 2>> gpurun_out/r5h/adapter.err || return 1
    NFCS_LIB=$dir/libnfcs.so timeout -k 10 300 python3 -u bench.py --no-cpu --no-replay --no-mix --no-c4 --steps 10 \
      > gpurun_out/r5h/host_${lib}_$r.json 2>> gpurun_out/r5h/bench.err || return 1
  done; done
  # (as it ran, --no-c4 also skipped the host sub-line: only the adapter bench measured; call i repeats)
}

call_i() {
  # round 5, GPU call i: call h again, with the host sub-line (bench.py without --no-c4; the line's C4
  # shard runs too) and the adapter bench, 3 alternating rounds of product / hostbase
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5i || return 1
  local r lib dir
  for r in 1 2 3; do for lib in cur hostbase; do
    dir=netflow_amd; [ "$lib" = cur ] || dir=tools/r05/$lib
    LD_LIBRARY_PATH=$dir timeout -k 10 200 tests/cpp/_ref/netflow_adapter_test adapterbench 1048576 3 16 81cc3905092d7f44 \
      > gpurun_out/r5i/adapter_${lib}_$r.json 2>> gpurun_out/r5i/adapter.err || return 1
    NFCS_LIB=$dir/libnfcs.so timeout -k 10 300 python3 -u bench.py --no-cpu --no-replay --no-mix --steps 10 \
      > gpurun_out/r5i/host_${lib}_$r.json 2>> gpurun_out/r5i/bench.err || return 1
  done; done
}

call_l() {
  # round 5, GPU call l (tools/r05/host_pipe and host_phases): the gather -> H2D pipeline without the
  # kernel overlaps (28.8 ms for 1M C1 frames against 33.1 H2D alone), the product call took 35.1 ms
  cd /root/repo && mkdir -p gpurun_out/r5l && \
  timeout -k 10 300 tools/r05/host_pipe 1048576 5 8 > gpurun_out/r5l/pipe.json 2> gpurun_out/r5l/pipe.err && \
  timeout -k 10 120 tools/r05/host_phases 1048576 5 > gpurun_out/r5l/phases.json 2> gpurun_out/r5l/phases.err
}

call_m() {
  # round 5, GPU call m: the host pipelines wait for a slot's copies in (`staged`) instead of its whole
  # chunk before staging the next one, validate scattered bursts over the workers and apply patch
  # records over the workers (the product) against the sources before (hostbase2); the host GPU tests
  # first; then 3 alternating rounds of host_phases, the adapter bench and bench.py's host sub-line
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5m && \
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    -k "host or adapter or pool or frames or ring" > gpurun_out/r5m/pytest.log 2>&1 || return 1
  local r lib dir
  for r in 1 2 3; do for lib in cur hostbase2; do
    dir=netflow_amd; [ "$lib" = cur ] || dir=tools/r05/$lib
    LD_LIBRARY_PATH=$dir timeout -k 10 120 tools/r05/host_phases 1048576 5 > gpurun_out/r5m/phases_${lib}_$r.json \
      2>> gpurun_out/r5m/phases.err || return 1
    LD_LIBRARY_PATH=$dir timeout -k 10 200 tests/cpp/_ref/netflow_adapter_test adapterbench 1048576 3 16 81cc3905092d7f44 \
      > gpurun_out/r5m/adapter_${lib}_$r.json 2>> gpurun_out/r5m/adapter.err || return 1
    NFCS_LIB=$dir/libnfcs.so timeout -k 10 300 python3 -u bench.py --no-cpu --no-replay --no-mix --steps 10 \
      > gpurun_out/r5m/host_${lib}_$r.json 2>> gpurun_out/r5m/bench.err || return 1
  done; done
}

call_n() {
  # round 5, GPU call n (run inline): the bench tests of the N = 1 line with its new `more` sub-lines
  # (child runs of C2, forward C1 / 4M, VLAN, flow keys), then the default line (profiles/r05_n_*)
  cd /root/repo && mkdir -p gpurun_out/r5n && \
  timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread -k "one_gpu" \
    > gpurun_out/r5n/pytest.log 2>&1 && \
  timeout -k 10 300 python bench.py > gpurun_out/r5n/bench.json 2> gpurun_out/r5n/bench.err
}

call_o() {
  # round 5, GPU call o: the fused forward's short-mix shape as 16-lane rows at 7 waves/SIMD (the
  # update's short shape) with buffer loads (libfwd16buf) or global loads (libfwd16), segment stores
  # past the caches (tools/r05/fwd16_exp.py), against the product's 8-lane rows of 12 slots; the
  # forward on the C3 mix, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5o && \
  ab_lines gpurun_out/r5o 3 "cur fwd16buf fwd16" "fwdc3 --op l3fwd --config 3 --steps 40"
}

call_r() {
  # round 5, GPU call r: the flow-key kernel's header-line loads with other cache policies (nt / sc1 /
  # sc0 sc1 / sc0 sc1 nt; tools/r05/fk_exp.py) against the default: 3 alternating rounds of the
  # flow-key line (C1 1M, 4 rotated batches, digest of the records), then per library the PMC
  # traffic of one call (tools/pmc_traffic.py: FETCH_SIZE, WRITE_SIZE, EA read requests incl. 32-byte)
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5r && \
  ab_lines gpurun_out/r5r 3 "cur fk_nt fk_sc1 fk_sc fk_scnt" "fk --op flowkey --steps 50" || return 1
  local lib path
  for lib in cur fk_nt fk_sc1 fk_sc fk_scnt; do
    path=tools/r05/lib$lib.so; [ "$lib" = cur ] && path=netflow_amd/libnfcs.so
    NFCS_LIB=$path timeout -k 10 200 python3 -u tools/pmc_traffic.py --out gpurun_out/r5r/pmc_$lib --configs 1 \
      --ops flowkey --steps 5 > gpurun_out/r5r/pmc_$lib.log 2>&1 || return 1
  done
}

call_s() {
  # round 5, GPU call s: load cache policies under rotation (tools/r05/pol_exp.py): the row kernels'
  # header slot non-temporal (upd_hdrnt), VLAN's loads non-temporal (vlan_nt; slots 1.. only:
  # vlan_nt1), against the product (flow keys' header loads already nt); C1, C3, the forward's C3
  # mix, VLAN C1, 3 alternating rounds; then the flow-key PMC traffic of the product (absolute library
  # paths: pmc_traffic runs rocprofv3 from /tmp)
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5s && \
  ab_lines gpurun_out/r5s 3 "cur upd_hdrnt vlan_nt vlan_nt1" "c1 --steps 50" "c3 --config 3 --steps 40" \
    "fwdc3 --op l3fwd --config 3 --steps 40" "vlan --op vlan --steps 24" && \
  NFCS_LIB=$PWD/netflow_amd/libnfcs.so timeout -k 10 200 python3 -u tools/pmc_traffic.py --out gpurun_out/r5s/pmc_cur \
    --configs 1 --ops flowkey --steps 5 > gpurun_out/r5s/pmc_cur.log 2>&1
}

call_t() {
  # round 5, GPU call t: rocprofv3 kernel stats of the flow-key line on the product with non-temporal
  # header loads, and of the default line (--no-ops: its child lines are profiled alone above)
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t && \
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r5t/flowkey" -o flowkey -- \
    python3 bench.py --op flowkey --steps 50 --no-cpu > gpurun_out/r5t/flowkey.json 2> gpurun_out/r5t/flowkey.err && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r5t/default" -o default -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --no-ops > gpurun_out/r5t/default.json 2> gpurun_out/r5t/default.err
}

call_v() {
  # round 5, GPU call v: store policies under rotation (tools/r05/pol_exp.py vlan_wt vlan_plain
  # fk_recplain): VLAN's long-frame rows write-through / plain instead of past the caches, flow-key
  # records plain instead of non-temporal; VLAN C1 and flow keys C1, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5v && \
  ab_lines gpurun_out/r5v 3 "cur vlan_wt vlan_plain fk_recplain" "vlan --op vlan --steps 24" "fk --op flowkey --steps 50"
}

call_w() {
  # round 5, GPU call w: the update's inline checksum-byte stores under rotation (tools/r05/pol_exp.py
  # c3_wt c3_plain): the short shape write-through instead of past the caches; every inline store
  # plain; C3, 1M x 64-byte frames (tiny shape) and C1, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5w && \
  ab_lines gpurun_out/r5w 3 "cur c3_wt c3_plain" "c3 --config 3 --steps 40" "tiny --config 0 --packets 1048576 --steps 40" "c1 --steps 50"
}

call_x() {
  # round 5, GPU call x: block orders (tools/r05/pol_exp.py wp_xcd fk_noxcd vlan_xcd): the write passes
  # in the read pass's XCD-aware order; flow keys in dispatch order; VLAN XCD-aware; C1, the C4 shard,
  # the forward on 4M frames (deferred: apply_fwd_kernel), flow keys, VLAN; 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5x && \
  ab_lines gpurun_out/r5x 3 "cur wp_xcd fk_noxcd vlan_xcd" "c1 --steps 50" "c4shard --packets 4194304 --steps 12" \
    "fwd4m --op l3fwd --packets 4194304 --steps 12" "fk --op flowkey --steps 50" "vlan --op vlan --steps 24"
}

call_y() {
  # round 5, GPU call y: the forward's short-mix segment stores plain instead of past the caches
  # (tools/r05/pol_exp.py fwd_plain); the forward on the C3 mix, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5y && \
  ab_lines gpurun_out/r5y 3 "cur fwd_plain" "fwdc3 --op l3fwd --config 3 --steps 40"
}

call_z() {
  # round 5, GPU call z: the row kernels' read pass and the write passes in dispatch order instead of
  # XCD-aware (tools/r05/pol_exp.py rp_noxcd); C1, C3, the C4 shard, the forward's C3 mix, 3 rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5z && \
  ab_lines gpurun_out/r5z 3 "cur rp_noxcd" "c1 --steps 50" "c3 --config 3 --steps 40" \
    "c4shard --packets 4194304 --steps 12" "fwdc3 --op l3fwd --config 3 --steps 40"
}

call_aa() {
  # round 5, GPU call aa: the update's short shape as 8-lane rows of 12 slots (the forward's short-mix
  # form; round 3 measured it 6% slower on a replayed batch), stores write-through (c3r8) or past the
  # caches (c3r8nt); C3 under rotation, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5aa && \
  ab_lines gpurun_out/r5aa 3 "cur c3r8 c3r8nt" "c3 --config 3 --steps 40"
}

call_ab() {
  # round 5, GPU call ab: flow keys with descriptors loaded non-temporally (fk_descnt) / hashes stored
  # non-temporally (fk_hashnt), against the product; C1 under rotation, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ab && \
  ab_lines gpurun_out/r5ab 3 "cur fk_descnt fk_hashnt" "fk --op flowkey --steps 50"
}

call_ac() {
  # round 5, GPU call ac: VERDICT r4 item 2's test on the final product: the forward's C3 mix (and the
  # update's C3) in the product and in two libraries whose data sections move g_zero_line by a page
  # (PAD 1536 / 2304, build_lib.sh), 4 alternating rounds, each line its own process
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ac && \
  ab_lines gpurun_out/r5ac 4 "cur cur_p1536 cur_p2304" "fwdc3 --op l3fwd --config 3 --steps 40" "c3 --config 3 --steps 40"
}

call_ad() {
  # round 5, GPU call ad: the update's short shape in 256-thread workgroups (c3_wg256; round 3 chose
  # one-wave workgroups on a replayed batch), C3 under rotation, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ad && \
  ab_lines gpurun_out/r5ad 3 "cur c3_wg256" "c3 --config 3 --steps 40"
}

call_ae() {
  # round 5, GPU call ae: the forward's short-mix rows in 256-thread workgroups (fwd_wg256), the
  # forward on the C3 mix under rotation, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ae && \
  ab_lines gpurun_out/r5ae 3 "cur fwd_wg256" "fwdc3 --op l3fwd --config 3 --steps 40"
}

call_af() {
  # round 5, GPU call af: call ae again with 6 alternating rounds (its 3 rounds fell in two modes)
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5af && \
  ab_lines gpurun_out/r5af 6 "cur fwd_wg256" "fwdc3 --op l3fwd --config 3 --steps 40"
}

call_ag() {
  # round 5, GPU call ag: rocprofv3 kernel stats of the lines whose kernels changed after call
  # r5final3 (the short shape's and the forward short-mix's 256-thread workgroups): C3, the forward
  # on the C3 mix, and the default line without its child lines
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ag && \
  for spec in "c3 --config 3 --steps 30 --no-cpu --no-replay --no-host --no-c4" \
              "l3fwd_c3 --op l3fwd --config 3 --steps 20 --no-cpu" \
              "default --steps 20 --warmup 5 --no-cpu --no-ops"; do
    read -r name args <<< "$spec"
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r5ag/$name" -o $name -- \
      python3 bench.py $args > gpurun_out/r5ag/$name.json 2> gpurun_out/r5ag/$name.err || return 1
  done
}

call_ah() {
  # round 5, GPU call ah: the long shape's continuation batches double-buffered (libdb: batch j+1's
  # loads issued before batch j is summed; 82 VGPRs, still 5 waves/SIMD) against the product before
  # (libpre_db); C2 (jumbo frames: 6 batches each), C1 and the C4 shard, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ah && \
  ab_lines gpurun_out/r5ah 3 "pre_db db" "c2 --config 2 --steps 20" "c1 --steps 50" "c4shard --packets 4194304 --steps 12"
}

call_ai() {
  # round 5, GPU call ai: the tiny shapes in 256-thread workgroups (tiny_wg256), 1M x 64-byte frames,
  # the update and the forward, under rotation, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5ai && \
  ab_lines gpurun_out/r5ai 3 "cur tiny_wg256" "tiny --config 0 --packets 1048576 --steps 40" \
    "fwdtiny --op l3fwd --config 0 --packets 1048576 --steps 40"
}

call_aj() {
  # round 5, GPU call aj: the forward's write pass (apply_fwd_kernel) with 2-byte stores write-through
  # (fwdwp_wt) or plain (fwdwp_plain) instead of past the caches; the forward on C1 and on 4M frames
  # (both deferred), 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5aj && \
  ab_lines gpurun_out/r5aj 3 "cur fwdwp_wt fwdwp_plain" "fwdc1 --op l3fwd --steps 40" \
    "fwd4m --op l3fwd --packets 4194304 --steps 12"
}

call_al() {
  # round 5, GPU call al: the short shape's inline byte stores with `nt` alone (c3_st_nt) / `sc1 nt`
  # (c3_st_sc1nt) instead of `sc0 sc1 nt`; C3 under rotation, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5al && \
  ab_lines gpurun_out/r5al 3 "cur c3_st_nt c3_st_sc1nt" "c3 --config 3 --steps 40"
}

call_an() {
  # round 5, GPU call an: the forward's deferred long-frame read pass with line-aligned windows in
  # every wave (fwd_lam1; round 3 measured it 1.3% slower on replayed 128-byte starts); the forward
  # on C1 and 4M frames under rotation, 3 alternating rounds
  cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5an && \
  ab_lines gpurun_out/r5an 3 "cur fwd_lam1" "fwdc1 --op l3fwd --steps 40" "fwd4m --op l3fwd --packets 4194304 --steps 12"
}

"call_$1"
