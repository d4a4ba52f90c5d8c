#!/bin/bash
# The round-6 GPU calls, one function per call (the exact command each ran through gpurun, from the repo
# root): `bash tools/r06/calls.sh <letter>`. Their results are in profiles/r06_*; the libraries they name
# are built here by tools/r05/build_lib.sh (git-ignored).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp

# one bench line per (library, spec), alternating within each round, on one box
ab_lines() {  # ab_lines OUTDIR ROUNDS "LIBS" "NAME ARGS" ... (LIB "cur" = the product library)
  local out=$1 rounds=$2 libs=$3; shift 3
  local specs=("$@") r lib spec name args path
  for r in $(seq 1 "$rounds"); do for lib in $libs; do
    path=tools/r06/lib$lib.so; [ "$lib" = cur ] && path=netflow_amd/libnfcs.so
    for spec in "${specs[@]}"; do
      read -r name args <<< "$spec"
      NFCS_LIB=$path timeout -k 10 200 python3 -u bench.py $args --no-cpu --no-host --no-c4 --no-replay --no-mix --no-ops \
        > "$out/${name}_${lib}_$r.json" 2>> "$out/bench.err" || return 1
    done
  done; done
}

call_a() {
  # round 6, GPU call a: packed C3 (16-byte frame starts) on the round-5 product, beside C3 at
  # 128-byte starts, alternating on one box; its rocprofv3 kernel stats; PMC traffic and instruction counts
  local o=gpurun_out/r6a; mkdir -p $o
  ab_lines $o 2 "cur" "c3p --config 3 --align 16 --steps 40" "c3 --config 3 --align 128 --steps 40" && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c3p -o p -- \
    python3 bench.py --config 3 --align 16 --steps 20 --no-cpu --no-host --no-c4 --no-replay > $o/prof_c3p.log 2>&1 && \
  PMC_GROUPS="FETCH_SIZE;WRITE_SIZE TCC_EA0_WRREQ_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
    bash tools/pmc.sh r6a/pmc_c3p --config 3 --align 16 --steps 10 --no-host --no-c4 --no-replay
}



call_b() {
  # round 6, GPU call b: packed C3 ran the tiny shape (8-lane rows: its 782-byte mean footprint is under
  # kTinyMeanBytes, call a); the same batches in the short and long shapes by slot hint, alternating
  local o=gpurun_out/r6b; mkdir -p $o
  ab_lines $o 2 "cur" "c3p_auto --config 3 --align 16 --steps 40" "c3p_short --config 3 --align 16 --steps 40 --slot-bytes 900" \
    "c3p_long --config 3 --align 16 --steps 40 --slot-bytes 1536" "c3a64 --config 3 --align 64 --steps 40" \
    "c3a64_short --config 3 --align 64 --steps 40 --slot-bytes 900"
}

call_c() {
  # round 6, GPU call c: the packed-mix shape rule (sample_footprint counts frames past one 8-lane row
  # pass; kTinyLongMax): the GPU tests of the launch shapes and the host ring; packed C3 by default shape
  # against the short-shape hint, alternating; the default bench line (its new c3_packed sub-line)
  local o=gpurun_out/r6c; mkdir -p $o
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_slot_hint.py tests/test_gpu_host_ring.py tests/test_gpu_abi_errors.py \
    -q -x --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 && \
  ab_lines $o 2 "cur" "c3p_auto --config 3 --align 16 --steps 40" "c3p_short --config 3 --align 16 --steps 40 --slot-bytes 900" \
    "l3c3p_auto --op l3fwd --config 3 --align 16 --steps 40" "l3c3_auto --op l3fwd --config 3 --align 128 --steps 40" && \
  timeout -k 10 400 python3 -u bench.py --no-ops > $o/bench_default.json 2> $o/bench_default.err
}

call_d() {
  # round 6, GPU call d: the per-RX-burst operating point: burstbench alone, then the
  # host lines of the default bench (host, host_adapter, host_bursts)
  local o=gpurun_out/r6d; mkdir -p $o
  timeout -k 10 300 tests/cpp/_ref/netflow_adapter_test burstbench 64,256,1024,4096,16384,65536 1048576 0.4 16 81cc3905092d7f44 \
    > $o/burstbench.json 2> $o/burstbench.err
}

call_e() {
  # round 6, GPU call e: burstbench's host-side fault of call d, with a stack dump and progress lines
  local o=gpurun_out/r6e; mkdir -p $o
  timeout -k 10 120 tests/cpp/_ref/netflow_adapter_test burstbench 256,4096 65536 0.1 16 ffffffffffffffff > $o/burstbench_small.json 2> $o/burstbench_small.err
  echo "rc=$?" >> $o/burstbench_small.err
}

call_f() {
  # round 6, GPU call f: direct chunks (no DMA for chunks of <= 2 MiB) and the lower host-copy split
  # thresholds: the host-path GPU tests, then burstbench per library (pre = before the change; d0 = the
  # change without direct chunks; d8 = direct chunks up to 8 MiB), alternating, two rounds
  local o=gpurun_out/r6f; mkdir -p $o
  timeout -k 10 500 python3 -u -m pytest tests/test_gpu_host_ring.py tests/test_gpu_abi_errors.py tests/test_netflow_adapter.py \
    tests/test_gpu_parity.py tests/test_gpu_large_arena.py -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || return 1
  local r lib exe
  for r in 1 2; do for lib in cur pre d0 d8; do
    exe=tests/cpp/_ref/netflow_adapter_test_$lib; [ $lib = cur ] && exe=tests/cpp/_ref/netflow_adapter_test
    timeout -k 10 300 $exe burstbench 64,256,1024,4096,16384,65536 1048576 0.4 16 81cc3905092d7f44 \
      > $o/burst_${lib}_$r.json 2> $o/burst_${lib}_$r.err || return 1
  done; done
}

call_g() {
  # round 6, GPU call g: the fused forward's bound on C3 (tools/r06/fwd_bound.py), its
  # issue / stall counters beside the update's C3; the per-rank roofline of the N > 1 line (2-rank test, a
  # 4-rank rehearsal on this one GPU); the default bench line with its host_bursts sub-line
  local o=gpurun_out/r6g; mkdir -p $o
  timeout -k 10 300 python3 -u tools/r06/fwd_bound.py --variants 0,1,2,3,4,5 --rounds 3 > $o/fwd_bound.jsonl 2> $o/fwd_bound.err && \
  PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD;SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
    bash tools/pmc.sh r6g/pmc_fwd_c3 --op l3fwd --config 3 --steps 10 --no-host --no-c4 --no-replay && \
  PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD;SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
    bash tools/pmc.sh r6g/pmc_upd_c3 --config 3 --steps 10 --no-host --no-c4 --no-replay && \
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dist.py -q -x --timeout 280 --timeout-method thread -k two_ranks_one_gpu > $o/pytest_dist.log 2>&1 && \
  NFCS_BENCH_DEVICE=0 timeout -k 10 300 python3 -u bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu > $o/bench_gpus4_one_box.json 2> $o/bench_gpus4.err && \
  timeout -k 10 500 python3 -u bench.py > $o/bench_default.json 2> $o/bench_default.err
}

call_h() {
  # round 6, GPU call h: every GPU test on the round-6 product; rocprofv3 stats of the default bench line
  # and of packed C3; PMC traffic of packed C3 in its new shape (merged into a copy of profiles/traffic.json)
  local o=gpurun_out/r6h; mkdir -p $o
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $o/pytest_gpu.log 2>&1 || return 1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$o/default" -o default -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --no-ops > $o/default.json 2> $o/default.err || return 1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$o/c3p" -o c3p -- \
    python3 bench.py --config 3 --align 16 --steps 30 --no-cpu --no-replay --no-host --no-c4 > $o/c3p.json 2> $o/c3p.err || return 1
  cp profiles/traffic.json $o/traffic_in.json
  timeout -k 10 600 python3 tools/pmc_traffic.py --out "$PWD/$o/pmc" --configs 3 --align 16 --merge "$PWD/$o/traffic_in.json" \
    > $o/pmc.log 2>&1
}

call_i() {
  # round 6, GPU call i: where a per-RX-burst call's time goes (tools/r06/host_lat.hip)
  local o=gpurun_out/r6i; mkdir -p $o
  timeout -k 10 120 tools/r06/host_lat > $o/host_lat.json 2> $o/host_lat.err
}

call_j() {
  # round 6, GPU call j: pinned bursts of <= 32 MiB run zero-copy by default, zero-copy descriptors and
  # statuses through the slot's pinned block: the host-path GPU tests, host_lat, then burstbench against the
  # library before the change (direct = git 4f91a02), alternating, two rounds
  local o=gpurun_out/r6j; mkdir -p $o
  timeout -k 10 500 python3 -u -m pytest tests/test_gpu_host_ring.py tests/test_gpu_abi_errors.py tests/test_netflow_adapter.py \
    tests/test_gpu_parity.py tests/test_gpu_large_arena.py tests/test_gpu_slot_hint.py -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || return 1
  timeout -k 10 120 tools/r06/host_lat > $o/host_lat.json 2> $o/host_lat.err || return 1
  local r lib exe
  for r in 1 2; do for lib in cur direct; do
    exe=tests/cpp/_ref/netflow_adapter_test_$lib; [ $lib = cur ] && exe=tests/cpp/_ref/netflow_adapter_test
    timeout -k 10 300 $exe burstbench 64,256,1024,4096,16384,65536 1048576 0.4 16 81cc3905092d7f44 \
      > $o/burst_${lib}_$r.json 2> $o/burst_${lib}_$r.err || return 1
  done; done
}

call_k() {
  # round 6, GPU call k: direct chunks signal completion through a host-mapped flag (nfcs::DoneReq) instead
  # of the event: host-path GPU tests; host_lat; burstbench against the library before (zc = git f873852);
  # the device lines C1 / C3 / forward C3 against it too (the kernel's early exit moved), alternating
  local o=gpurun_out/r6k; mkdir -p $o
  timeout -k 10 500 python3 -u -m pytest tests/test_gpu_host_ring.py tests/test_gpu_abi_errors.py tests/test_netflow_adapter.py \
    tests/test_gpu_parity.py tests/test_gpu_large_arena.py tests/test_gpu_slot_hint.py -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || return 1
  timeout -k 10 120 tools/r06/host_lat > $o/host_lat.json 2> $o/host_lat.err || return 1
  local r lib exe
  for r in 1 2; do for lib in cur zc; do
    exe=tests/cpp/_ref/netflow_adapter_test_$lib; [ $lib = cur ] && exe=tests/cpp/_ref/netflow_adapter_test
    timeout -k 10 300 $exe burstbench 64,256,1024,4096,16384,65536 1048576 0.4 16 81cc3905092d7f44 \
      > $o/burst_${lib}_$r.json 2> $o/burst_${lib}_$r.err || return 1
  done; done
  ab_lines $o 2 "cur zc" "c1 --steps 50" "c3 --config 3 --steps 40" "fwdc3 --op l3fwd --config 3 --steps 40"
}

call_l() {
  # round 6, GPU call l: the completion-flag kernel change against git f873852 on the device lines it might
  # move (the forward's C3 mix, C1), four alternating rounds
  local o=gpurun_out/r6l; mkdir -p $o
  ab_lines $o 4 "cur zc" "fwdc3 --op l3fwd --config 3 --steps 40" "c1 --steps 50"
}

call_m() {
  # round 6, GPU call m: every GPU test on the product after the host-path changes, then the default bench
  # line (the driver's command) and smoke()
  local o=gpurun_out/r6m; mkdir -p $o
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $o/pytest_gpu.log 2>&1 || return 1
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || return 1
  timeout -k 10 600 python3 -u bench.py > $o/bench_default.json 2> $o/bench_default.err
}

call_n() {
  # round 6, GPU call n: host chunk sizes for mid-size bursts — the product (chunks of >= 4 MiB, ~4 per
  # burst) against >= 2 MiB / 1 MiB / 512 KiB chunks, ~8 per burst (tools/r06/build_variant.sh), burstbench
  # with the pageable ring, alternating, two rounds
  local o=gpurun_out/r6n; mkdir -p $o
  local r lib exe
  for r in 1 2; do for lib in cur ch2m8 ch1m8 ch512k8; do
    exe=tests/cpp/_ref/netflow_adapter_test_$lib; [ $lib = cur ] && exe=tests/cpp/_ref/netflow_adapter_test
    timeout -k 10 300 $exe burstbench 256,1024,4096,16384,65536 1048576 0.3 16 81cc3905092d7f44 \
      > $o/burst_${lib}_$r.json 2> $o/burst_${lib}_$r.err || return 1
  done; done
}

call_o() {
  # round 6, GPU call o: every wave releases its own stores before signal_done's barrier (instead of lane 0
  # of the workgroup alone): the host-path and slot tests, host_lat, burstbench
  local o=gpurun_out/r6o; mkdir -p $o
  timeout -k 10 500 python3 -u -m pytest tests/test_gpu_host_ring.py tests/test_gpu_abi_errors.py tests/test_netflow_adapter.py \
    tests/test_gpu_parity.py tests/test_gpu_slot_hint.py -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || return 1
  timeout -k 10 120 tools/r06/host_lat > $o/host_lat.json 2> $o/host_lat.err || return 1
  timeout -k 10 300 tests/cpp/_ref/netflow_adapter_test burstbench 64,256,1024,4096,16384,65536 1048576 0.3 16 81cc3905092d7f44 \
      > $o/burst_cur_1.json 2> $o/burst_cur_1.err
}

call_p() {
  # round 6, GPU call p: host copy split per thread from 512 KiB (product) against 256 / 128 KiB, burstbench
  # alternating, two rounds
  local o=gpurun_out/r6p; mkdir -p $o
  local r lib exe
  for r in 1 2; do for lib in cur cp256k cp128k; do
    exe=tests/cpp/_ref/netflow_adapter_test_$lib; [ $lib = cur ] && exe=tests/cpp/_ref/netflow_adapter_test
    timeout -k 10 300 $exe burstbench 64,256,1024,4096,16384 1048576 0.3 16 81cc3905092d7f44 \
      > $o/burst_${lib}_$r.json 2> $o/burst_${lib}_$r.err || return 1
  done; done
}

call_q() {
  # round 6, GPU call q: frames longer than a staging slot in the arena host path (staged as their relevant
  # prefix): the host-path GPU tests
  local o=gpurun_out/r6q; mkdir -p $o
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host_ring.py tests/test_gpu_abi_errors.py \
    tests/test_netflow_adapter.py tests/test_gpu_large_arena.py -q -x --timeout 280 --timeout-method thread > $o/pytest.log 2>&1
}

call_r() {
  # round 6, GPU call r: where the forward's long-frame read pass loses 4% to the update's (C1, deferred
  # forms: update_rows_kernel<6,16,1,256,false,SF_DEFER,1,7> vs <6,16,7,256,true,SF_DEFER,2,7>): issue and
  # stall counters and fetched bytes per dispatch, both ops on C1
  local o=gpurun_out/r6r
  PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD;FETCH_SIZE;SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
    bash tools/pmc.sh r6r/pmc_fwd_c1 --op l3fwd --steps 20 --no-host --no-c4 --no-replay && \
  PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD;FETCH_SIZE;SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
    bash tools/pmc.sh r6r/pmc_upd_c1 --steps 20 --no-host --no-c4 --no-replay && \
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$o/prof_fwd_c1" -o p -- \
    python3 bench.py --op l3fwd --steps 30 --no-cpu > $o/prof_fwd_c1.json 2> $o/prof_fwd_c1.err
}

call_s() {
  # round 6, GPU call s: the round's evidence on the final kernels (tools/r06/prof_all.sh)
  bash tools/r06/prof_all.sh r6s
}

call_t() {
  # round 6, GPU call t: pinned arenas at interior / unaligned addresses (zero-copy by default only when
  # 16-byte aligned): the host-path GPU tests
  local o=gpurun_out/r6t; mkdir -p $o
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_host_ring.py tests/test_gpu_abi_errors.py tests/test_gpu_parity.py \
    -q -x --timeout 280 --timeout-method thread > $o/pytest.log 2>&1
}

call_u() {
  # round 6, GPU call u: BufferPool bursts spanning <= NFCS_HOST_ZERO_COPY_AUTO_BYTES go to nfcs_update_host
  # (zero-copy, the kernel reads only the frames) instead of the gather, whatever their slots' fill: the
  # host and adapter tests, then burstbench with the buffer_pool path against the header before
  # (poolpre: test binary built against git 9ba4fd5's packet.hpp), alternating, two rounds
  local o=gpurun_out/r6u; mkdir -p $o
  timeout -k 10 600 python3 -u -m pytest tests/test_netflow_adapter.py tests/test_cpp_api.py tests/test_gpu_host_ring.py \
    -q -x --timeout 280 --timeout-method thread > $o/pytest.log 2>&1 || return 1
  local r lib exe
  for r in 1 2; do for lib in cur poolpre; do
    exe=tests/cpp/_ref/netflow_adapter_test_$lib; [ $lib = cur ] && exe=tests/cpp/_ref/netflow_adapter_test
    timeout -k 10 300 $exe burstbench 64,256,1024,4096,16384,65536 1048576 0.3 16 81cc3905092d7f44 \
      > $o/burst_${lib}_$r.json 2> $o/burst_${lib}_$r.err || return 1
  done; done
}

call_v() {
  # round 6, GPU call v: the forward's deferred long-frame read pass without row_stage's sched_barrier
  # (nosb; measurement build) against the product: forward C1 and 4M, three alternating rounds
  local o=gpurun_out/r6v; mkdir -p $o
  ab_lines $o 3 "cur nosb" "fwdc1 --op l3fwd --steps 40" "fwd4m --op l3fwd --packets 4194304 --steps 20"
}

call_w() {
  # round 6, GPU call w: the N > 1 line's host_all_ranks sub-line (every rank's pinned C1 arena through
  # nfcs_update_host at once): the 2-rank one-GPU test, a 4-rank rehearsal
  local o=gpurun_out/r6w; mkdir -p $o
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dist.py -q -x --timeout 280 --timeout-method thread -k two_ranks > $o/pytest_dist.log 2>&1 && \
  NFCS_BENCH_DEVICE=0 timeout -k 10 300 python3 -u bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu > $o/bench_gpus4_one_box.json 2> $o/bench_gpus4.err
}
call_x() {
  # round 6, GPU call x: the launch-shape audit (tools/r06/shape_audit.py): 45 layouts (uniform lengths at
  # 16- / 128-byte starts, 2048-byte ring slots, bimodal / IMIX / uniform-range mixes), auto against every
  # shape forced by the slot hint, calls rotating over 2 batches
  local o=gpurun_out/r6x; mkdir -p $o
  timeout -k 10 120 python3 -u tools/r06/shape_audit.py $o/shape_audit_quick.jsonl --quick 2> $o/quick.err && \
  timeout -k 10 600 python3 -u tools/r06/shape_audit.py $o/shape_audit.jsonl 2> $o/full.err
}
call_y() {
  # round 6, GPU call y: the shape audit's threshold set (tools/r06/shape_audit.py --threshold): 64 / 1500-
  # and 64 / 1024-byte mixes by long fraction, U{64..hi}, mid-size frames in 2048 / 4096-byte ring slots
  # against the same frames packed at the same packet count; the main set for the fused forward
  local o=gpurun_out/r6y; mkdir -p $o
  timeout -k 10 400 python3 -u tools/r06/shape_audit.py $o/shape_audit_threshold.jsonl --threshold 2> $o/threshold.err && \
  timeout -k 10 400 python3 -u tools/r06/shape_audit.py $o/shape_audit_l3fwd.jsonl --l3fwd 2> $o/l3fwd.err
}
call_z() {
  # round 6, GPU call z: the shape audit found the fused forward faster in 8-lane rows of 6 slots (slot hint
  # 256) than in its long shape on 1280-1500-byte frames (call y); the bench's own forward lines (C1 1M,
  # 4M) and the update's C1 by slot hint (0 = the product's choice, 256, 1000), three alternating rounds;
  # then kTinyMixMeanBytes (mixes below a 512-byte mean stay on 8-lane rows): the slot-hint tests, the
  # audit's threshold set again
  local o=gpurun_out/r6z; mkdir -p $o
  ab_lines $o 3 "cur" "fwd_auto --op l3fwd --steps 40" "fwd_tiny --op l3fwd --steps 40 --slot-bytes 256" \
    "fwd_short --op l3fwd --steps 40 --slot-bytes 1000" \
    "fwd4m_auto --op l3fwd --packets 4194304 --steps 20" "fwd4m_tiny --op l3fwd --packets 4194304 --steps 20 --slot-bytes 256" \
    "upd_auto --steps 40" "upd_tiny --steps 40 --slot-bytes 256" && \
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_slot_hint.py -q -x --timeout 120 --timeout-method thread > $o/pytest_slot_hint.log 2>&1 && \
  timeout -k 10 400 python3 -u tools/r06/shape_audit.py $o/shape_audit_threshold_mix512.jsonl --threshold 2> $o/threshold.err
}
call_aa() {
  # round 6, GPU call aa: the forward's shapes on long frames by TCP share (shape_audit.py --fwdcheck
  # --l3fwd, TTL re-stamped before the warm-up instead of right before the timed calls), then the same
  # layouts for the update
  local o=gpurun_out/r6aa; mkdir -p $o
  for t in 0 0.5 1; do
    timeout -k 10 200 python3 -u tools/r06/shape_audit.py $o/fwdcheck_l3fwd_tcp$t.jsonl --fwdcheck --l3fwd --tcp $t 2>> $o/fwdcheck.err || return 1
  done
  for t in 0 1; do
    timeout -k 10 200 python3 -u tools/r06/shape_audit.py $o/fwdcheck_update_tcp$t.jsonl --fwdcheck --tcp $t 2>> $o/fwdcheck.err || return 1
  done
}
call_ab() {
  # round 6, GPU call ab: the forward check again with C1's and C3's own generated frames beside the audit's
  # random-payload ones (the audit timed the forward's long shape 12% slower than bench.py does)
  local o=gpurun_out/r6ab; mkdir -p $o
  timeout -k 10 200 python3 -u tools/r06/shape_audit.py $o/fwdcheck_l3fwd_gen.jsonl --fwdcheck --l3fwd --tcp 0 2> $o/fwdcheck.err && \
  timeout -k 10 200 python3 -u tools/r06/shape_audit.py $o/fwdcheck_update_gen.jsonl --fwdcheck --tcp 0 2>> $o/fwdcheck.err
}
call_ac() {
  # round 6, GPU call ac: C1's own frames with some of the audit's header bytes on top (IP ID / flags zero,
  # DF set, the whole stamp), forward and update, all shapes
  local o=gpurun_out/r6ac; mkdir -p $o
  timeout -k 10 200 python3 -u tools/r06/shape_audit.py $o/fwdbytes_l3fwd.jsonl --fwdbytes --l3fwd --tcp 0 2> $o/fwdbytes.err && \
  timeout -k 10 200 python3 -u tools/r06/shape_audit.py $o/fwdbytes_update.jsonl --fwdbytes --tcp 0 2>> $o/fwdbytes.err
}
call_ad() {
  # round 6, GPU call ad: the forward's long shape 13-22% slower after header stamps that rewrite bytes with
  # the values they hold (call ac, equal digests): rocprofv3 kernel stats of C1's own frames against the
  # TTL-stamped ones, one process each — kernel time or idle time between the calls?
  local o=gpurun_out/r6ad; mkdir -p $o
  for l in C1_generated C1_stamp_ttl; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_$l -o p -- \
      python3 -u tools/r06/shape_audit.py $o/fwd_$l.jsonl --fwdbytes --l3fwd --tcp 0 --only $l > $o/prof_$l.log 2>&1 || return 1
  done
}
call_ae() {
  # round 6, GPU call ae: order or stamp? The same layouts in the reverse order in one process
  # (stamped first), then alternating
  local o=gpurun_out/r6ae; mkdir -p $o
  timeout -k 10 300 python3 -u tools/r06/shape_audit.py $o/fwd_order.jsonl --fwdbytes --l3fwd --tcp 0 \
    --only C1_stamp_ttl,C1_generated,C1_stamp_ttl,C1_generated,uniform1500_1M,C1_generated 2> $o/fwd_order.err
}
call_af() {
  # round 6, GPU call af: stamped frames stay slow for the forward's long shape in any order (call ae);
  # the TTL stamp followed by a whole-line rewrite of the arena (copy out and back)
  local o=gpurun_out/r6af; mkdir -p $o
  timeout -k 10 300 python3 -u tools/r06/shape_audit.py $o/fwd_rw.jsonl --fwdbytes --l3fwd --tcp 0 \
    --only C1_generated,C1_stamp_ttl,C1_stamp_ttl_rw,C1_generated,C1_stamp_ttl_rw 2> $o/fwd_rw.err
}
call_ag() {
  # round 6, GPU call ag: frames built on the host and uploaded whole (--host-gen) against C1's own generated
  # frames, forward: do DMA-written frames behave like the generator's?
  local o=gpurun_out/r6ag; mkdir -p $o
  timeout -k 10 300 python3 -u tools/r06/shape_audit.py $o/fwd_hostgen.jsonl --fwdbytes --l3fwd --tcp 0 --host-gen \
    --only C1_generated,uniform1500_1M,C1_generated,uniform1500_1M 2> $o/fwd_hostgen.err
}
call_ah() {
  # round 6, GPU call ah: one set of buffers, the frames reset by the generator alone / + a torch TTL stamp /
  # + a torch whole-arena copy, forward long shape and 8-lane rows (tools/r06/fwd_state.py)
  local o=gpurun_out/r6ah; mkdir -p $o
  timeout -k 10 300 python3 -u tools/r06/fwd_state.py > $o/fwd_state.jsonl 2> $o/fwd_state.err
}
call_ai() {
  # round 6, GPU call ai: after kTinyMixMeanBytes — the whole GPU suite, smoke(), the default bench line
  local o=gpurun_out/r6ai; mkdir -p $o
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $o/pytest_gpu.log 2>&1 && \
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && \
  timeout -k 10 600 python3 -u bench.py > $o/bench_default.json 2> $o/bench_default.err
}
call_aj() {
  # round 6, GPU call aj: VLAN push/pop on the mixes kTinyMixMeanBytes moved to 8-lane rows (the rule is
  # shared by every launch), auto against each VLAN shape by hint (shape_audit.py --vlanset --vlan)
  local o=gpurun_out/r6aj; mkdir -p $o
  timeout -k 10 400 python3 -u tools/r06/shape_audit.py $o/vlan_audit.jsonl --vlanset --vlan 2> $o/vlan_audit.err
}
call_ak() {
  # round 6, GPU call ak: VLAN push/pop shapes by frame alignment: uniform 128-1024 B, IMIX, 64/1500 and
  # U{64..hi} mixes at 16- and 128-byte starts, 2 KiB ring slots (shape_audit.py --vlanset2 --vlan)
  local o=gpurun_out/r6ak; mkdir -p $o
  timeout -k 10 500 python3 -u tools/r06/shape_audit.py $o/vlan_audit2.jsonl --vlanset2 --vlan 2> $o/vlan_audit2.err
}
call_al() {
  # round 6, GPU call al: VLAN's 8-lane store policy from the sample's new bits (frames off their lines,
  # varying lengths -> write-through): the slot-hint and VLAN GPU tests, the VLAN audit sets again, the
  # VLAN C1 bench line
  local o=gpurun_out/r6al; mkdir -p $o
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_slot_hint.py tests/test_gpu_vlan.py -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 && \
  timeout -k 10 500 python3 -u tools/r06/shape_audit.py $o/vlan_audit2.jsonl --vlanset2 --vlan 2> $o/vlan_audit2.err && \
  timeout -k 10 300 python3 -u tools/r06/shape_audit.py $o/vlan_audit.jsonl --vlanset --vlan 2> $o/vlan_audit.err && \
  timeout -k 10 200 python3 -u bench.py --op vlan --steps 40 --no-cpu --no-host --no-c4 --no-replay --no-mix --no-ops > $o/bench_vlan.json 2> $o/bench_vlan.err
}
call_am() {
  # round 6, GPU call am: kVlanMixMeanBytes (VLAN keeps mixes on write-through 8-lane rows up to a 640-byte
  # mean): the same tests, audits and VLAN C1 line as call al
  local o=gpurun_out/r6am; mkdir -p $o
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_slot_hint.py tests/test_gpu_vlan.py -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 && \
  timeout -k 10 500 python3 -u tools/r06/shape_audit.py $o/vlan_audit2.jsonl --vlanset2 --vlan 2> $o/vlan_audit2.err && \
  timeout -k 10 300 python3 -u tools/r06/shape_audit.py $o/vlan_audit.jsonl --vlanset --vlan 2> $o/vlan_audit.err && \
  timeout -k 10 200 python3 -u bench.py --op vlan --steps 40 --no-cpu --no-host --no-c4 --no-replay --no-mix --no-ops > $o/bench_vlan.json 2> $o/bench_vlan.err
}
call_an() {
  # round 6, GPU call an: the fused forward on the threshold set (64/1500, 64/1024 mixes, U{64..hi}, ring
  # slots) with kTinyMixMeanBytes in place: 8-lane rows against the short-mix rows on mixes
  local o=gpurun_out/r6an; mkdir -p $o
  timeout -k 10 500 python3 -u tools/r06/shape_audit.py $o/fwd_threshold.jsonl --threshold --l3fwd 2> $o/fwd_threshold.err
}
call_ao() {
  # round 6, GPU call ao: after the VLAN store rule — the whole GPU suite, smoke(), the default bench line,
  # and rocprofv3 kernel stats of the C1 line
  local o=gpurun_out/r6ao; mkdir -p $o
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $o/pytest_gpu.log 2>&1 && \
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && \
  timeout -k 10 600 python3 -u bench.py > $o/bench_default.json 2> $o/bench_default.err && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c1 -o p -- \
    python3 bench.py --steps 20 --no-cpu --no-host --no-c4 --no-replay --no-mix --no-ops > $o/prof_c1.log 2>&1
}
call_ap() {
  # round 6, GPU call ap: mid-size frames of one length in a ring -> 8-lane rows (peek_shape ring_rows8): the
  # slot-hint and line-window tests, the threshold audit for the update and the forward
  local o=gpurun_out/r6ap; mkdir -p $o
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_slot_hint.py tests/test_gpu_line_windows.py -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 && \
  timeout -k 10 400 python3 -u tools/r06/shape_audit.py $o/upd_threshold.jsonl --threshold 2> $o/upd_threshold.err && \
  timeout -k 10 400 python3 -u tools/r06/shape_audit.py $o/fwd_threshold.jsonl --threshold --l3fwd 2> $o/fwd_threshold.err
}
call_aq() {
  # round 6, GPU call aq: after the ring rule — the whole GPU suite, smoke(), the default bench line
  local o=gpurun_out/r6aq; mkdir -p $o
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $o/pytest_gpu.log 2>&1 && \
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && \
  timeout -k 10 600 python3 -u bench.py > $o/bench_default.json 2> $o/bench_default.err
}
call_ar() {
  # round 6, GPU call ar: the forward keeps bimodal mixes (hardly any frames between minimum and full size,
  # kObsMidShift) on 8-lane rows of 6 slots: slot-hint and L3 tests, the forward's threshold and main
  # audit sets, the default line's C3 sub-lines (no host / CPU legs)
  local o=gpurun_out/r6ar; mkdir -p $o
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_slot_hint.py tests/test_gpu_l3.py -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 && \
  timeout -k 10 400 python3 -u tools/r06/shape_audit.py $o/fwd_threshold.jsonl --threshold --l3fwd 2> $o/fwd_threshold.err && \
  timeout -k 10 400 python3 -u tools/r06/shape_audit.py $o/fwd_main.jsonl --l3fwd 2> $o/fwd_main.err && \
  timeout -k 10 400 python3 -u bench.py --no-cpu --no-host --no-ops > $o/bench_mix.json 2> $o/bench_mix.err
}
call_as() {
  # round 6, GPU call as: after the forward's bimodal rule — the whole GPU suite, smoke(), the default line
  local o=gpurun_out/r6as; mkdir -p $o
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $o/pytest_gpu.log 2>&1 && \
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && \
  timeout -k 10 600 python3 -u bench.py > $o/bench_default.json 2> $o/bench_default.err
}
call_at() {
  # round 6, GPU call at: the forward samples packed mid-size bursts and runs frames of one length on their
  # lines in 8-lane rows: slot-hint and L3 tests, the forward's main and threshold audits, the C3 sub-lines
  local o=gpurun_out/r6at; mkdir -p $o
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_slot_hint.py tests/test_gpu_l3.py -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 && \
  timeout -k 10 400 python3 -u tools/r06/shape_audit.py $o/fwd_threshold.jsonl --threshold --l3fwd 2> $o/fwd_threshold.err && \
  timeout -k 10 400 python3 -u tools/r06/shape_audit.py $o/fwd_main.jsonl --l3fwd 2> $o/fwd_main.err && \
  timeout -k 10 400 python3 -u bench.py --no-cpu --no-host --no-ops > $o/bench_mix.json 2> $o/bench_mix.err
}
call_au() {
  # round 6, GPU call au: C3 and the forward's C3 mix on the product against the libraries at the round's
  # start (r6start) and after the VLAN rule (vlanrule; tools/r06/build_lib_commit.sh), three alternating
  # rounds on one box: did the round's shape rules cost the BASELINE mix lines anything?
  local o=gpurun_out/r6au; mkdir -p $o
  ab_lines $o 3 "cur r6start vlanrule" "c3 --config 3 --steps 40" "l3c3 --op l3fwd --config 3 --steps 40"
}
call_av() {
  # round 6, GPU call av: after the forward's packed mid-size rule — the whole GPU suite, smoke(), the
  # default bench line
  local o=gpurun_out/r6av; mkdir -p $o
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $o/pytest_gpu.log 2>&1 && \
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && \
  timeout -k 10 600 python3 -u bench.py > $o/bench_default.json 2> $o/bench_default.err
}
call_aw() {
  # round 6, GPU call aw: the round's evidence again on the final product (after the shape rules; same
  # kernels for every BASELINE line): tools/r06/prof_all.sh
  bash tools/r06/prof_all.sh r6aw
}
call_ax() {
  # round 6, GPU call ax: the N > 1 line as the driver's 8-GPU run will produce it, rehearsed with 8 ranks on
  # this one GPU (per-rank fractions and digests, host_all_ranks with 8 pinned arenas)
  local o=gpurun_out/r6ax; mkdir -p $o
  NFCS_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --gpus 8 --steps 3 --warmup 1 --no-cpu > $o/bench_gpus8_one_box.json 2> $o/bench_gpus8.err
}
call_ay() {
  # round 6, GPU call ay: the slot-hint tests with the new ring-rule test
  local o=gpurun_out/r6ay; mkdir -p $o
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_slot_hint.py -v -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
}
call_az() {
  # round 6, GPU call az: the whole GPU suite with the ring-rule test, smoke()
  local o=gpurun_out/r6az; mkdir -p $o
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $o/pytest_gpu.log 2>&1 && \
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
}
"call_$1"
