#!/usr/bin/env python3
"""bench.py — device-resident batched checksum throughput (BASELINE.json metric).

A "step" is one pass of the hot path — NetFlow++'s Packet::update_checksums()
(packet.hpp:722-890), batched on the gfx950 engine — over one batch of synthetic frames that
is already resident in HBM. At N=1 the workload is BASELINE config C1 (1 M x 1500 B IPv4+UDP
on 1 MI355X); with --gpus N > 1 it is BASELINE config C4 (32 M x 1500 B sharded across 8 GPUs):
each rank owns its own batch of 4 M packets (packets [rank*n, (rank+1)*n)), so per-GPU work is
fixed (weak scaling) and there is no collective on the data path: ranks only meet at the
timing barriers.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1] [--packets n] [--no-cpu]
                  [--op update|l3fwd|flowkey]

--op l3fwd measures the fused transit-IPv4 forward instead (TTL--, MAC rewrite,
update_checksums; nfcs_l3_forward_device) on C1 with next hop i % 9 (8 = no route).
--op flowkey measures PacketClassifier::extract_flow_key + hash_flow (SURVEY.md §8 f4;
nfcs_flow_keys_device: 64-byte records + u32 hashes) in packets/s.

Prints ONE JSON line on rank 0. `value` = sum over ranks of frame bytes per step / the max
over ranks of the timed wall time per step. `roofline` uses the kernel's HIP-event time on its
own stream; `cpu_baseline` times the reference update_checksums() (oracle/_ref, compiled from
/root/reference) or, if that .so is absent, the oracle port, on a bounded sample on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import netflow_amd as nf  # noqa: E402

SEED = 20250620
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip parameters)
# measured on the MI355X box (tools/stream_read.hip, tools/stream_rw.hip; profiles/r01_stream_microbench.md):
STREAM_READ_GBPS = 7007.0  # best read-only stream (nt loads)
STREAM_RW_GBPS = 4839.0    # best read stream with one in-place store per 1536-byte frame
DEFAULT_PACKETS = {0: 1024, 1: 1 << 20, 2: 1 << 20, 3: 1 << 22}
C4_PACKETS_PER_GPU = 1 << 22
# bench.py --packets 4194304 on one MI355X, session 4: 5218.8 / 5399.6 / 5424.6 GB/s on three
# boxes (profiles/r01_s4_bench_c4_shard_1gpu*.json); the median
C4_SHARD_1GPU_GBPS = 5399.6
WORKLOAD = {
    0: "C0: 1024 x 64 B IPv4 (header checksum only)",
    1: "C1: 1M x 1500 B IPv4+UDP, device-resident",
    2: "C2: 1M x 9000 B IPv4+TCP jumbo, device-resident",
    3: "C3: 4M x U{64..1500} B IPv4 TCP/UDP mix, device-resident",
}
WORKLOAD_C4 = ("C4: 1500 B IPv4+UDP sharded as independent per-GPU batches, 4M packets per GPU "
               "(32M over 8 GPUs), device-resident")


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


class Dist:
    """Barrier + max-over-ranks. Uses torch.distributed (RCCL via backend 'nccl' when GPUs
    are visible to torch, else gloo); a no-op at world size 1."""

    def __init__(self, ws, rank, local):
        self.ws, self.rank, self.local = ws, rank, local
        self.pg = None
        if ws > 1:
            import torch
            import torch.distributed as dist
            backend = os.environ.get("NFCS_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
            if backend == "nccl":
                torch.cuda.set_device(local)
            dist.init_process_group(backend=backend)
            self.dist, self.torch, self.backend = dist, torch, backend

    def _t(self, v):
        t = self.torch.tensor([float(v)], dtype=self.torch.float64)
        return t.cuda() if self.backend == "nccl" else t

    def barrier(self):
        if self.ws > 1:
            self.dist.all_reduce(self._t(0.0))

    def max(self, v: float) -> float:
        if self.ws == 1:
            return float(v)
        t = self._t(v)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v: float) -> float:
        if self.ws == 1:
            return float(v)
        t = self._t(v)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.ws > 1:
            self.dist.destroy_process_group()


def device_sync():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass


def shard(rank: int, n_per_rank: int) -> tuple[int, int]:
    """Packet index range of a rank (weak scaling: every rank owns n_per_rank packets)."""
    return rank * n_per_rank, n_per_rank


def golden_digest(config: int, first: int, n: int):
    try:
        g = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))
    except OSError:
        return None
    c = g["configs"].get(str(config))
    if c and c["first"] == first and c["n"] == n:
        return c["digest_out"]
    if config == 1:
        for sh in g.get("c1_rank_shards", []) + g.get("c4_rank_shards", []):
            if sh["first"] == first and sh["n"] == n:
                return sh["digest_out"]
    return None


def golden_l3():
    try:
        g = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))
    except OSError:
        return None
    return g.get("l3fwd_c1")


def cpu_baseline(config: int, threads: int, min_seconds: float = 10.0, op: str = "update"):
    """Reference update_checksums() on host cores over a bounded sample of the workload."""
    try:
        import oracle
    except Exception as e:  # pragma: no cover
        return {"value": None, "error": repr(e)}
    kind = "reference" if oracle.ref_available() else "port"
    # at least ~1.2 GB so the sample streams from DRAM like the GPU batch, not from a large L3
    n = {0: 1024, 1: 1 << 20, 2: 1 << 17, 3: 1 << 21}[config]
    arena, desc = oracle.gen_config(config, SEED, 0, n)
    nbytes = float(desc["len"].astype(np.float64).sum())
    recs = hashes = None
    if op == "flowkey":
        recs = np.zeros((n, 64), dtype=np.uint8)
        hashes = np.zeros(n, dtype=np.uint32)
        if kind == "reference":
            R = oracle.ref()
            run = lambda: R.nfref_flow_keys_batch(oracle._ptr(arena), desc.ctypes.data, n,
                                                  oracle._ptr(recs), oracle._ptr(hashes, oracle._u32p),
                                                  threads)
        else:
            L = oracle.lib()
            run = lambda: L.nfo_flow_keys_batch(oracle._ptr(arena), arena.nbytes, desc.ctypes.data, n,
                                                oracle._ptr(recs), oracle._ptr(hashes, oracle._u32p))
            threads = 1
    elif op == "vlan":
        # push_vlan(100, 3) / pop_vlan() alternately (each pass leaves the batch ready for the
        # next), 1536-byte buffers: the frames are laid out 128-byte aligned as on the GPU
        arena, desc = oracle.gen_config(config, SEED, 0, n, 128)
        ops = [np.full(n, oracle.vlan_op("push", 100, 3), np.uint32),
               np.full(n, oracle.vlan_op("pop"), np.uint32)]
        flip = [0]
        if kind == "reference":
            R = oracle.ref()

            def run():
                R.nfref_vlan_batch(oracle._ptr(arena), desc.ctypes.data,
                                   oracle._ptr(ops[flip[0]], oracle._u32p), n, 1536, threads)
                flip[0] ^= 1
        else:
            def run():
                oracle.vlan_batch(arena, desc, ops[flip[0]], None, cap_all=1536)
                flip[0] ^= 1
            threads = 1
    elif op == "l3fwd":
        g = golden_l3()
        table = np.frombuffer(bytes.fromhex(g["table"]), dtype=np.uint8).copy()
        nh = (np.arange(n) % 9).astype(np.uint32)
        if kind == "reference":
            R = oracle.ref()
            run = lambda: R.nfref_l3_forward_batch(oracle._ptr(arena), desc.ctypes.data,
                                                   oracle._ptr(nh, oracle._u32p), n,
                                                   oracle._ptr(table), 8, threads)
        else:
            L = oracle.lib()
            run = lambda: L.nfo_l3_forward_batch(oracle._ptr(arena), arena.nbytes, desc.ctypes.data,
                                                 oracle._ptr(nh, oracle._u32p), n,
                                                 oracle._ptr(table), 8, None)
            threads = 1
    elif kind == "reference":
        R = oracle.ref()
        run = lambda: R.nfref_update_batch(oracle._ptr(arena), desc.ctypes.data, n, threads)
    else:
        L = oracle.lib()
        run = lambda: L.nfo_update_batch(oracle._ptr(arena), arena.nbytes, desc.ctypes.data, n,
                                         None, None, threads)
    # l3fwd mutates TTLs (each pass forwards once): restore the frames before every pass,
    # outside the timed part
    pristine = arena.copy() if op == "l3fwd" else None
    run()  # warm
    reps, el = 0, 0.0
    while el < min_seconds:
        if pristine is not None:
            np.copyto(arena, pristine)
        t0 = time.perf_counter()
        run()
        el += time.perf_counter() - t0
        reps += 1
    gbs = nbytes * reps / el / 1e9
    if op == "flowkey":
        return {"value": round(n * reps / el / 1e6, 3), "unit": "Mpkt/s", "cores": threads,
                "kind": kind, "sample": f"{n} packets of config C{config} x {reps} passes, "
                                        f"{threads} threads, g++ -O2, {el:.1f} s"}
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": threads, "kind": kind,
            "sample": f"{n} packets of config C{config} ({nbytes / 1e6:.0f} MB) x {reps} passes, "
                      f"{threads} threads, g++ -O2, {el:.1f} s"}


def load_traffic(config: int, n: int, op: str = "update"):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py),
    for the default batch size of the config; None otherwise."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        t = json.load(open(p)).get(f"C{config}" + ("" if op == "update" else f"_{op}"))
    except (OSError, ValueError):
        return None
    if not t or n != DEFAULT_PACKETS[config]:
        return None
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=1, choices=[0, 1, 2, 3])
    ap.add_argument("--packets", type=int, default=0, help="packets per GPU (default: config size)")
    ap.add_argument("--align", type=int, default=128,
                    help="frame start alignment in the arena: 128 = one L2 line per frame start, as "
                         "NIC/DPDK buffer rings lay frames out (16 = densely packed)")
    ap.add_argument("--warm-seconds", type=float, default=0.5,
                    help="minimum untimed warm-up time (on top of --warmup steps)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--op", choices=["update", "l3fwd", "flowkey", "vlan"], default="update")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    args = ap.parse_args()

    ws, rank, local = dist_env()
    D = Dist(ws, rank, local)
    n = args.packets or DEFAULT_PACKETS[args.config]
    c4 = ws > 1 and args.config == 1 and not args.packets
    if c4:  # BASELINE C4: 32M x 1500 B over 8 GPUs = 4M packets per GPU (also at 2 and 4 GPUs)
        n = C4_PACKETS_PER_GPU
    first, n = shard(rank, n)

    # NFCS_BENCH_DEVICE pins every rank to one device: rehearsing the N-rank path on a 1-GPU box
    eng = nf.Engine(int(os.environ.get("NFCS_BENCH_DEVICE", local)))
    d_arena, nbytes, d_desc, hdesc = eng.config_batch(args.config, SEED, first, n, args.align)
    frame_bytes = float(hdesc["len"].astype(np.float64).sum())
    algo_bytes = frame_bytes + 12.0 * n  # + 2x2 B checksum writes + 8 B descriptor per packet
    l3 = args.op == "l3fwd"
    if l3:
        # every launch decrements TTL (64 in the generator): K + 1 launches per fresh batch
        if args.steps > 60:
            raise SystemExit("--op l3fwd: --steps <= 60 (TTL 64 runs out after 63 forwards)")
        g3 = golden_l3()
        table = np.frombuffer(bytes.fromhex(g3["table"]), dtype=np.uint8).copy()
        d_tab = eng.alloc(table.nbytes).upload(table)
        d_nh = eng.alloc(4 * n).upload(((np.arange(first, first + n)) % 9).astype(np.uint32))
        algo_bytes = frame_bytes + 37.0 * n  # + 4 csum + 12 MAC + 1 TTL written, 8 desc + 4 nh + 8 table read
        step = lambda: eng.l3_forward_device(d_arena, nbytes, d_desc, d_nh, n, d_tab, 8)
        regen = lambda: (eng.gen_config_device(args.config, SEED, first, n, d_arena, nbytes, d_desc),
                         eng.sync())
    elif args.op == "flowkey":
        d_keys = eng.alloc(64 * n)
        d_hash = eng.alloc(4 * n)
        # moved per packet: the header line (min(len, 128) bytes) + 8 B descriptor read,
        # 64 B record + 4 B hash written
        hdr = float(np.minimum(hdesc["len"].astype(np.float64), 128.0).sum())
        algo_bytes = hdr + 76.0 * n
        step = lambda: eng.flow_keys_device(d_arena, nbytes, d_desc, n, d_keys, d_hash)
        regen = lambda: None
    elif args.op == "vlan":
        if args.config != 1:
            raise SystemExit("--op vlan: config 1 (1536-byte buffers per 1500-byte frame)")
        # push_vlan(100, 3) and pop_vlan() alternate, each on every frame; per packet the pass
        # reads the frame, writes it back from byte 12 (moved by 4 bytes) and updates its length:
        # push 2*len + 4 B, pop (len' = len + 4) 2*len' - 4 B; +8 B descriptor read, 4 B written
        VPUSH, VCAP = nf.vlan_push_op(100, 3), 1536
        flip = [0]

        def step():
            eng.vlan_device(d_arena, nbytes, d_desc, n, None, VPUSH if flip[0] == 0 else nf.VLAN_POP,
                            None, VCAP)
            flip[0] ^= 1
        algo_bytes = 2.0 * frame_bytes + 4.0 * n + 12.0 * n
        regen = lambda: step() if flip[0] else None  # back to untagged frames (pop)
    else:
        step = lambda: eng.update_device(d_arena, nbytes, d_desc, n)
        regen = lambda: None

    # torch (for the synchronize around the timed region) is imported and initialised before
    # the warm-up: its first import takes ~1.5 s, and an idle GPU between warm-up and timed
    # region re-enters the timed steps cold (rocprofv3 trace: C3 kernels 0.78 -> 0.99 ms)
    device_sync()
    # untimed warm-up: W steps, continued until --warm-seconds have passed so the timed steps
    # run at the clock the GPU holds under this load (a cold start measured ~4% slower)
    tw = time.perf_counter()
    done = 0
    while done < args.warmup or time.perf_counter() - tw < args.warm_seconds:
        step()
        done += 1
        if done % 16 == 0:
            eng.sync()
    eng.sync()
    regen()  # l3fwd: fresh TTLs for the timed steps

    # timed region: barrier + device sync on both sides, max over ranks
    D.barrier()
    device_sync()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    device_sync()
    t1 = time.perf_counter()
    D.barrier()
    wall = D.max(t1 - t0)
    ms_per_step = wall / args.steps * 1e3
    total_frame_bytes = D.sum(frame_bytes)

    # kernel duration with HIP events on the launch stream (roofline), same launches
    if l3:
        regen()
        ev_ms = eng.time_l3_forward_device(d_arena, nbytes, d_desc, d_nh, n, d_tab, 8,
                                           args.steps) / args.steps
        # parity: one forward of a fresh batch vs the reference's digest (C1, rank 0 shard)
        regen()
        step()
        eng.sync()
        want = g3["digest_out"] if (args.config == 1 and first == 0 and n == g3["n"]) else None
    elif args.op == "vlan":
        regen()
        ev_ms = eng.time_vlan_device(d_arena, nbytes, d_desc, n, VPUSH, nf.VLAN_POP, VCAP,
                                     2 * ((args.steps + 1) // 2)) / (2 * ((args.steps + 1) // 2))
        # parity: one push of the untagged batch vs the reference's digest, then one pop
        gv = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json"))).get("vlan_c1", {})
        on_ref = first == 0 and n == gv.get("n")
        step()
        eng.sync()
        got_push = f"{eng.digest_device(d_arena, nbytes, d_desc, n, first):016x}"
        step()
        eng.sync()
        want = gv.get("digest_push_pop") if on_ref else golden_digest(1, first, n)
        if on_ref and got_push != gv["digest_push"]:
            want = "push digest " + gv["digest_push"] + " != " + got_push
    elif args.op == "flowkey":
        ev_ms = eng.time_flow_keys_device(d_arena, nbytes, d_desc, n, d_keys, d_hash,
                                          args.steps) / args.steps
        # parity: digest of the 64-byte records (they hold the hashes too) vs the reference's
        gk = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json"))).get("flowkey_c1", {})
        want = None
        if first == 0 and n == gk.get("n") and args.align == gk.get("align"):
            eng.flow_keys_device(d_arena, nbytes, d_desc, n, d_keys, d_hash)
            rdesc = np.zeros(n, dtype=nf.DESC_DTYPE)
            rdesc["off16"] = np.arange(n, dtype=np.uint32) * 4
            rdesc["len"] = 64
            d_rdesc = eng.alloc(rdesc.nbytes).upload(rdesc)
            eng.sync()
            got_fk = f"{eng.digest_device(d_keys, 64 * n, d_rdesc, n, 0):016x}"
            want = gk["digest_records"]
            d_rdesc.free()
    else:
        ev_ms = eng.time_update_device(d_arena, nbytes, d_desc, n, args.steps) / args.steps
        # parity of what was measured: digest of the updated arena vs the reference's
        want = golden_digest(args.config, first, n)
    achieved = algo_bytes / (ev_ms * 1e-3) / 1e9
    got = f"{eng.digest_device(d_arena, nbytes, d_desc, n, first):016x}"
    if args.op == "flowkey" and want is not None:
        got = got_fk
    parity_ok = None if want is None else (got == want)
    parity_all = D.sum(0.0 if parity_ok is False else 1.0) == ws

    traffic = load_traffic(args.config, n, args.op) if args.align == 128 else None
    fk = args.op == "flowkey"
    total_packets = D.sum(float(n))
    out = {
        "metric": ("flow keys + hash_flow per second, batched packets, MI355X" if fk else
                   "device-resident payload GB/s checksummed, batched packets, 1/2/4/8 MI355X"
                   + (" (fused L3 forward: TTL--, MAC rewrite, checksums)" if l3 else "")
                   + (" (VLAN push/pop + checksums)" if args.op == "vlan" else "")),
        "value": round(total_packets / (wall / args.steps) / 1e6, 2) if fk else
                 round(total_frame_bytes / (wall / args.steps) / 1e9, 2),
        "unit": "Mpkt/s" if fk else "GB/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16 one's-complement (u8 frames, u32 word sums)",
        "data": "synthetic (seeded generator, DESIGN.md §6), generated in HBM",
        "config": {"workload": (WORKLOAD_C4 if c4 else WORKLOAD[args.config])
                   + (", fused L3 forward (next hop i % 9)" if l3 else "")
                   + (", flow keys (header line only)" if fk else "")
                   + (", push_vlan(100, 3) / pop_vlan() alternating, 1536-byte buffers"
                      if args.op == "vlan" else ""),
                   "packets_per_gpu": n, "frame_align": args.align,
                   "frame_bytes_per_gpu": int(frame_bytes), "parallelism": f"independent shards x{ws}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None if traffic is None else int(traffic["hbm_bytes"]),
                     "traffic_read_write": None if traffic is None else
                     [int(traffic["fetch_bytes"]), int(traffic["write_bytes"])],
                     "kernel_ms": round(ev_ms, 4),
                     "algorithmic_bytes_per_launch": int(algo_bytes)},
        "parity": {"digest": got, "reference_digest": want, "match": parity_ok, "all_ranks": parity_all},
    }
    if args.op == "update":
        # frame-only and checksummed-only (frame minus its 14-byte L2 header;
        # the synthetic frames are untagged) rates, and the fraction of the read-only stream
        # ceiling measured on the same MI355X (profiles/r01_stream_microbench.md)
        t_step = wall / args.steps
        csum_bytes = D.sum(frame_bytes - 14.0 * n)
        out["bytes"] = {"frame_GBps": round(total_frame_bytes / t_step / 1e9, 2),
                        "checksummed_GBps": round(csum_bytes / t_step / 1e9, 2),
                        "algorithmic_GBps_kernel": round(achieved, 1)}
        out["stream_ceiling"] = {"read_only_GBps": STREAM_READ_GBPS,
                                 "frac_of_read_only": round(achieved / STREAM_READ_GBPS, 4),
                                 "read_plus_one_store_per_frame_GBps": STREAM_RW_GBPS,
                                 "source": "profiles/r01_stream_microbench.md"}
    if c4:
        # the same 4M-packet shard on ONE GPU (profiles/r01_s4_bench_c4_shard_1gpu.json): the
        # per-GPU rate this line scales, lower than the N = 1 (C1, 1M-packet) line because a
        # 6.3 GB batch does not stay partly cached between launches
        out["one_gpu_same_shard"] = {"value": C4_SHARD_1GPU_GBPS, "unit": "GB/s",
                                     "linear_at_n": round(C4_SHARD_1GPU_GBPS * ws, 1),
                                     "source": "profiles/r01_s4_bench_c4_shard_1gpu.json"}
    if rank == 0 and ws == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_threads, args.cpu_seconds, args.op)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    d_arena.free()
    eng.close()
    D.close()


if __name__ == "__main__":
    main()
