#!/usr/bin/env python3
"""bench.py — device-resident batched checksum throughput (BASELINE.json metric).

A "step" is one pass of the hot path — NetFlow++'s Packet::update_checksums()
(packet.hpp:722-890), batched on the gfx950 engine (one nfcs_update_device call: the read pass and,
for waves of long frames, the non-temporal write pass) — over one batch of synthetic frames that is
already resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1] [--packets n] [--no-cpu]
                  [--op update|l3fwd|flowkey|vlan] [--strong]

Workloads (BASELINE.json configs):
  N = 1   config C1: 1M x 1500 B IPv4+UDP (configs[1]). The timed calls rotate over 4 separately
          generated batches (2 above 1M packets), so no call re-processes what the previous one just
          wrote (a NIC ring's steady state; --batches 1 replays one batch). The line also carries the
          one-batch `replay` sub-line, the `c4_shard` sub-line (the per-GPU batch of N > 1), the
          `c3` and `l3fwd_c3` sub-lines (config C3's 4M-frame mix through the update and the fused
          forward) and the `host` sub-line (the same frames in host memory through nfcs_update_host,
          PCIe included).
  N > 1   config C4: 32M x 1500 B sharded as independent 4M-packet batches, one per GPU (also at 2
          and 4 GPUs): per-GPU work fixed, scaling "weak". `--strong` instead splits ONE batch of
          the config's size across the ranks by bytes (nfcs_shard_bytes; e.g. the mixed C3), whose
          per-rank digests must sum to the reference's digest of the whole batch.
Without a launcher, `--gpus N > 1` starts `torch.distributed.run` with N ranks as a child process
(this process touches no GPU) and exits with its status; under a launcher WORLD_SIZE must equal N.

Prints ONE JSON line on rank 0. `value` = sum over ranks of frame bytes per step / the max over
ranks of the timed wall time per step. `roofline` uses the kernels' HIP-event time on the launch
stream (one call = both passes); `cpu_baseline` times the reference update_checksums()
(oracle/_ref, compiled from /root/reference) or, if that .so is absent, the oracle port, on a
bounded sample on rank 0 at N = 1, on all allotted host cores and on one core.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import netflow_amd as nf  # noqa: E402  (loads no library and touches no GPU until used)

SEED = 20250620
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip parameters)
# round 1's best read-only stream on the MI355X box (tools/stream_read.hip, nt loads;
# profiles/r01_stream_microbench.md); the line's stream_ceiling is measured in each run
STREAM_READ_GBPS = 7007.0
DEFAULT_PACKETS = {0: 1024, 1: 1 << 20, 2: 1 << 20, 3: 1 << 22}
C4_PACKETS_PER_GPU = 1 << 22
FRESH_BATCHES = 4
NAMES = {0: "C0: {n} x 64 B IPv4 (header checksum only)",
         1: "C1: {n} x 1500 B IPv4+UDP, device-resident",
         2: "C2: {n} x 9000 B IPv4+TCP jumbo, device-resident",
         3: "C3: {n} x U{{64..1500}} B IPv4 TCP/UDP mix, device-resident"}


def human(n: int) -> str:
    return f"{n >> 20}M" if n % (1 << 20) == 0 else str(n)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


class stdout_to_stderr:
    """Point file descriptor 1 at stderr for a block (C++ libraries write to it directly)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


class Dist:
    """Barrier + max/sum over ranks; a no-op at world size 1. Only the timing barriers and a few
    scalars cross ranks — the data path has no collective — so they go over gloo
    on 127.0.0.1 after each rank has synchronised its own GPU: no RCCL communicator, no GPU memory
    and no xGMI traffic for them. NFCS_DIST_BACKEND=nccl carries them over RCCL instead."""

    def __init__(self, ws, rank, local):
        self.ws, self.rank, self.local = ws, rank, local
        if ws > 1:
            import torch
            import torch.distributed as dist
            backend = os.environ.get("NFCS_DIST_BACKEND") or "gloo"
            if backend == "nccl":
                torch.cuda.set_device(int(os.environ.get("NFCS_BENCH_DEVICE", local)))
            self.dist, self.torch, self.backend = dist, torch, backend
            # gloo's connection log goes to the process's stdout ("[Gloo] Rank r is connected to
            # ..."): route fd 1 to stderr while the group forms, so stdout carries only the line
            with stdout_to_stderr():
                dist.init_process_group(backend=backend)
                self.barrier()

    def _t(self, v, dtype=None):
        t = self.torch.tensor([v], dtype=dtype or self.torch.float64)
        return t.cuda() if self.backend == "nccl" else t

    def barrier(self):
        if self.ws > 1:
            self.dist.all_reduce(self._t(0.0))

    def max(self, v: float) -> float:
        if self.ws == 1:
            return float(v)
        t = self._t(float(v))
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v: float) -> float:
        if self.ws == 1:
            return float(v)
        t = self._t(float(v))
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def sum_u64(self, v: int) -> int:
        """Exact sum mod 2^64 (int64 all-reduce wraps in two's complement)."""
        if self.ws == 1:
            return int(v) % (1 << 64)
        s = int(v) % (1 << 64)
        t = self._t(s - (1 << 64) if s >= (1 << 63) else s, self.torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return int(t.item()) % (1 << 64)

    def gather(self, v: float) -> list:
        if self.ws == 1:
            return [float(v)]
        out = [self._t(0.0) for _ in range(self.ws)]
        self.dist.all_gather(out, self._t(float(v)))
        return [float(x.item()) for x in out]

    def gather_u64(self, v: int) -> list:
        """Every rank's u64, exact (an int64 all-gather in two's complement)."""
        s = int(v) % (1 << 64)
        if self.ws == 1:
            return [s]
        out = [self._t(0, self.torch.int64) for _ in range(self.ws)]
        self.dist.all_gather(out, self._t(s - (1 << 64) if s >= (1 << 63) else s, self.torch.int64))
        return [int(x.item()) % (1 << 64) for x in out]

    def close(self):
        if self.ws > 1:
            self.dist.destroy_process_group()


def torch_device_init(device: int) -> bool:
    """Initialise torch's HIP device BEFORE the engine loads libnfcs.so. The PyTorch-ROCm wheel
    bundles its own HIP runtime; loaded first, it is the one libnfcs.so binds to (same SONAME), so
    torch.cuda.synchronize() below sees the engine's work. Loaded after the engine, torch would
    load a second runtime that finds no GPU."""
    try:
        import torch
    except ImportError:
        return False
    if not torch.cuda.is_available():
        return False
    torch.cuda.set_device(device)
    torch.cuda.init()
    return True


def device_sync():
    """torch.cuda.synchronize() (the bench contract), on the runtime the engine shares."""
    import torch
    torch.cuda.synchronize()


def shard(rank: int, n_per_rank: int) -> tuple[int, int]:
    """Weak scaling: rank r owns packets [r*n, (r+1)*n) of the seeded stream (uniform lengths, so
    the byte balance of nfcs_shard_bytes is the packet-count split)."""
    return rank * n_per_rank, n_per_rank


def shard_strong(config: int, total: int, rank: int, ws: int) -> tuple[int, int]:
    """Strong scaling: ONE batch of `total` packets split into contiguous ranges by frame bytes
    (nfcs_shard_bytes)."""
    desc, _ = nf.layout_config(config, SEED, 0, total, 128)
    b = nf.shard_bytes(desc, ws)
    return int(b[rank]), int(b[rank + 1] - b[rank])


def golden():
    try:
        return json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))
    except OSError:
        return {}


def golden_digest(config: int, first: int, n: int):
    g = golden()
    c = g.get("configs", {}).get(str(config))
    if c and c["first"] == first and c["n"] == n:
        return c["digest_out"]
    if config == 1:
        for sh in g.get("c1_rank_shards", []) + g.get("c4_rank_shards", []):
            if sh["first"] == first and sh["n"] == n:
                return sh["digest_out"]
    return None


def cgroup_cpu_quota():
    """CPUs of run time the cgroup allows per period (cgroup v2 cpu.max), None if unlimited/unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def allotted_cpus() -> list:
    """The CPUs this process may run on, interleaved across NUMA nodes (node0[0], node1[0],
    node0[1], ...) so that any prefix of the list is spread over every node."""
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(os.cpu_count() or 1))
    nodes = {}
    base = "/sys/devices/system/node"
    try:
        for d in sorted(os.listdir(base)):
            if d.startswith("node") and d[4:].isdigit():
                for part in open(os.path.join(base, d, "cpulist")).read().strip().split(","):
                    a, _, b = part.partition("-")
                    for c in range(int(a), int(b or a) + 1):
                        nodes[c] = int(d[4:])
    except (OSError, ValueError):
        nodes = {}
    by = {}
    for c in cpus:
        by.setdefault(nodes.get(c, 0), []).append(c)
    lists = [by[k] for k in sorted(by)]
    out = []
    for i in range(max(len(x) for x in lists)):
        out += [x[i] for x in lists if i < len(x)]
    return out


def cpu_info() -> dict:
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        allotted = len(os.sched_getaffinity(0))
    except AttributeError:
        allotted = os.cpu_count()
    nnodes = len([d for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit()]) \
        if os.path.isdir("/sys/devices/system/node") else None
    return {"cpu_model": model, "nproc": allotted, "machine_cpus": os.cpu_count(),
            "cgroup_cpu_quota": cgroup_cpu_quota(), "numa_nodes": nnodes}


def cpu_baseline(config: int, threads: int = 0, min_seconds: float = 10.0, op: str = "update",
                 one_core_seconds: float = 5.0, quota_seconds: float = 5.0):
    """The reference's own update_checksums() (oracle/_ref, compiled from /root/reference) on the
    host cores over a bounded sample of the workload: by default one std::thread per allotted CPU
    (every CPU in the process's affinity set, each thread pinned to one, interleaved across NUMA
    nodes; SURVEY.md §8d "all host cores"), then on one thread, and — when the cgroup grants fewer
    CPUs of run time than the affinity set holds — on as many threads as the quota."""
    try:
        import oracle
    except Exception as e:  # pragma: no cover
        return {"value": None, "error": repr(e)}
    kind = "reference" if oracle.ref_available() else "port"
    info = cpu_info()
    cpus = allotted_cpus()
    threads = max(1, min(threads or len(cpus), len(cpus)))
    # at least ~1.2 GB so the sample streams from DRAM like the GPU batch, not from a large L3
    n = {0: 1024, 1: 1 << 20, 2: 1 << 17, 3: 1 << 21}[config]
    arena, desc = oracle.gen_config(config, SEED, 0, n)
    nbytes = float(desc["len"].astype(np.float64).sum())
    recs = hashes = None
    if op == "flowkey":
        recs = np.zeros((n, 64), dtype=np.uint8)
        hashes = np.zeros(n, dtype=np.uint32)

    def runner(t):
        if op == "flowkey":
            if kind == "reference":
                R = oracle.ref()
                return lambda: R.nfref_flow_keys_batch(oracle._ptr(arena), desc.ctypes.data, n,
                                                       oracle._ptr(recs), oracle._ptr(hashes, oracle._u32p), t)
            L = oracle.lib()
            return lambda: L.nfo_flow_keys_batch(oracle._ptr(arena), arena.nbytes, desc.ctypes.data, n,
                                                 oracle._ptr(recs), oracle._ptr(hashes, oracle._u32p))
        if op == "vlan":
            ops = [np.full(n, oracle.vlan_op("push", 100, 3), np.uint32), np.full(n, oracle.vlan_op("pop"), np.uint32)]
            flip = [0]

            def run():
                if kind == "reference":
                    oracle.ref().nfref_vlan_batch(oracle._ptr(varena), vdesc.ctypes.data,
                                                  oracle._ptr(ops[flip[0]], oracle._u32p), n, 1536, t)
                else:
                    oracle.vlan_batch(varena, vdesc, ops[flip[0]], None, cap_all=1536)
                flip[0] ^= 1
            return run
        if op == "l3fwd":
            table = np.frombuffer(bytes.fromhex(golden()["l3fwd_c1"]["table"]), dtype=np.uint8).copy()
            nh = (np.arange(n) % 9).astype(np.uint32)
            if kind == "reference":
                R = oracle.ref()
                return lambda: R.nfref_l3_forward_batch(oracle._ptr(arena), desc.ctypes.data,
                                                        oracle._ptr(nh, oracle._u32p), n, oracle._ptr(table), 8, t)
            L = oracle.lib()
            return lambda: L.nfo_l3_forward_batch(oracle._ptr(arena), arena.nbytes, desc.ctypes.data,
                                                  oracle._ptr(nh, oracle._u32p), n, oracle._ptr(table), 8, None)
        if kind == "reference":
            import ctypes
            R = oracle.ref()
            cl = (ctypes.c_int * len(cpus))(*cpus)
            return lambda: R.nfref_update_batch_on(oracle._ptr(arena), desc.ctypes.data, n, t, cl, len(cpus))
        L = oracle.lib()
        return lambda: L.nfo_update_batch(oracle._ptr(arena), arena.nbytes, desc.ctypes.data, n, None, None, t)

    if op == "vlan":  # 1536-byte buffers, frames 128-byte aligned as on the GPU
        varena, vdesc = oracle.gen_config(config, SEED, 0, n, 128)
    # l3fwd mutates TTLs (each pass forwards once): restore the frames before every pass, untimed
    pristine = arena.copy() if op == "l3fwd" else None

    def timed(t, seconds):
        run = runner(t)
        run()  # warm
        reps, el = 0, 0.0
        while el < seconds:
            if pristine is not None:
                np.copyto(arena, pristine)
            t0 = time.perf_counter()
            run()
            el += time.perf_counter() - t0
            reps += 1
        return reps, el

    port = kind == "port" and op != "update"  # the oracle's other batch entries are single-threaded
    t_all = 1 if port else threads
    unit, scale = ("Mpkt/s", n / 1e6) if op == "flowkey" else ("GB/s", nbytes / 1e9)
    reps, el = timed(t_all, min_seconds)
    reps1, el1 = timed(1, one_core_seconds)
    runs = {t_all: (reps, el)}
    quota = info.get("cgroup_cpu_quota")
    q = int(quota) if quota else 0
    note = ""
    if not port and 1 < q < t_all:
        # the cgroup grants q CPUs of run time: t_all threads share that much, q threads may not
        runs[q] = timed(q, quota_seconds)
        note = (f"; the cgroup grants {quota:g} CPUs of run time, so {t_all} threads share that much; "
                f"{q} threads: x {runs[q][0]} passes ({runs[q][1]:.1f} s)")
    rates = {t: scale * r / e for t, (r, e) in runs.items()}
    best = max(rates, key=rates.get)  # the fastest thread count measured is the baseline
    out = {"value": round(rates[best], 3), "unit": unit, "cores": best, "kind": kind,
           "one_core": round(scale * reps1 / el1, 3),
           "runs": [{"threads": t, "value": round(v, 3)} for t, v in sorted(rates.items())],
           "selection": "value = the fastest of the thread counts measured (every allotted CPU; as "
                        "many threads as the cgroup's CPU quota when it grants fewer); cores = its threads",
           **info}
    out["sample"] = (f"{n} packets of config C{config} ({nbytes / 1e6:.0f} MB) x {reps} passes on "
                     f"{t_all} threads pinned over the allotted CPUs ({el:.1f} s) and x {reps1} on 1 thread "
                     f"({el1:.1f} s), g++ -O2" + note)
    return out


def load_traffic(config: int, n: int, op: str = "update"):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py), for
    the default batch size of the config or, for C1-shaped frames, the 4M-packet C4 shard; None
    otherwise."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    shard = config == 1 and op in ("update", "l3fwd") and n == 1 << 22
    if not shard and n != DEFAULT_PACKETS[config]:
        return None
    try:
        return json.load(open(p)).get(("C4_shard" if shard else f"C{config}") + ("" if op == "update" else f"_{op}"))
    except (OSError, ValueError):
        return None


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def relaunch(n: int) -> int:
    """--gpus N > 1 without a launcher: N ranks under torch.distributed.run, started as a child
    process (this process has made no GPU call), on 127.0.0.1."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.run(cmd).returncode


def make_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=1, choices=[0, 1, 2, 3])
    ap.add_argument("--packets", type=int, default=0, help="packets per GPU (default: config size; "
                                                           "with --strong: of the whole batch)")
    ap.add_argument("--strong", action="store_true",
                    help="N > 1: split one batch across the ranks by bytes instead of one batch per GPU")
    ap.add_argument("--align", type=int, default=128,
                    help="frame start alignment in the arena: 128 = one L2 line per frame start, as "
                         "NIC/DPDK buffer rings lay frames out (16 = densely packed)")
    ap.add_argument("--slot-bytes", type=int, default=0,
                    help="the context's slot-size hint (nfcs_ctx_set_slot_bytes; speed only): 0 = the "
                         "launch shape follows the batch's mean footprint")
    ap.add_argument("--warm-seconds", type=float, default=0.5,
                    help="minimum untimed warm-up time (on top of --warmup steps)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--batches", type=int, default=0,
                    help="update: batches the timed calls rotate over (default 4 up to 1M packets, 2 "
                         "above; 1 = replay one batch)")
    ap.add_argument("--no-replay", action="store_true", help="skip the one-batch replay sub-line")
    ap.add_argument("--no-c4", action="store_true", help="N = 1: skip the C4-shard sub-line")
    ap.add_argument("--no-host", action="store_true", help="N = 1: skip the host-memory (PCIe) sub-line")
    ap.add_argument("--no-mix", action="store_true", help="N = 1: skip the C3-mix sub-lines (update, fused forward)")
    ap.add_argument("--no-ops", action="store_true",
                    help="N = 1: skip the C2 / forward / VLAN / flow-key sub-lines (child bench runs)")
    ap.add_argument("--op", choices=["update", "l3fwd", "flowkey", "vlan"], default="update")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: every CPU in the affinity set)")
    return ap


def main():
    ap = make_parser()
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus))
    ws, rank, local = dist_env()
    if ws != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}: launch N ranks for --gpus N",
              file=sys.stderr)
        sys.exit(2)

    D = Dist(ws, rank, local)
    if ws > 1 and args.strong:
        total = args.packets or DEFAULT_PACKETS[args.config]
        first, n = shard_strong(args.config, total, rank, ws)
        workload = NAMES[args.config].format(n=human(total)) + f", one batch split by bytes over {ws} GPUs"
        scaling = "strong"
    else:
        c4 = ws > 1 and args.config == 1 and not args.packets
        first, n = shard(rank, C4_PACKETS_PER_GPU if c4 else (args.packets or DEFAULT_PACKETS[args.config]))
        if c4:  # BASELINE C4: 32M x 1500 B over 8 GPUs = 4M packets per GPU (also at 2 and 4 GPUs)
            workload = ("C4: 1500 B IPv4+UDP sharded as independent per-GPU batches, 4M packets per GPU "
                        "(32M over 8 GPUs), device-resident")
        else:
            workload = NAMES[args.config].format(n=human(n)) + (f" per GPU x {ws}" if ws > 1 else "")
            if args.packets and args.config == 1:
                workload = workload.replace("C1: ", "C1-shaped: ")
        scaling = "weak"

    # the reference's call convention end to end (the host_adapter sub-line of the N = 1 line): a child
    # process, run before this one touches the GPU, so its host copy threads have the host to themselves
    # (run after the device-resident lines, the same binary measured 29 against 47 GB/s standalone:
    # profiles/r05_b_*)
    host_adapter = host_bursts = None
    if (ws == 1 and args.op == "update" and args.config == 1 and not args.packets and not args.no_c4
            and not args.no_host):
        host_adapter = host_adapter_line(DEFAULT_PACKETS[1])
        host_bursts = host_bursts_line(DEFAULT_PACKETS[1])
    # NFCS_BENCH_DEVICE pins every rank to one device: rehearsing the N-rank path on a 1-GPU box
    dev = int(os.environ.get("NFCS_BENCH_DEVICE", local))
    if not torch_device_init(dev):
        raise SystemExit("bench.py: torch sees no GPU (needs a ROCm GPU for torch.cuda.synchronize)")
    eng = nf.Engine(dev)
    if args.slot_bytes:
        eng.set_slot_bytes(args.slot_bytes)
    d_arena, nbytes, d_desc, hdesc = eng.config_batch(args.config, SEED, first, n, args.align)
    frame_bytes = float(hdesc["len"].astype(np.float64).sum())
    algo_bytes = frame_bytes + 12.0 * n  # + 2x2 B checksum writes + 8 B descriptor per packet
    l3 = args.op == "l3fwd"
    fk = args.op == "flowkey"
    extra_roofline = {}
    # The steady state of a NIC ring, for every op: the calls rotate over `nrot`
    # separately generated batches, so no call re-processes what the previous call wrote and no
    # header line is still in the memory-side cache from an earlier pass over the same frames.
    # 4 batches up to 1M packets (4 x 128 MB of header lines > the 256 MB Infinity Cache), 2 above
    # (a 4M batch alone is 25x the cache). --batches 1 replays one batch.
    nrot = args.batches or (FRESH_BATCHES if n <= (1 << 20) else 2)
    batches = [(d_arena, nbytes, d_desc)] + [eng.config_batch(args.config, SEED, first, n, args.align)[:3]
                                             for _ in range(nrot - 1)]
    ctr = [0]

    def nxt():
        k = ctr[0]
        ctr[0] += 1
        return k, batches[k % nrot]
    if l3:
        # every launch decrements TTL (64 in the generator): each batch is forwarded once per nrot
        # timed steps, and every batch is regenerated before the timed steps
        if args.steps > 60:
            raise SystemExit("--op l3fwd: --steps <= 60 (TTL 64 runs out after 63 forwards)")
        g3 = golden()["l3fwd_c1"]
        table = np.frombuffer(bytes.fromhex(g3["table"]), dtype=np.uint8).copy()
        d_tab = eng.alloc(table.nbytes).upload(table)
        d_nh = eng.alloc(4 * n).upload(((np.arange(first, first + n)) % 9).astype(np.uint32))
        algo_bytes = frame_bytes + 37.0 * n  # + 4 csum + 12 MAC + 1 TTL written, 8 desc + 4 nh + 8 table read

        def step():
            _, (a, b, d) = nxt()
            eng.l3_forward_device(a, b, d, d_nh, n, d_tab, 8)

        def regen():
            for a, b, d in batches:
                eng.gen_config_device(args.config, SEED, first, n, a, b, d)
            eng.sync()
            ctr[0] = 0
    elif fk:
        d_keys = eng.alloc(64 * n)
        d_hash = eng.alloc(4 * n)
        # moved per packet: the frame's first 128-byte line (every field the key reads lies below
        # byte 82, which spans two 64-byte sectors of that line) + 8 B descriptor read, 64 B
        # record + 4 B hash written. `frac` is on these bytes; `frac_needed_bytes` on the 82
        # header bytes the key needs + the same 76.
        hdr = float(np.minimum(hdesc["len"].astype(np.float64), 128.0).sum())
        algo_bytes = hdr + 76.0 * n
        needed = float(np.minimum(hdesc["len"].astype(np.float64), 82.0).sum()) + 76.0 * n

        def step():
            _, (a, b, d) = nxt()
            eng.flow_keys_device(a, b, d, n, d_keys, d_hash)
        regen = lambda: None
    elif args.op == "vlan":
        if args.config != 1:
            raise SystemExit("--op vlan: config 1 (1536-byte buffers per 1500-byte frame)")
        # push_vlan(100, 3) and pop_vlan() alternate on each batch (round r of the rotation pushes
        # when r is even, pops when odd), each on every frame; per packet the pass reads the frame,
        # writes it back from byte 12 (moved by 4 bytes) and updates its length: push 2*len + 4 B,
        # pop (len' = len + 4) 2*len' - 4 B; +8 B descriptor read, 4 B written
        VPUSH, VCAP = nf.vlan_push_op(100, 3), 1536

        def step():
            k, (a, b, d) = nxt()
            eng.vlan_device(a, b, d, n, None, VPUSH if (k // nrot) % 2 == 0 else nf.VLAN_POP, None, VCAP)
        algo_bytes = 2.0 * frame_bytes + 4.0 * n + 12.0 * n

        def regen():  # back to untagged frames: complete the round of pops
            while ctr[0] % (2 * nrot):
                step()
            eng.sync()
    else:
        def step():
            _, (a, b, d) = nxt()
            eng.update_device(a, b, d, n)
        regen = lambda: None

    # torch (for the synchronize around the timed region) was initialised before the engine
    # (torch_device_init), so nothing slow runs between warm-up and timed region: an idle GPU there
    # re-enters the timed steps cold (rocprofv3 trace: C3 kernels 0.78 -> 0.99 ms)
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
        if l3 and done % 48 == 0:
            regen()  # TTL 64: keep every warm-up launch forwarding (an expired packet is not written)
    eng.sync()
    regen()  # l3fwd: fresh TTLs for the timed steps

    # N > 1, weak scaling: rank 0's shard timed ALONE first (the other ranks wait at the barrier,
    # their GPUs idle), with the same steps and clock as the concurrent region below, so the line
    # carries the one-GPU rate of the very workload the N ranks scale
    timed = lambda pre=None: timed_steps(eng, step, args.steps, pre)
    solo, t_rank, wall = scaling_timings(D, timed, frame_bytes, args.steps, ws > 1 and scaling == "weak",
                                         regen if l3 else None, regen)
    t0, t1 = 0.0, t_rank
    ms_per_step = wall / args.steps * 1e3
    total_frame_bytes = D.sum(frame_bytes)
    rank_gbps = D.gather(frame_bytes / ((t1 - t0) / args.steps) / 1e9)

    # kernel duration with HIP events on the launch stream (roofline), same launches
    got = None
    if l3:
        regen()
        ev_ms = event_ms(eng, step, args.steps) / args.steps
        # parity: one forward of a fresh batch vs the reference's digest (C1, rank 0 shard)
        regen()
        step()
        eng.sync()
        want = g3["digest_out"] if (args.config == 1 and first == 0 and n == g3["n"]) else None
        for g in golden().get("l3fwd_more", []):  # C3's 4M mix, 4M C1 frames
            if g["config"] == args.config and g["first"] == first and g["n"] == n:
                want = g["digest_out"]
    elif args.op == "vlan":
        regen()
        vsteps = 2 * nrot * -(-args.steps // (2 * nrot))  # whole push + pop rounds: ends untagged
        ev_ms = event_ms(eng, step, vsteps) / vsteps
        # parity: one push of the untagged batch vs the reference's digest, then one pop
        gv = golden().get("vlan_c1", {})
        on_ref = first == 0 and n == gv.get("n")
        eng.vlan_device(d_arena, nbytes, d_desc, n, None, VPUSH, None, VCAP)
        eng.sync()
        got_push = f"{eng.digest_device(d_arena, nbytes, d_desc, n, first):016x}"
        eng.vlan_device(d_arena, nbytes, d_desc, n, None, nf.VLAN_POP, None, VCAP)
        eng.sync()
        want = gv.get("digest_push_pop") if on_ref else golden_digest(1, first, n)
        if on_ref and got_push != gv["digest_push"]:
            want = "push digest " + gv["digest_push"] + " != " + got_push
    elif fk:
        ev_ms = event_ms(eng, step, args.steps) / args.steps
        # parity: digest of the 64-byte records (they hold the hashes too) vs the reference's; the
        # records depend on the frames' bytes only, so the digest holds at any --align
        gk = golden().get("flowkey_c1", {})
        want = None
        if args.config == 1 and first == 0 and n == gk.get("n"):
            eng.flow_keys_device(d_arena, nbytes, d_desc, n, d_keys, d_hash)
            rdesc = np.zeros(n, dtype=nf.DESC_DTYPE)
            rdesc["off16"] = np.arange(n, dtype=np.uint32) * 4
            rdesc["len"] = 64
            d_rdesc = eng.alloc(rdesc.nbytes).upload(rdesc)
            eng.sync()
            got = f"{eng.digest_device(d_keys, 64 * n, d_rdesc, n, 0):016x}"
            want = gk["digest_records"]
            d_rdesc.free()
        extra_roofline = {"frac_needed_bytes": round(needed / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "needed_bytes_per_packet": "min(len, 82) header + 8 descriptor + 64 record + 4 hash",
                          "frac_is_on": "min(len, 128): the frame's first 128-byte line, the two 64-byte "
                                        "sectors the 82 header bytes span"}
    if args.op != "update":
        extra_roofline["batches_rotated"] = nrot
        extra_roofline["kernel_ms_timing"] = ("HIP events (torch.cuda.Event on the engine's own stream, "
                                              "torch.cuda.ExternalStream) around the rotated calls")
    else:
        # the same rotation, HIP events on the engine's stream around all the calls
        ev_ms = eng.time_update_batches(batches, n, args.steps) / args.steps
        # SURVEY.md §8d asks for the median of >= 20 reps: each call timed alone by its own events
        # (batch k % nrot, so each still runs over frames the previous call did not touch)
        single = sorted(eng.time_update_device(*batches[k % nrot][:2], batches[k % nrot][2], n, 1)
                        for k in range(max(args.steps, 20)))
        extra_roofline = {"kernel_ms_median_single": round(single[len(single) // 2], 4),
                          "kernel_ms_min_single": round(single[0], 4),
                          "single_reps": len(single),
                          "batches_rotated": nrot}
        # parity of what was measured: digest of every updated batch vs the reference's
        want = golden_digest(args.config, first, n)
        digests = [f"{eng.digest_device(a, b, d, n, first):016x}" for a, b, d in batches]
        got = digests[0] if len(set(digests)) == 1 else "batches differ: " + ",".join(digests)
    achieved = algo_bytes / (ev_ms * 1e-3) / 1e9
    if got is None:
        got = f"{eng.digest_device(d_arena, nbytes, d_desc, n, first):016x}"
    parity_ok = None if want is None else (got == want)
    parity = {"digest": got, "reference_digest": want, "match": parity_ok}
    if scaling == "strong" and args.op == "update":
        # the per-rank digests are order-independent sums: together they must equal the reference's
        # digest of the whole batch
        whole = D.sum_u64(int(got, 16))
        want_whole = golden_digest(args.config, 0, args.packets or DEFAULT_PACKETS[args.config])
        parity = {"digest_all_ranks": f"{whole:016x}", "reference_digest": want_whole,
                  "match": None if want_whole is None else f"{whole:016x}" == want_whole}
        parity_ok = parity["match"]
    parity["all_ranks"] = D.sum(0.0 if parity_ok is False else 1.0) == ws

    replay = None
    for a, _, d in batches[1:]:
        a.free()
        d.free()
    if args.op == "update":
        if ws == 1 and not args.no_replay and nrot > 1:
            replay = replay_line(eng, args, first, n, algo_bytes, d_arena, nbytes, d_desc)

    traffic = load_traffic(args.config, n, args.op) if args.align == 128 else None
    # N = 1: the C4 shard (4M x 1500 B, the per-GPU batch of the N > 1 lines) as a sub-line, so the
    # one-GPU line carries the anchor that the multi-GPU lines scale
    c4_wanted = (ws == 1 and args.op == "update" and args.config == 1 and not args.packets
                 and not args.no_c4)
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
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u16 one's-complement (u8 frames, u32 word sums)",
        "data": "synthetic (seeded generator, DESIGN.md §6), generated in HBM",
        "config": {"workload": workload
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
                     "kernel_ms": round(ev_ms, 4),  # mean over the back-to-back timed launches
                     "kernel_ms_spans": ("one nfcs_l3_forward_device call: update_rows_kernel<..., true, 0>" if l3 else
                                         "one nfcs_vlan_device call: vlan_rows_kernel" if args.op == "vlan" else
                                         "one nfcs_flow_keys_device call: flow_keys_kernel" if fk else
                                         "one nfcs_update_device call: update_rows_kernel (read pass) + "
                                         "apply_bytes_kernel (write pass) of every sub-batch; rocprofv3 lists "
                                         "both, their averages add up to it"),
                     "algorithmic_bytes_per_launch": int(algo_bytes), **extra_roofline},
        "parity": parity,
    }
    if ws > 1:
        out["per_gpu_GBps"] = [round(x, 1) for x in rank_gbps]  # each rank's own rate, this run
        # each rank's own roofline: its calls timed by HIP events on its own
        # engine's stream (the same rotation as rank 0's `roofline`, after the concurrent region), its
        # kernel-time fraction of 8 TB/s, and the digest of what it updated — so a GPU that lags, or
        # one whose result differs, shows by index, not only as lower efficiency
        out["per_gpu_kernel_ms"] = [round(x, 4) for x in D.gather(ev_ms)]
        out["per_gpu_frac"] = [round(x, 4) for x in D.gather(achieved / HBM_PEAK_GBS)]
        hexd = got if len(got) == 16 and all(ch in "0123456789abcdef" for ch in got) else None
        out["per_gpu_digest"] = [f"{x:016x}" for x in D.gather_u64(int(hexd, 16) if hexd else 0)]
        out["per_gpu_parity"] = [None if x < 0 else bool(x) for x in
                                 D.gather(-1.0 if parity_ok is None else float(bool(parity_ok)))]
        if args.op == "update" and not args.no_host:
            # every rank at once from host memory (round 6): what N GPUs, each behind its own PCIe
            # link, take end to end — the only way the path can outrun the host's own cores (§7)
            out["host_all_ranks"] = host_ranks_line(eng, D)
    if solo is not None:
        # the same shard on one GPU in this run (rank 0, alone), and value / (N x that)
        out["single_gpu_same_shard_GBps"] = round(solo, 2)
        out["efficiency"] = round(out["value"] / (ws * solo), 4)
        out["efficiency_note"] = ("value / (n_gpus x single_gpu_same_shard_GBps): rank 0's shard timed "
                                  "alone (other ranks idle at the barrier) before the concurrent region, "
                                  "same steps and wall clock")
        if os.environ.get("NFCS_BENCH_DEVICE") is not None:
            out["efficiency_note"] += "; NFCS_BENCH_DEVICE pins every rank to ONE GPU (a rehearsal)"
    if args.op == "update":
        # frame-only and checksummed-only (frame minus its 14-byte L2 header;
        # the synthetic frames are untagged) rates, and the fraction of the read-only stream
        # ceiling measured on the same MI355X (profiles/r01_stream_microbench.md)
        t_step = wall / args.steps
        csum_bytes = D.sum(frame_bytes - 14.0 * n)
        out["bytes"] = {"frame_GBps": round(total_frame_bytes / t_step / 1e9, 2),
                        "checksummed_GBps": round(csum_bytes / t_step / 1e9, 2),
                        "algorithmic_GBps_kernel": round(achieved, 1)}
        # the read-only stream ceiling measured here, on this GPU and over this batch's arena
        # (nfcs_time_stream_read in six forms; the fastest is the ceiling)
        it = max(args.steps, 5)
        forms = {0: "read_pass_shape", 1: "strided_512wg_nt", 2: "read_pass_shape_all_nt",
                 3: "8_loads_per_lane_nt", 4: "16_loads_per_lane_nt", 5: "4_loads_per_lane_nt"}
        sr = {forms[f]: nbytes / (eng.time_stream_read(d_arena, nbytes, it, form=f) / it * 1e-3) / 1e9 for f in forms}
        # and the batch's own frames read in the read pass's access pattern, nothing computed or
        # written (nfcs_time_frames_read): frame + descriptor bytes per time
        sr["frames_in_read_pass_pattern"] = (frame_bytes + 8.0 * n) / (eng.time_frames_read(d_arena, nbytes, d_desc, n, it)
                                                                    / it * 1e-3) / 1e9
        ceil = max(sr.values())
        out["stream_ceiling"] = {"read_only_GBps": round(ceil, 1),
                                 "frac_of_read_only": round(achieved / ceil, 4),
                                 "forms_GBps": {f: round(v, 1) for f, v in sr.items()},
                                 "source": "measured in this run, HIP events, "
                                           f"{it} launches per form: nfcs_time_stream_read over the batch's "
                                           f"{nbytes / 1e9:.3f} GB arena (arena bytes per time) and "
                                           "nfcs_time_frames_read over its frames (frame + descriptor bytes per time)",
                                 "round1_microbench_GBps": STREAM_READ_GBPS}
    if replay is not None:
        out["replay"] = replay
    if c4_wanted:
        d_arena.free()
        d_arena = None
        out["c4_shard"] = c4_shard_line(eng, args)
        if not args.no_mix:
            out["c3"] = mix_line(eng, args, "update")
            # SURVEY §8d's own layout, frames packed at 16-byte starts
            out["c3_packed"] = mix_line(eng, args, "update", 16)
            out["l3fwd_c3"] = mix_line(eng, args, "l3fwd")
        if not args.no_host:
            out["host"] = host_line(eng, args, n)
            if host_adapter is not None:
                out["host_adapter"] = host_adapter
            if host_bursts is not None:
                out["host_bursts"] = host_bursts
        if not args.no_ops:
            out["more"] = more_lines(args)
    if rank == 0 and ws == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_threads, args.cpu_seconds, args.op)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if d_arena is not None:
        d_arena.free()
    eng.close()
    D.close()


def scaling_timings(D, timed, frame_bytes: float, steps: int, solo_first: bool, pre=None, after=None):
    """The timed regions of one bench line. With solo_first (N > 1, weak scaling) rank 0 first runs
    its own shard ALONE — the other ranks wait at the barrier, their GPUs idle — with the same steps
    and clock as the concurrent region; `after` runs on every rank between the two (the fused
    forward's TTL refresh). Then every rank runs its shard at once between barriers. `timed(pre)`
    returns one rank's wall seconds for `steps` steps. Returns (rank 0's solo GB/s of frames or None,
    this rank's concurrent seconds, the max over ranks)."""
    solo = None
    if solo_first:
        D.barrier()
        solo_t = timed(pre) if D.rank == 0 else 0.0
        D.barrier()
        solo = D.sum(frame_bytes / (solo_t / steps) / 1e9 if D.rank == 0 else 0.0)
        if after is not None:
            after()
    D.barrier()
    t_rank = timed()
    D.barrier()
    return solo, t_rank, D.max(t_rank)


def event_ms(eng, step, steps: int) -> float:
    """Milliseconds between two HIP events recorded on the engine's own stream (wrapped as a torch
    ExternalStream) around `steps` step() calls, which launch on that stream."""
    import torch
    st = torch.cuda.ExternalStream(eng.stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(steps):
        step()
    e1.record(st)
    e1.synchronize()
    return float(e0.elapsed_time(e1))


def timed_steps(eng, step, steps: int, regen=None) -> float:
    """Wall time of `steps` back-to-back steps, bracketed by device syncs (torch's and the
    engine's stream). `regen` (the fused forward's TTL refresh) runs once, untimed, before."""
    if regen is not None:
        regen()
    device_sync()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    eng.sync()
    device_sync()
    return time.perf_counter() - t0


def c4_shard_line(eng, args):
    """BASELINE C4's per-GPU batch — rank 0's shard, packets [0, 4M) of the 1500-byte stream —
    on this one GPU, as the N > 1 lines run it: calls rotating over 2 separately generated shards
    (the steady state), warm-up, wall clock over the steps, the rotation's HIP-event time, the
    reference's digest of that shard (configs.json c4_rank_shards) for both copies."""
    n = C4_PACKETS_PER_GPU
    d_arena, nbytes, d_desc, hdesc = eng.config_batch(1, SEED, 0, n, args.align)
    batches = [(d_arena, nbytes, d_desc), eng.config_batch(1, SEED, 0, n, args.align)[:3]]
    frame_bytes = float(hdesc["len"].astype(np.float64).sum())
    algo_bytes = frame_bytes + 12.0 * n
    ctr = [0]

    def step():
        a, b, d = batches[ctr[0] % 2]
        ctr[0] += 1
        eng.update_device(a, b, d, n)
    steps = max(args.steps // 4, 6)
    tw = time.perf_counter()
    done = 0
    while done < args.warmup or time.perf_counter() - tw < 0.3:
        step()
        done += 1
    eng.sync()
    dt = timed_steps(eng, step, steps) / steps
    ev_ms = eng.time_update_batches(batches, n, steps) / steps
    # the read-only floor of the same frames in the read pass's pattern, and the best buffer stream
    rd_ms = eng.time_frames_read(d_arena, nbytes, d_desc, n, steps) / steps
    st_ms = eng.time_stream_read(d_arena, nbytes, steps, form=5) / steps
    ceil = max((frame_bytes + 8.0 * n) / (rd_ms * 1e-3) / 1e9, nbytes / (st_ms * 1e-3) / 1e9)
    want = golden_digest(1, 0, n)
    digests = [f"{eng.digest_device(a, b, d, n, 0):016x}" for a, b, d in batches]
    got = digests[0] if len(set(digests)) == 1 else "batches differ: " + ",".join(digests)
    for a, _, d in batches:
        a.free()
        d.free()
    return {"workload": "C4 shard: rank 0's 4M x 1500 B IPv4+UDP (the per-GPU batch of the N > 1 lines)",
            "packets": n, "steps": steps, "batches_rotated": 2, "value": round(frame_bytes / dt / 1e9, 2),
            "unit": "GB/s", "ms_per_step": round(dt * 1e3, 4), "kernel_ms": round(ev_ms, 4),
            "frac": round(algo_bytes / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "read_only_GBps": round(ceil, 1),
            "frac_of_read_only": round(algo_bytes / (ev_ms * 1e-3) / 1e9 / ceil, 4),
            "parity": {"digest": got, "reference_digest": want, "match": None if want is None else got == want}}


def mix_line(eng, args, op: str, align: int = 0):
    """BASELINE C3 — 4M x U{64..1500} B IPv4 TCP/UDP, the length-divergence stress and the lines
    furthest below roofline — as a sub-line of the N = 1 line, so the driver's clock covers it
    (VERDICT r4 item 1): `op` "update" (nfcs_update_device, the short shape) or "l3fwd" (the fused
    forward, switch.hpp:279-294, next hop i % 9, its short-mix shape). Calls rotate over 2 separately
    generated batches (the steady state), warm-up, wall clock over the steps, HIP events on the
    engine's stream around the rotated calls, the reference's digest of the result (configs.json
    configs[3] / l3fwd_more) for both batches. `align` (default --align): the frame starts; 16 packs
    the frames densely, SURVEY §8d's arena layout (the `c3_packed` sub-line)."""
    n = DEFAULT_PACKETS[3]
    align = align or args.align
    d_arena, nbytes, d_desc, hdesc = eng.config_batch(3, SEED, 0, n, align)
    batches = [(d_arena, nbytes, d_desc), eng.config_batch(3, SEED, 0, n, align)[:3]]
    frame_bytes = float(hdesc["len"].astype(np.float64).sum())
    ctr = [0]
    extra = []
    if op == "l3fwd":
        g3 = golden()["l3fwd_c1"]
        table = np.frombuffer(bytes.fromhex(g3["table"]), dtype=np.uint8).copy()
        d_tab = eng.alloc(table.nbytes).upload(table)
        d_nh = eng.alloc(4 * n).upload((np.arange(n) % 9).astype(np.uint32))
        extra = [d_tab, d_nh]
        algo_bytes = frame_bytes + 37.0 * n
        want = next((g["digest_out"] for g in golden().get("l3fwd_more", [])
                     if g["config"] == 3 and g["first"] == 0 and g["n"] == n), None)

        def call(a, b, d):
            eng.l3_forward_device(a, b, d, d_nh, n, d_tab, 8)

        def regen():  # TTL 64: fresh frames before every timed region and before the parity call
            for a, b, d in batches:
                eng.gen_config_device(3, SEED, 0, n, a, b, d)
            eng.sync()
    else:
        algo_bytes = frame_bytes + 12.0 * n
        want = golden_digest(3, 0, n)
        call = lambda a, b, d: eng.update_device(a, b, d, n)
        regen = lambda: None

    def step():
        a, b, d = batches[ctr[0] % 2]
        ctr[0] += 1
        call(a, b, d)
    steps = max(args.steps // 2, 10)
    if op == "l3fwd":
        # each of the 2 batches is forwarded steps / 2 times per timed region: TTL 64 allows 63
        # (an uncapped --steps ran the timed region over expired, unwritten packets)
        steps = min(steps, 2 * 63)
    tw, done = time.perf_counter(), 0
    while done < args.warmup or time.perf_counter() - tw < 0.3:
        step()
        done += 1
        if done % 48 == 0:
            regen()  # the forward: keep every warm-up call forwarding (TTL 64)
    eng.sync()
    regen()
    dt = timed_steps(eng, step, steps) / steps
    regen()
    if op == "l3fwd":
        ev_ms = event_ms(eng, step, steps) / steps
        regen()
        for a, b, d in batches:  # parity: one forward of each fresh batch
            call(a, b, d)
        eng.sync()
    else:
        ev_ms = eng.time_update_batches(batches, n, steps) / steps
    rd_ms = eng.time_frames_read(d_arena, nbytes, d_desc, n, steps) / steps
    digests = [f"{eng.digest_device(a, b, d, n, 0):016x}" for a, b, d in batches]
    got = digests[0] if len(set(digests)) == 1 else "batches differ: " + ",".join(digests)
    for a, _, d in batches:
        a.free()
        d.free()
    for x in extra:
        x.free()
    achieved = algo_bytes / (ev_ms * 1e-3) / 1e9
    return {"workload": "C3: 4M x U{64..1500} B IPv4 TCP/UDP mix, device-resident"
                        + (", fused L3 forward (next hop i % 9)" if op == "l3fwd" else ""),
            "frame_align": align, "packets": n, "steps": steps, "batches_rotated": 2, "value": round(frame_bytes / dt / 1e9, 2),
            "unit": "GB/s", "ms_per_step": round(dt * 1e3, 4), "kernel_ms": round(ev_ms, 4),
            "algorithmic_bytes_per_launch": int(algo_bytes),
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "frames_read_only_ms": round(rd_ms, 4),
            "frames_read_only_GBps": round((frame_bytes + 8.0 * n) / (rd_ms * 1e-3) / 1e9, 1),
            "frac_of_frames_read_only": round(achieved / ((frame_bytes + 8.0 * n) / (rd_ms * 1e-3) / 1e9), 4),
            "parity": {"digest": got, "reference_digest": want, "match": None if want is None else got == want}}


def replay_line(eng, args, first, n, algo_bytes, d_arena, nbytes, d_desc):
    """The same work REPLAYED on one batch (every call re-processes the frames the previous call
    wrote: their header lines are still in the memory-side cache, and the previous call's dirty
    lines are rewritten there instead of being written back to HBM) — the rounds 1-3 headline form,
    kept beside the steady-state rotation for comparison. Wall clock and HIP events; digest."""
    steps = max(args.steps, 8)
    tw, k = time.perf_counter(), 0
    while k < 8 or time.perf_counter() - tw < args.warm_seconds:  # warm as the main line
        eng.update_device(d_arena, nbytes, d_desc, n)
        k += 1
        if k % 16 == 0:
            eng.sync()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.update_device(d_arena, nbytes, d_desc, n)
    eng.sync()
    dt = (time.perf_counter() - t0) / steps
    ev_ms = eng.time_update_device(d_arena, nbytes, d_desc, n, steps) / steps
    want = golden_digest(args.config, first, n)
    got = f"{eng.digest_device(d_arena, nbytes, d_desc, n, first):016x}"
    return {"batches": 1, "steps": steps, "ms_per_step": round(dt * 1e3, 4), "kernel_ms": round(ev_ms, 4),
            "frac": round(algo_bytes / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "timing": "frac: HIP events on the engine's stream; ms_per_step: wall clock",
            "parity": None if want is None else got == want}


def host_line(eng, args, n, reps: int = 3):
    """The PCIe-inclusive rate (BASELINE north_star: the path starts and ends in host memory):
    C1's frames in a host arena, nfcs_update_host (frames H2D through the NUMA-local pinned ring,
    8-byte patch records back, applied on the host), from a pinned arena (nfcs_host_alloc) and from
    a pageable one; wall clock per call, min and median of `reps` calls, each on freshly restored
    frames; the digest of the result against the reference's. Never `value`."""
    d_arena, nbytes, d_desc, hdesc = eng.config_batch(1, SEED, 0, n, args.align)
    src = d_arena.download(np.uint8, nbytes)
    frame_bytes = float(hdesc["len"].astype(np.float64).sum())
    want = golden_digest(1, 0, n)
    out = {"workload": f"C1: {human(n)} x 1500 B IPv4+UDP in host memory, nfcs_update_host "
                       "(frames H2D, patch records D2H, applied on the host)",
           "timing": f"wall clock per call, min / median of {reps}", "unit": "GB/s"}
    pinned = eng.host_array(nbytes)
    ok = True
    try:
        for mode, arena in (("pinned", pinned), ("pageable", np.empty(nbytes, dtype=np.uint8))):
            arena[:] = src
            eng.update_host(arena, hdesc, want_status=False)  # warm
            ts = []
            for _ in range(reps):
                arena[:] = src
                t0 = time.perf_counter()
                eng.update_host(arena, hdesc, want_status=False)
                ts.append(time.perf_counter() - t0)
            d_arena.upload(arena)
            got = f"{eng.digest_device(d_arena, nbytes, d_desc, n, 0):016x}"
            ok = ok and (want is not None and got == want)
            ts.sort()
            out[mode] = {"GBps": round(frame_bytes / ts[0] / 1e9, 2),
                         "GBps_median": round(frame_bytes / ts[len(ts) // 2] / 1e9, 2),
                         "ms_per_call": round(ts[0] * 1e3, 3), "digest": got}
    finally:
        eng.host_free(pinned)
        d_arena.free()
        d_desc.free()
    node, local = eng.host_numa()
    out["gpu_numa_node"], out["staging_numa_local"] = node, local
    out["parity"] = {"reference_digest": want, "match": ok}
    return out


def host_ranks_line(eng, D, reps: int = 3):
    """N > 1: C1's first 1M frames in a pinned host arena on EVERY rank (NUMA-local to its GPU through
    the context's staging ring), nfcs_update_host on all ranks at once between barriers — the end-to-end
    (PCIe-inclusive) rate of N GPUs each behind its own link; per call the max over ranks, best of `reps`
    after one warm call, frames restored before each; each rank's result digest against the reference's.
    Never `value`."""
    n = DEFAULT_PACKETS[1]
    d_arena, nbytes, d_desc, hdesc = eng.config_batch(1, SEED, 0, n, 128)
    src = d_arena.download(np.uint8, nbytes)
    frame_bytes = float(hdesc["len"].astype(np.float64).sum())
    want = golden_digest(1, 0, n)
    pinned = eng.host_array(nbytes)
    mine, alls = [], []
    try:
        for r in range(reps + 1):
            pinned[:] = src
            D.barrier()
            t0 = time.perf_counter()
            eng.update_host(pinned, hdesc, want_status=False)
            t = time.perf_counter() - t0
            D.barrier()
            if r:  # the first call warms the staging ring
                mine.append(t)
                alls.append(D.max(t))
        d_arena.upload(pinned)
        got = f"{eng.digest_device(d_arena, nbytes, d_desc, n, 0):016x}"
    finally:
        eng.host_free(pinned)
        d_arena.free()
        d_desc.free()
    ok = want is not None and got == want
    node, local = eng.host_numa()
    return {"workload": f"C1: {human(n)} x 1500 B IPv4+UDP in a pinned host arena on every rank, nfcs_update_host "
                        "on all ranks at once (frames H2D over each GPU's own link, patch records back)",
            "timing": f"wall clock per call between barriers, the max over ranks; best of {reps}",
            "GBps_all_ranks": round(D.sum(frame_bytes) / min(alls) / 1e9, 2),
            "per_rank_GBps": [round(x, 2) for x in D.gather(frame_bytes / min(mine) / 1e9)],
            "per_rank_numa_node": [int(x) for x in D.gather(float(node))],
            "per_rank_staging_numa_local": [bool(x) for x in D.gather(float(local))],
            "parity": {"reference_digest": want, "per_rank_match": [bool(x) for x in D.gather(float(ok))]}}


# The other bench lines of DESIGN.md's scope table, each run as its own child bench.py (its own
# process, warm-up, rotation, HIP events and reference digest) after the default line's own work, so
# that the driver's run of the default line times them too ("every config other than C1
# and the C4 shard is builder-run only"). name -> extra arguments.
MORE_LINES = {
    "c2": ["--config", "2", "--steps", "20"],
    "l3fwd_c1": ["--op", "l3fwd", "--steps", "20"],
    "l3fwd_4m": ["--op", "l3fwd", "--packets", "4194304", "--steps", "12"],
    "vlan_c1": ["--op", "vlan", "--steps", "24"],
    "flowkey_c1": ["--op", "flowkey", "--steps", "50"],
}


def more_lines(args):
    """MORE_LINES, each a child `bench.py <args> --no-cpu --no-replay --no-c4 --no-host --no-mix
    --no-ops` on this GPU, summarised: its value, ms per call, roofline frac and kernel time, parity.
    A child that fails is reported as such; the default line is unaffected."""
    res = {}
    common = ["--no-cpu", "--no-replay", "--no-c4", "--no-host", "--no-mix", "--no-ops",
              "--warmup", str(args.warmup), "--align", str(args.align)]
    for name, extra in MORE_LINES.items():
        cmd = [sys.executable, os.path.abspath(__file__), *extra, *common]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            rf = d.get("roofline", {})
            res[name] = {"workload": d["config"]["workload"], "value": d["value"], "unit": d["unit"],
                         "ms_per_step": d["ms_per_step"], "kernel_ms": rf.get("kernel_ms"), "frac": rf.get("frac"),
                         "batches_rotated": rf.get("batches_rotated"), "parity": d.get("parity"),
                         "args": " ".join(extra)}
        except (subprocess.TimeoutExpired, ValueError, IndexError, KeyError, TypeError, AttributeError) as e:
            res[name] = {"error": repr(e)[:300], "args": " ".join(extra)}
    return res


def host_adapter_line(n: int):
    """The reference's own call convention end to end: C1's frames in n separately
    allocated netflow::PacketBuffers (one `new[]` each, packet_buffer.hpp:21-31) as one burst of
    netflow::Packet* through netflow_amd::update_checksums_batch (include/netflow_amd/netflow_adapter.hpp
    -> nfcs_update_host_frames: gather into the pinned ring, H2D, GPU, checksum bytes written back in
    place, pipelined); the same frames in netflow_amd::BufferPool slots of one pinned arena (no gather);
    and the reference's per-packet Packet::update_checksums() over the same PacketBuffers on 1 and on
    as many threads as the cgroup grants CPUs (16 at most) — wall clock per call, best and median of 3,
    each result's digest against the reference's. Run by tests/cpp/_ref/netflow_adapter_test
    `adapterbench` (compiled against the reference's headers by build(); it travels with the tree) as a
    child process. Never `value`."""
    exe = os.path.join(ROOT, "tests", "cpp", "_ref", "netflow_adapter_test")
    if not os.path.exists(exe):
        return {"error": f"{exe} missing (built by __graft_entry__.build() where /root/reference is)"}
    quota = cgroup_cpu_quota()
    threads = max(1, min(16, int(quota) if quota else len(allotted_cpus())))
    want = golden_digest(1, 0, n) or ""
    try:
        r = subprocess.run([exe, "adapterbench", str(n), "3", str(threads), want], capture_output=True, text=True,
                           timeout=300)
        out = json.loads(r.stdout.strip().splitlines()[-1])
    except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
        return {"error": repr(e)}
    out["workload"] = (f"C1: {human(n)} x 1500 B IPv4+UDP, one netflow::PacketBuffer each (the reference's "
                       "own classes), as one burst of netflow::Packet*")
    out["timing"] = "wall clock per call, frames restored before each; best / median of 3"
    out["rc"] = r.returncode
    out["parity"] = {"reference_digest": want,
                     "match": all(out.get(k, {}).get("match") for k in
                                  ("adapter", "buffer_pool", "reference_1_thread", "reference_threads"))}
    return out


BURST_SIZES = (64, 256, 1024, 4096, 16384, 65536)


def host_bursts_line(ring: int, sizes=BURST_SIZES, seconds: float = 0.25):
    """The per-RX-burst operating point INTEGRATION.md §2 prescribes: a ring of C1
    frames checksummed in consecutive bursts of b packets for each b in `sizes` — through
    netflow_amd::update_checksums_batch on the reference's own netflow::PacketBuffers (`adapter`),
    through nfcs_update_host on a pinned ring (`pinned_ring`, and its zero-copy form), and by the
    reference's per-packet Packet::update_checksums() on 1 thread (the switch's own loop,
    switch.hpp:213-294) and on as many threads as the cgroup grants (16 at most); µs per call (median of
    every call in `seconds` per leg), GB/s, and the ring's digest per path against the reference's.
    `crossover_vs_reference_1_thread`: the smallest burst at which the adapter path's median call is
    shorter than the reference's own loop over the same burst. A child process (tests/cpp/_ref/
    netflow_adapter_test burstbench), run before this process touches the GPU. Never `value`."""
    exe = os.path.join(ROOT, "tests", "cpp", "_ref", "netflow_adapter_test")
    if not os.path.exists(exe):
        return {"error": f"{exe} missing (built by __graft_entry__.build() where /root/reference is)"}
    quota = cgroup_cpu_quota()
    threads = max(1, min(16, int(quota) if quota else len(allotted_cpus())))
    want = golden_digest(1, 0, ring) or ""
    try:
        r = subprocess.run([exe, "burstbench", ",".join(str(b) for b in sizes), str(ring), str(seconds), str(threads),
                            want], capture_output=True, text=True, timeout=400)
        out = json.loads(r.stdout.strip().splitlines()[-1])
    except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
        return {"error": repr(e)}
    out["rc"] = r.returncode
    paths = [k for k, v in out.items() if isinstance(v, dict) and "bursts" in v]
    out["parity"] = {"reference_digest": want, "match": bool(paths) and all(out[k]["match"] for k in paths)}

    def crossover(path, ref):
        try:
            return next((b for b in sizes if out[path]["bursts"][str(b)]["us_per_call"]
                         < out[ref]["bursts"][str(b)]["us_per_call"]), None)
        except KeyError:
            return None
    gpu_paths = ("adapter", "pinned_ring", "pinned_ring_zero_copy", "pageable_ring", "buffer_pool")
    out["crossover_vs_reference_1_thread"] = {p: crossover(p, "reference_1_thread") for p in gpu_paths}
    out["crossover_vs_reference_threads"] = {p: crossover(p, "reference_threads") for p in gpu_paths}
    out["workload"] = (f"C1 frames (1500 B IPv4+UDP) in a ring of {human(ring)}, checksummed in consecutive bursts "
                       f"of {', '.join(str(b) for b in sizes)} packets")
    out["timing"] = "steady clock per call; median (and 10th percentile) of every call in the leg"
    return out


if __name__ == "__main__":
    main()
