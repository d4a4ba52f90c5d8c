"""bench.py's N-rank path on a GPU box, both ranks on cuda:0 here
(NFCS_BENCH_DEVICE=0; the timing barriers go over gloo, bench.py's default):
(a) `bench.py --gpus 2` with no launcher starts its own two ranks (torch.distributed.run as a child
process); each owns its own 4M-packet shard of BASELINE config C4 and checks its digest against the
reference's per-rank C4 digests; rank 0's one JSON line reports n_gpus 2, weak scaling, every rank
bit-exact; (b) as the driver launches N > 1 (torch.distributed.run, 127.0.0.1), `--strong` over C3:
one mixed batch split by bytes, the per-rank digests summing to the reference's C3 digest."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_one_gpu_bench_line():
    env = dict(os.environ, NFCS_BENCH_DEVICE="0")  # the default barrier backend (gloo)
    env.pop("WORLD_SIZE", None)
    env.pop("NFCS_DIST_BACKEND", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout  # rank 0's line, nothing else
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["packets_per_gpu"] == 1 << 22
    assert d["parity"]["match"] is True and d["parity"]["all_ranks"] is True
    assert d["value"] > 0 and d["roofline"]["kernel_ms"] > 0
    assert len(d["per_gpu_GBps"]) == 2
    # round 6: every rank's own roofline and digest, by index
    assert len(d["per_gpu_frac"]) == 2 and all(0 < f < 1.0 for f in d["per_gpu_frac"])
    assert len(d["per_gpu_kernel_ms"]) == 2 and all(t > 0 for t in d["per_gpu_kernel_ms"])
    assert d["per_gpu_frac"][0] == d["roofline"]["frac"]
    assert d["per_gpu_parity"] == [True, True]
    assert d["per_gpu_digest"][0] == d["parity"]["digest"] and len(set(d["per_gpu_digest"])) == 2
    # and both ranks at once from host memory (each rank its own pinned C1 arena), digests the reference's
    ha = d["host_all_ranks"]
    assert ha["parity"]["per_rank_match"] == [True, True] and ha["GBps_all_ranks"] > 0
    assert len(ha["per_rank_GBps"]) == 2 and all(x > 0 for x in ha["per_rank_GBps"])
    # the same shard on one GPU, timed alone in the same run, and the efficiency against it (both
    # ranks share cuda:0 here, so about 0.5)
    assert d["single_gpu_same_shard_GBps"] > 0
    assert abs(d["efficiency"] - d["value"] / (2 * d["single_gpu_same_shard_GBps"])) < 1e-3
    assert 0 < d["efficiency"] <= 1.1


def test_one_gpu_line_carries_c4_shard_host_and_cpu_baseline():
    """The N = 1 line (C1, BASELINE configs[1]) times the steady state — calls rotating over 4 separately
    generated batches, every batch's digest the reference's — and carries the one-batch replay
    sub-line, the C4-shard sub-line (the per-GPU batch the N > 1 lines scale, with its own roofline
    fraction and the reference's digest of that shard), the C3 and forward-C3 sub-lines, the
    host-memory (PCIe-inclusive) sub-lines — an arena from pinned and pageable memory, and one
    netflow::PacketBuffer per frame — with the reference's digest, and the CPU baseline at the
    fastest thread count measured."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "8", "--warmup", "2",
           "--cpu-seconds", "1", "--no-ops"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["parity"]["match"] is True
    assert d["roofline"]["batches_rotated"] == 4
    assert d["replay"]["parity"] is True and 0.3 < d["replay"]["frac"] < 1.0
    c4 = d["c4_shard"]
    assert c4["packets"] == 1 << 22 and c4["parity"]["match"] is True and c4["batches_rotated"] == 2
    assert 0.3 < c4["frac"] < 1.0 and c4["value"] > 0
    h = d["host"]
    assert h["parity"]["match"] is True and h["pinned"]["GBps"] > 0 and h["pageable"]["GBps"] > 0
    # round 5: BASELINE C3's mix through the update and the fused forward, under the same clock
    for k in ("c3", "l3fwd_c3", "c3_packed"):
        assert d[k]["parity"]["match"] is True and 0.2 < d[k]["frac"] < 1.0, (k, d[k])
    assert d["c3_packed"]["frame_align"] == 16 and d["c3"]["frame_align"] == 128  # round 6: SURVEY's layout
    # and the reference's own call convention (one netflow::PacketBuffer per frame) end to end
    ha = d["host_adapter"]
    assert ha["rc"] == 0 and ha["parity"]["match"] is True and ha["adapter"]["GBps"] > 0, ha
    # round 6: the per-RX-burst sweep (64 to 64K packets per call) against the reference's own loop,
    # every path's result over the whole ring the reference's
    hb = d["host_bursts"]
    assert hb["rc"] == 0 and hb["parity"]["match"] is True, {k: v for k, v in hb.items() if k != "adapter"}
    for p in ("adapter", "pinned_ring", "pageable_ring", "buffer_pool", "reference_1_thread", "reference_threads"):
        assert set(hb[p]["bursts"]) == {"64", "256", "1024", "4096", "16384", "65536"}, p
        assert all(v["us_per_call"] > 0 for v in hb[p]["bursts"].values()), p
    assert set(hb["crossover_vs_reference_1_thread"]) == {"adapter", "pinned_ring", "pinned_ring_zero_copy",
                                                          "pageable_ring", "buffer_pool"}
    cb = d["cpu_baseline"]
    assert cb["value"] == max(x["value"] for x in cb["runs"]) and cb["value"] > 0
    assert max(x["threads"] for x in cb["runs"]) == cb["nproc"] == len(os.sched_getaffinity(0))
    sc = d["stream_ceiling"]
    assert sc["read_only_GBps"] == max(sc["forms_GBps"].values())


@pytest.mark.timeout(300)
def test_one_gpu_line_carries_the_other_scope_lines():
    """The N = 1 line's `more` sub-lines (round 5): C2, the fused forward on C1 and on 4M frames,
    VLAN push/pop and flow keys, each a child bench run with its own rotation and HIP events, each
    result's digest the reference's (the flow keys: their 64-byte records)."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "1",
           "--no-cpu", "--no-replay", "--no-mix", "--no-host"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.strip()][-1])
    more = d["more"]
    assert set(more) == {"c2", "l3fwd_c1", "l3fwd_4m", "vlan_c1", "flowkey_c1"}, more
    for k, v in more.items():
        assert "error" not in v, (k, v)
        assert v["parity"]["match"] is True and 0.2 < v["frac"] < 1.0 and v["value"] > 0, (k, v)


def test_two_ranks_strong_split_c3():
    env = dict(os.environ, NFCS_BENCH_DEVICE="0", NFCS_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "3", "--strong", "--steps", "3",
           "--warmup", "1", "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["parity"]["match"] is True and d["parity"]["all_ranks"] is True
