"""shape_audit.py — measurement tool (not product): is the launch shape
nfcs_update_device picks from a burst's footprint the fastest of its three for layouts OTHER than the
configs the rule was calibrated on? Round 6 found packed C3 in the wrong shape (8-lane rows, 0.51
against 0.64 in the short shape); this sweeps the frame-length distributions and frame alignments a
caller may bring, device-resident, and reports per layout how far the automatic choice is from the
best forced one.

Per layout: two batches of n frames (random payload — torch.randint on the device — under IPv4 TCP/UDP
headers of the layout's lengths, IHL 5, UDP length = frame length - 34), calls rotating over the two
(HIP events on the stream the calls run on; the steady state of a NIC ring). Forms:
  auto   no slot hint; each batch's footprint sample adapts the shape after its first call;
  tiny   slot hint 256  (8-lane rows, 8 packets per one-wave workgroup, inline stores);
  short  slot hint 1000 (16-lane rows, 7 waves/SIMD, inline stores);
  long   slot hint 4096 (16-lane rows, line-aligned windows, deferred stores + write pass, sub-batches).
Two alternating rounds per layout; ms per call = the lower of the two. Every form's digest of both
batches after its calls must equal auto's (the shape picks speed only; the update is idempotent, so
the frames after any number of calls are the frames after one). Parity against the oracle is the GPU
tests' job (tests/test_gpu_slot_hint.py runs every shape against it).

  python3 tools/r06/shape_audit.py OUT.jsonl [--quick | --threshold | --fwdcheck | --vlanset] [--l3fwd | --vlan]
      [--tcp F] [--host-gen] [--only NAME,...]
(--l3fwd: the fused forward, nfcs_l3_forward_device, in place of the update; its shapes by the same
hints: 8-lane rows of 6 slots / 8-lane rows of 12 slots / 16-lane rows with the deferred record pass)
One JSON line per layout, progress on stderr."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import netflow_amd as nf  # noqa: E402

PEAK = 8.0e12
FORMS = (("auto", 0), ("tiny", 256), ("short", 1000), ("long", 4096))
# VLAN push/pop (nfcs_kernels.hip launch_vlan): 8-lane rows storing write-through (< kVlanWtMeanBytes),
# 8-lane rows storing past the caches (< kTinyMeanBytes), 16-lane rows
FORMS_VLAN = (("auto", 0), ("tiny_wt", 128), ("tiny", 512), ("rows16", 1000))
TARGET_BYTES = 1.0e9  # arena bytes per batch (two batches: past the 256 MB memory-side cache)
ITERS = 16
STREAM = None
SEED_GEN = 20250620
HOST_GEN = False  # --host-gen: frames built on the host and uploaded (the forward's long shape ran 8-17%
# slower on frames whose headers a device kernel had stamped byte by byte, even with the same bytes:
# calls ac-af)
TCP_FRAC = 0.5  # --tcp F: the fraction of TCP frames (the rest UDP)


class Ptr:
    """A device address for the Engine calls that take a DeviceBuffer."""

    def __init__(self, p):
        self.ptr = int(p)


def lengths(kind, n, rng):
    if kind[0] == "uniform":  # (kind[2]: a fixed packet count for the layout)
        return np.full(n, kind[1], dtype=np.int64)
    if kind[0] == "range":  # U{lo..hi}
        return rng.integers(kind[1], kind[2] + 1, n)
    if kind[0] == "bimodal":  # 64 / 1500 (or kind[2]) with a fraction p of long frames
        return np.where(rng.random(n) < kind[1], kind[2] if len(kind) > 2 else 1500, 64).astype(np.int64)
    if kind[0] == "imix":  # 7:4:1 of 64 / 570 / 1500
        return rng.permutation(np.tile(np.array([64] * 7 + [570] * 4 + [1500]), n // 12 + 1)[:n])
    raise ValueError(kind)


def layout(kind, align, slot, rng, room=0):
    """(desc, arena_bytes, lens) for about TARGET_BYTES: frames packed at `align`-byte starts, or at
    the starts of fixed `slot`-byte ring slots."""
    probe = lengths(kind, 4096, rng)
    per = slot if slot else float(np.mean(-(-(probe + room) // align) * align))
    n = int(min(4 << 20, max(256 << 10, TARGET_BYTES / per))) & ~15
    if kind[0] == "uniform" and len(kind) > 2:
        n = kind[2]
    lens = lengths(kind, n, rng)
    if slot:
        off = np.arange(n, dtype=np.int64) * slot
    else:
        step = -(-(lens + room) // align) * align
        off = np.concatenate([[0], np.cumsum(step)[:-1]])
    nbytes = int(off[-1] + (slot if slot else step[-1]))
    desc = np.zeros(n, dtype=nf.DESC_DTYPE)
    desc["off16"] = (off // 16).astype(np.uint32)
    desc["len"] = lens.astype(np.uint32)
    if room:  # VLAN: each frame's capacity from its start (its slot)
        caps = np.full(n, slot, dtype=np.uint32) if slot else step.astype(np.uint32)
        return desc, nbytes, lens, caps
    return desc, nbytes, lens


def stamp(arena_t, desc, lens, seed, only=None):
    """IPv4 TCP/UDP headers at every frame start of a random-payload device arena."""
    dev = arena_t.device
    off = torch.from_numpy(desc["off16"].astype(np.int64) * 16).to(dev)
    L = torch.from_numpy(lens).to(dev)
    g = torch.Generator(device="cpu").manual_seed(seed)
    udp = (torch.rand(len(lens), generator=g) >= TCP_FRAC).to(dev)
    cols = {12: 0x08, 13: 0x00, 14: 0x45, 15: 0x00, 16: (L - 14) >> 8, 17: (L - 14) & 0xFF,
            18: 0, 19: 0, 20: 0, 21: 0, 22: 64, 23: torch.where(udp, 17, 6)}
    for c, v in cols.items():
        if only is not None and c not in only:
            continue
        v = v if torch.is_tensor(v) else torch.full_like(L, v)
        arena_t[off + c] = v.to(torch.uint8)
    if only is not None and 38 not in only:
        return
    u = off[udp]
    arena_t[u + 38] = ((L[udp] - 34) >> 8).to(torch.uint8)
    arena_t[u + 39] = ((L[udp] - 34) & 0xFF).to(torch.uint8)


def stamp_host(arena, desc, lens, seed):
    """stamp() on a host arena (numpy): the same header bytes."""
    off = desc["off16"].astype(np.int64) * 16
    L = lens.astype(np.int64)
    g = torch.Generator(device="cpu").manual_seed(seed)
    udp = (torch.rand(len(lens), generator=g) >= TCP_FRAC).numpy()
    cols = {12: 0x08, 13: 0x00, 14: 0x45, 15: 0x00, 16: (L - 14) >> 8, 17: (L - 14) & 0xFF,
            18: 0, 19: 0, 20: 0, 21: 0, 22: 64, 23: np.where(udp, 17, 6)}
    for c, v in cols.items():
        arena[off + c] = np.asarray(v).astype(np.uint8)
    u = off[udp]
    arena[u + 38] = ((L[udp] - 34) >> 8).astype(np.uint8)
    arena[u + 39] = ((L[udp] - 34) & 0xFF).astype(np.uint8)


def audit(eng, name, kind, align, slot, seed, bufs, op="update"):
    rng = np.random.default_rng(seed)
    gen = kind[0] == "config"  # a BASELINE config's own frames (nfcs_gen_config_device), as bench.py's
    if gen:
        desc, nbytes = nf.layout_config(kind[1], SEED_GEN, 0, kind[2], align)
        lens = desc["len"].astype(np.int64)
    elif op == "vlan":
        desc, nbytes, lens, caps = layout(kind, align, slot, rng, room=4)
    else:
        desc, nbytes, lens = layout(kind, align, slot, rng)
    n = len(desc)
    batches = []
    torch.cuda.synchronize()

    host = []
    if HOST_GEN and not gen:  # each batch built on the host and uploaded whole (DMA, full lines)
        for k in range(2):
            h = np.frombuffer(np.random.default_rng(seed * 2 + k).bytes(nbytes), dtype=np.uint8).copy()
            stamp_host(h, desc, lens, seed * 2 + k)
            host.append(torch.from_numpy(h).pin_memory())

    def generate(k):
        a, b, d = batches[k]
        if host:
            bufs[k][:nbytes].copy_(host[k], non_blocking=True)
        elif gen:
            eng.gen_config_device(kind[1], SEED_GEN + k, 0, n, Ptr(a), b, d, stream=STREAM.cuda_stream)
            if len(kind) > 3:  # ("config", c, n, variant): some of the audit's header bytes on top
                off = torch.from_numpy(desc["off16"].astype(np.int64) * 16).to(bufs[k].device)
                if kind[3] in ("id0", "stamp"):
                    for c in (18, 19, 20, 21):
                        bufs[k][off + c] = 0
                if kind[3] == "df":
                    bufs[k][off + 20] = 0x40
                    bufs[k][off + 21] = 0
                if kind[3] == "stamp":
                    stamp(bufs[k], desc, lens, seed * 2 + k)
                parts = {"eth": (12, 13, 14, 15, 16, 17), "ttl": (22, 23), "udplen": (38, 39)}
                if kind[3] in parts:
                    stamp(bufs[k], desc, lens, seed * 2 + k, only=parts[kind[3]])
                if kind[3] == "ttl_rw":  # the TTL stamp, then every line rewritten whole (a copy out and back)
                    stamp(bufs[k], desc, lens, seed * 2 + k, only=(22, 23))
                    tmp = bufs[k][:nbytes].clone()
                    bufs[k][:nbytes].copy_(tmp)
                    del tmp
        else:
            stamp(bufs[k], desc, lens, seed * 2 + k)
    for k in range(2):
        a = bufs[k]
        assert a.numel() >= nbytes
        a[:nbytes].random_(generator=torch.Generator(device=a.device).manual_seed(seed * 2 + k))
        batches.append((a.data_ptr(), nbytes, eng.alloc(desc.nbytes).upload(desc)))
        generate(k)
    torch.cuda.synchronize()
    frame_bytes = float(lens.sum())
    st = STREAM  # a stream of its own (the legacy default stream's handle is 0, which the engine
    # reads as "the context's stream"): the stamps, the calls and the events all run on it
    if op == "l3fwd":
        # the forward (switch.hpp:279-294) with next hop i % 9 over 8 routes (index 8: no route), as
        # bench.py's l3fwd lines; TTL 64 re-stamped before every warm / timed / parity run, each of
        # which forwards a batch at most 10 times
        algo = frame_bytes + 37.0 * n
        table = eng.alloc(96).upload(np.random.default_rng(5).integers(0, 256, 96, dtype=np.uint8))
        nh = eng.alloc(4 * n).upload((np.arange(n) % 9).astype(np.uint32))
        extra = [table, nh]
        call = lambda a, b, d: eng.l3_forward_device(a, b, d, nh, n, table, 8, stream=st.cuda_stream)

        def restamp():
            for k in range(2):
                generate(k)
    elif op == "vlan":
        # Packet::push_vlan / pop_vlan + update_checksums (packet.hpp:655-720): each batch alternates
        # push (VID 100, PCP 3) and pop, so after an even number of calls per batch its frames and
        # lengths are back where they started; frames read and written whole
        algo = 2.0 * frame_bytes + 16.0 * n
        d_caps = eng.alloc(4 * n).upload(caps)
        extra = [d_caps]
        parity = {}
        push = nf.vlan_push_op(100, 3)

        def call(a, b, d):
            k = parity.get(a, 0)
            parity[a] = k + 1
            eng.vlan_device(a, b, d, n, None, push if k % 2 == 0 else nf.VLAN_POP, d_caps, 0,
                            stream=st.cuda_stream)
        restamp = lambda: None
    else:
        algo = frame_bytes + 12.0 * n
        extra = []
        call = lambda a, b, d: eng.update_device(a, b, d, n, stream=st.cuda_stream)
        restamp = lambda: None
    ms = {f: [] for f, _ in (FORMS_VLAN if op == "vlan" else FORMS)}
    digests = {}
    auto_fp = None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    forms = FORMS_VLAN if op == "vlan" else FORMS
    for rnd in range(2):
        for form, hint in forms:
            eng.set_slot_bytes(hint)
            restamp()  # the forward: TTL 64, then 2 warm + ITERS / 2 timed forwards per batch
            for _ in range(2):  # warm: each batch twice (auto: its sample lands and is used)
                for a, b, d in batches:
                    call(a, b, d)
            st.synchronize()
            if form == "auto":
                auto_fp = [eng.launch_footprint(b, d, n) for a, b, d in batches]
            e0.record(st)
            for i in range(ITERS):  # calls rotating over the two batches, HIP events on their stream
                call(*batches[i % 2])
            e1.record(st)
            e1.synchronize()
            ms[form].append(round(e0.elapsed_time(e1) / ITERS, 4))
            restamp()
            if op == "l3fwd":
                for a, b, d in batches:
                    call(a, b, d)
            st.synchronize()
            dg = tuple(eng.digest_device(Ptr(a), b, d, n, stream=st.cuda_stream) for a, b, d in batches)
            digests.setdefault(form, dg)
            assert digests[form] == dg, (name, form)
    # the statuses of one call on batch 0 (fresh frames), by value
    eng.set_slot_bytes(0)
    restamp()
    d_st = eng.alloc(n)
    a, b, d = batches[0]
    if op == "l3fwd":
        eng.l3_forward_device(a, b, d, nh, n, table, 8, d_st, stream=st.cuda_stream)
    elif op == "vlan":
        call(a, b, d)  # a push and its pop: the statuses of the pop
        eng.vlan_device(a, b, d, n, None, nf.VLAN_POP, d_caps, 0, d_st, stream=st.cuda_stream)
        parity[a] += 1
    else:
        eng.update_device(a, b, d, n, d_st, stream=st.cuda_stream)
    st.synchronize()
    hist = np.bincount(d_st.download(np.uint8, n), minlength=256)
    d_st.free()
    for _, _, d in batches:
        d.free()
    for x in extra:
        x.free()
    best = {f: min(v) for f, v in ms.items()}
    fastest = min((f for f in best if f != "auto"), key=lambda f: best[f])
    if op == "vlan":
        shape = lambda fp: "tiny_wt" if fp < 256 else ("tiny" if fp < 800 else "rows16")
    else:
        shape = lambda fp: "tiny" if fp < 800 else ("short" if fp < 1200 else "long")
    return {
        "op": op, "tcp_frac": TCP_FRAC, "layout": name, "align": align, "slot": slot, "n": n, "mean_len": round(frame_bytes / n, 1),
        "arena_bytes_per_packet": round(nbytes / n, 1), "auto_footprint": auto_fp,
        "auto_shape": [shape(fp) for fp in auto_fp], "ms_per_call": ms, "fastest": fastest,
        "auto_vs_fastest": round(best["auto"] / best[fastest], 4),
        "frac": {f: round(algo / (best[f] * 1e-3) / PEAK, 4) for f in best},
        "digests_equal": len(set(digests.values())) == 1,
        "digest": "%016x" % digests["auto"][0],
        "status_hist": {"0x%02x" % v: int(c) for v, c in enumerate(hist) if c},
    }


def main():
    out = sys.argv[1]
    quick = "--quick" in sys.argv
    op = "l3fwd" if "--l3fwd" in sys.argv else ("vlan" if "--vlan" in sys.argv else "update")
    specs = []
    for L in (64, 128, 256, 384, 512, 640, 704, 768, 832, 896, 1024, 1152, 1280, 1500):
        for align in ((16,) if quick else (16, 128)):
            specs.append((f"uniform{L}", ("uniform", L), align, 0))
    for L in (64, 256, 512, 1024, 1500):
        specs.append((f"ring2048_{L}", ("uniform", L), 16, 2048))
    for p in (0.1, 0.25, 0.5, 0.75):
        for align in (16, 128):
            specs.append((f"bimodal{int(p * 100)}", ("bimodal", p), align, 0))
    for align in (16, 128):
        specs.append(("imix", ("imix",), align, 0))
        specs.append(("U64_1500", ("range", 64, 1500), align, 0))
        specs.append(("U64_512", ("range", 64, 512), align, 0))
        specs.append(("U512_1500", ("range", 512, 1500), align, 0))
        specs.append(("U64_9000", ("range", 64, 9000), align, 0))
    if quick:
        specs = specs[:6]
    global TCP_FRAC, HOST_GEN
    HOST_GEN = "--host-gen" in sys.argv
    if "--tcp" in sys.argv:
        TCP_FRAC = float(sys.argv[sys.argv.index("--tcp") + 1])
    if "--vlanset" in sys.argv:
        # round 6, call aj: VLAN push/pop on the mixes kTinyMixMeanBytes moved (its launches share the rule)
        specs = [(f"bimodal{int(p * 100)}", ("bimodal", p), 16, 0) for p in (0.1, 0.2, 0.25, 0.3, 0.35, 0.5)]
        specs += [("bimodal1024_40", ("bimodal", 0.4, 1024), 16, 0), ("U64_1000", ("range", 64, 1000), 16, 0),
                  ("U64_1500", ("range", 64, 1500), 16, 0), ("imix", ("imix",), 16, 0),
                  ("uniform64", ("uniform", 64), 16, 0), ("uniform1500", ("uniform", 1500), 128, 0),
                  ("ring2048_1024", ("uniform", 1024), 16, 2048)]
    if "--vlanset2" in sys.argv:
        # round 6, call ak: VLAN's store policy by frame alignment (call aj: on mixes packed at 16-byte
        # starts 8-lane rows storing write-through beat those storing past the caches by 15-45%)
        specs = []
        for align in (16, 128):
            for L in (128, 256, 384, 512, 640, 768, 1024):
                specs.append((f"uniform{L}", ("uniform", L), align, 0))
            specs += [("imix", ("imix",), align, 0), ("bimodal20", ("bimodal", 0.2), align, 0),
                      ("bimodal30", ("bimodal", 0.3), align, 0), ("bimodal50", ("bimodal", 0.5), align, 0),
                      ("U64_1000", ("range", 64, 1000), align, 0), ("U64_1500", ("range", 64, 1500), align, 0),
                      ("U64_512", ("range", 64, 512), align, 0)]
        specs += [("ring2048_512", ("uniform", 512), 16, 2048), ("ring2048_256", ("uniform", 256), 16, 2048)]
    if "--fwdbytes" in sys.argv:
        # round 6, call ac: which header bytes make the forward's long shape slower on the audit's
        # frames than on C1's own (call ab: 0.309 against 0.265 ms per 1M call)
        specs = [("C1_generated", ("config", 1, 1 << 20), 128, 0),
                 ("C1_ipid0", ("config", 1, 1 << 20, "id0"), 128, 0),
                 ("C1_df", ("config", 1, 1 << 20, "df"), 128, 0),
                 ("C1_stamped", ("config", 1, 1 << 20, "stamp"), 128, 0),
                 ("C1_stamp_eth", ("config", 1, 1 << 20, "eth"), 128, 0),
                 ("C1_stamp_ttl", ("config", 1, 1 << 20, "ttl"), 128, 0),
                 ("C1_stamp_udplen", ("config", 1, 1 << 20, "udplen"), 128, 0),
                 ("C1_stamp_ttl_rw", ("config", 1, 1 << 20, "ttl_rw"), 128, 0),
                 ("uniform1500_1M", ("uniform", 1500, 1 << 20), 128, 0)]
    if "--fwdcheck" in sys.argv:
        # round 6, call aa: the forward's long shape against 8-lane rows on long frames, by TCP share
        specs = [("C1_generated", ("config", 1, 1 << 20), 128, 0), ("C3_generated_1M", ("config", 3, 1 << 20), 128, 0),
                 ("uniform1500", ("uniform", 1500), 128, 0), ("uniform1500_1M", ("uniform", 1500, 1 << 20), 128, 0),
                 ("uniform1280", ("uniform", 1280), 128, 0), ("ring2048_1500", ("uniform", 1500), 16, 2048),
                 ("U64_1500", ("range", 64, 1500), 128, 0), ("bimodal50", ("bimodal", 0.5), 16, 0)]
    if "--threshold" in sys.argv:
        # round 6, call y: where 8-lane rows stop paying for mixes of short and long frames (the
        # fraction p of frames past one 8-lane row pass, kTinyLongMax), and mid-size frames in sparse
        # ring slots against the same frames packed at the same n
        specs = []
        for p in (0.2, 0.3, 0.35, 0.4, 0.45):
            for align in (16, 128):
                specs.append((f"bimodal{int(p * 100)}", ("bimodal", p), align, 0))
        for p in (0.25, 0.4, 0.6):
            specs.append((f"bimodal1024_{int(p * 100)}", ("bimodal", p, 1024), 16, 0))
        for hi in (1000, 1100, 1200, 1300, 1400):
            specs.append((f"U64_{hi}", ("range", 64, hi), 16, 0))
        for L in (640, 768, 832, 896, 960, 1024, 1088, 1152, 1216):
            specs.append((f"ring2048_{L}", ("uniform", L), 16, 2048))
        for L in (896, 1024, 1152):
            specs.append((f"ring4096_{L}", ("uniform", L), 16, 4096))
            specs.append((f"packed488K_{L}", ("uniform", L, 488272), 16, 0))
    if "--only" in sys.argv:
        keep = sys.argv[sys.argv.index("--only") + 1].split(",")  # in this order, repeats allowed
        specs = [next(x for x in specs if x[0] == k) for k in keep]
    eng = nf.Engine(0)
    cap = int(TARGET_BYTES * 1.7) + (64 << 20)  # up to 1M x 1536 B (uniform1500_1M)
    bufs = [torch.empty(cap, dtype=torch.uint8, device="cuda:0") for _ in range(2)]
    global STREAM
    STREAM = torch.cuda.Stream()
    assert STREAM.cuda_stream != 0
    torch.cuda.set_stream(STREAM)
    t0 = time.time()
    with open(out, "w") as f:
        for i, (name, kind, align, slot) in enumerate(specs):
            r = audit(eng, name, kind, align, slot, 1000 + i, bufs, op)
            f.write(json.dumps(r) + "\n")
            f.flush()
            print(f"[{time.time() - t0:6.1f}s] {name:14s} align {align:3d} slot {slot:4d}: auto {r['auto_shape']} "
                  f"{min(r['ms_per_call']['auto']):.4f} ms, fastest {r['fastest']} x{r['auto_vs_fastest']}",
                  file=sys.stderr, flush=True)
    eng.close()


if __name__ == "__main__":
    main()
