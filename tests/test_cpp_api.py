"""The C++ host API (include/netflow_amd/packet.hpp): compiled with g++ against the C ABI,
PacketBuffer/Packet semantics on CPU, bit-exact batched and single-packet updates on GPU."""
import json
import os
import subprocess

import pytest

import netflow_amd as nf
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "packet_shim_test.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "packet_shim_test")


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(nf.LIB_PATH):
        nf.build()
    libdir = os.path.dirname(nf.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I" + os.path.join(ROOT, "include"), SRC,
                    "-o", EXE, "-L" + libdir, "-l:" + os.path.basename(nf.LIB_PATH),
                    "-Wl,-rpath," + libdir, "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return EXE


def test_cpp_api_semantics_cpu(exe):
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True)
    assert "api_failures=0" in r.stdout, r.stdout + r.stderr
    if not os.path.exists("/dev/kfd"):
        assert "engine_without_gpu_throws=1" in r.stdout  # no silent CPU fallback
        assert "batch_rc=-4" in r.stdout and "vlan_batch_rc=-4" in r.stdout  # NFCS_ENODEV, no throw


def _frames():
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "kat.json")))
    names = sorted(kat)
    frames = [bytes.fromhex(kat[k]["in"]) for k in names] + oracle.fuzz_frames(31337, 0, 3000)
    return frames


@pytest.mark.parametrize("mode", [pytest.param("batch", marks=pytest.mark.gpu), "single"])
def test_cpp_update_matches_oracle(exe, mode):
    """update_checksums_batch (GPU) and Packet::update_checksums() (one packet, host CPU)."""
    frames = _frames() if mode == "batch" else _frames()[:200]
    r = subprocess.run([exe, mode], input="\n".join(f.hex() for f in frames) + "\n",
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(frames)
    for f, line in zip(frames, lines):
        st, hx = (line.split(" ") + [""])[:2]
        exp, est = oracle.update_frame(f)
        if (est & 0x3F) == 14:  # outside the parity domain: untouched
            assert hx == f.hex()
            continue
        assert hx == exp.hex()
        if mode == "batch":
            assert int(st) == est


@pytest.mark.parametrize("mode", [pytest.param("vlan", marks=pytest.mark.gpu), "vlan1"])
def test_cpp_vlan_matches_reference_behaviour(exe, mode):
    """netflow_amd::vlan_batch (GPU) and Packet::push_vlan / pop_vlan (one packet, host CPU)
    against the oracle (pinned to the reference by tests/golden/kat_vlan.json / vlan_ref.npz): new
    bytes, length and return."""
    import numpy as np
    from vlan_common import random_vlan_case
    frames, ops, caps = random_vlan_case(77, 3000 if mode == "vlan" else 150)
    room = [int(c) for c in caps]  # the buffer's bytes from the data start = the push capacity
    inp = "\n".join(f"{int(o)} {r} {f.hex()}" for o, r, f in zip(ops, room, frames)) + "\n"
    r = subprocess.run([exe, mode], input=inp, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(frames)
    for i, (f, line) in enumerate(zip(frames, lines)):
        okv, st, nlen, hx = line.split(" ")
        buf = np.zeros(max(room[i], oracle.vlan_window(len(f))), dtype=np.uint8)
        buf[:len(f)] = np.frombuffer(f, dtype=np.uint8)
        ln = np.array([len(f)], dtype=np.uint32)
        est = oracle.lib().nfo_vlan(oracle._ptr(buf), oracle._ptr(ln, oracle._u32p), room[i], int(ops[i]))
        if (est & 0x1F) == 14:
            continue
        assert int(okv) == (1 if est & 0x20 else 0), i
        assert int(nlen) == int(ln[0]), i
        assert hx == buf[:room[i]].tobytes().hex(), i
        if mode == "vlan":
            assert int(st) == est, i


@pytest.mark.gpu
def test_cpp_l3_forward_matches_oracle(exe):
    """netflow_amd::l3_forward_batch against the oracle (pinned to the reference's switch data
    path by tests/golden/kat_l3.json / l3fwd_ref.npz): frame bytes and status per packet."""
    import numpy as np
    frames = _frames()
    rng = np.random.default_rng(9)
    table = rng.integers(0, 256, size=(4, 12), dtype=np.uint8)
    nh = [int(x) for x in (np.arange(len(frames)) % 5)]  # 4 = no route
    inp = table.tobytes().hex() + "\n" + "\n".join(f"{h} {f.hex()}" for h, f in zip(nh, frames)) + "\n"
    r = subprocess.run([exe, "l3"], input=inp, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(frames)
    arena, desc = oracle.pack_frames(frames)
    rst = oracle.l3_forward_batch(arena, desc, np.array(nh, dtype=np.uint32), table)
    for i, (f, line) in enumerate(zip(frames, lines)):
        st, hx = (line.split(" ") + [""])[:2]
        if (rst[i] & 0x3F) == 14:
            continue
        o = int(desc[i]["off16"]) * 16
        assert hx == arena[o:o + len(f)].tobytes().hex(), i
        assert int(st) == int(rst[i]), i


@pytest.mark.gpu
def test_cpp_flow_keys_match_oracle(exe):
    """netflow_amd::flow_keys_batch against the oracle (pinned to the reference's
    packet_classifier.cpp by tests/golden/kat_flow.json / flow_ref.npz), frames of all lengths
    (only the first 128 bytes travel)."""
    frames = _frames() + oracle.fuzz_frames(5150, 0, 500)
    r = subprocess.run([exe, "flow"], input="\n".join(f.hex() for f in frames) + "\n",
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(frames)
    for i, (f, line) in enumerate(zip(frames, lines)):
        h, rec = line.split(" ")
        erec, eh = oracle.flow_key(f)
        assert int(h) == eh, i
        assert rec == erec.hex(), i


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["pool", "poolzc"])
def test_cpp_buffer_pool_batch_matches_oracle(exe, mode):
    """netflow_amd::BufferPool (buffer_pool.hpp:57-123 semantics, slots of one pinned arena):
    a burst checksummed in place with no gather copy (poolzc: the kernel reads the pinned
    arena over PCIe), bit-exact with the oracle; allocate / free / refcount behaviour."""
    frames = _frames()[:3000]
    r = subprocess.run([exe, mode], input="\n".join(f.hex() for f in frames) + "\n",
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "pool_failures=0" in r.stderr
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(frames)
    for f, line in zip(frames, lines):
        st, hx = (line.split(" ") + [""])[:2]
        exp, est = oracle.update_frame(f)
        if (est & 0x3F) == 14:
            assert hx == f.hex()
            continue
        assert hx == exp.hex()
        assert int(st) == est


def test_cpp_api_host_code_under_asan_ubsan():
    """the C++ host API (PacketBuffer / Packet semantics, the engine's refusal to
    run without a device) compiled with -fsanitize=address,undefined (host code only)."""
    if not os.path.exists(nf.LIB_PATH):
        nf.build()
    libdir = os.path.dirname(nf.LIB_PATH)
    exe = os.path.join(ROOT, "tests", "cpp", "packet_shim_test_asan")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
                    "-I" + os.path.join(ROOT, "include"), SRC, "-o", exe, "-L" + libdir,
                    "-l:" + os.path.basename(nf.LIB_PATH), "-Wl,-rpath," + libdir,
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")  # the HIP runtime's own allocations
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode in (0,) and "api_failures=0" in r.stdout, r.stdout + r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 3])
def test_cpp_multi_gpu_host_burst_matches_oracle(exe, k):
    """netflow_amd::MultiGpu (include/netflow_amd/multi_gpu.hpp): one host burst
    split by frame bytes over k contexts (all on device 0 here), one host thread and one staging
    ring each; every frame bit-exact with the oracle, statuses at their own indices, the ranges
    tiling the burst within one frame of byte balance."""
    frames = _frames()
    r = subprocess.run([exe, "multi", str(k)], input="\n".join(f.hex() for f in frames) + "\n",
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(frames)
    for f, line in zip(frames, lines):
        st, hx = (line.split(" ") + [""])[:2]
        exp, est = oracle.update_frame(f)
        if (est & 0x3F) == 14:
            assert hx == f.hex()
            continue
        assert hx == exp.hex()
        assert int(st) == est
    b = [int(x) for x in r.stderr.strip().split("bounds", 1)[1].split()]
    assert len(b) == k + 1 and b[0] == 0 and b[-1] == len(frames) and b == sorted(b)
    per = [sum(len(f) for f in frames[b[p]:b[p + 1]]) for p in range(k)]
    assert max(per) - min(per) <= 2 * max(len(f) for f in frames)
