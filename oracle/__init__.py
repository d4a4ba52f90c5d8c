"""oracle — TEST INFRASTRUCTURE ONLY.

ctypes bindings for
  * ``libnfcs_oracle.so``  — the plain-C restatement of NetFlow++'s
    ``Packet::update_checksums()`` (include/netflow++/packet.hpp:722-912), and
  * ``_ref/libnfref.so``   — the reference path itself, compiled from /root/reference by
    ``make -C oracle ref`` (only where /root/reference exists; the GPU box gets the built
    .so through the gpurun snapshot, never the source).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package. The product (``netflow_amd``) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "libnfcs_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libnfref.so")
REFERENCE_ROOT = "/root/reference"

DESC_DTYPE = np.dtype([("off16", "<u4"), ("len", "<u4")])

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def _ptr(a: np.ndarray, t=_u8p):
    return a.ctypes.data_as(t)


def build(ref: bool | None = None) -> None:
    """Compile the C restatement (and the reference shim when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    if ref is None:
        ref = os.path.isdir(os.path.join(REFERENCE_ROOT, "include", "netflow++"))
    if ref:
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


_lib = None
_ref = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
        L = ctypes.CDLL(ORACLE_SO)
        L.nfo_update.argtypes = [_u8p, ctypes.c_size_t]
        L.nfo_update.restype = ctypes.c_int
        L.nfo_calculate_checksum.argtypes = [_u8p, ctypes.c_size_t]
        L.nfo_calculate_checksum.restype = ctypes.c_uint16
        L.nfo_update_batch.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                       _u8p, _u32p, ctypes.c_int]
        L.nfo_update_batch.restype = ctypes.c_int
        L.nfo_config_len.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        L.nfo_config_len.restype = ctypes.c_uint32
        L.nfo_layout_config.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        L.nfo_layout_config.restype = ctypes.c_uint64
        L.nfo_gen_config.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_uint32, _u8p, ctypes.c_void_p]
        L.nfo_gen_config.restype = None
        L.nfo_fuzz_frame.argtypes = [ctypes.c_uint64, ctypes.c_uint64, _u8p]
        L.nfo_fuzz_frame.restype = ctypes.c_uint32
        L.nfo_mix64.argtypes = [ctypes.c_uint64]
        L.nfo_mix64.restype = ctypes.c_uint64
        L.nfo_frame_hash.argtypes = [_u8p, ctypes.c_uint32]
        L.nfo_frame_hash.restype = ctypes.c_uint64
        L.nfo_digest.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64]
        L.nfo_digest.restype = ctypes.c_uint64
        L.nfo_config_digest.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_int, _u64p, _u64p, _u64p]
        L.nfo_config_digest.restype = None
        L.nfo_l3_forward.argtypes = [_u8p, ctypes.c_size_t, _u8p]
        L.nfo_l3_forward.restype = ctypes.c_int
        L.nfo_l3_forward_batch.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_void_p, _u32p,
                                           ctypes.c_uint32, _u8p, ctypes.c_uint32, _u8p]
        L.nfo_l3_forward_batch.restype = ctypes.c_int
        L.nfo_vlan.argtypes = [_u8p, _u32p, ctypes.c_uint32, ctypes.c_uint32]
        L.nfo_vlan.restype = ctypes.c_int
        L.nfo_vlan_batch.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_void_p, _u32p, ctypes.c_uint32,
                                     _u32p, ctypes.c_uint32, ctypes.c_uint32, _u8p]
        L.nfo_vlan_batch.restype = ctypes.c_int
        L.nfo_flow_key.argtypes = [_u8p, ctypes.c_size_t, _u8p]
        L.nfo_flow_key.restype = ctypes.c_uint32
        L.nfo_flow_keys_batch.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                          _u8p, _u32p]
        L.nfo_flow_keys_batch.restype = None
        _lib = L
    return _lib


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref() -> ctypes.CDLL:
    """The compiled reference path (oracle/_ref/libnfref.so)."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_SO):
            raise FileNotFoundError(f"{REF_SO} not built (make -C oracle ref needs {REFERENCE_ROOT})")
        R = ctypes.CDLL(REF_SO)
        R.nfref_update.argtypes = [_u8p, ctypes.c_size_t]
        R.nfref_update.restype = None
        R.nfref_update_batch.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
        R.nfref_update_batch.restype = None
        R.nfref_update_batch_on.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        R.nfref_update_batch_on.restype = None
        R.nfref_struct_sizes.argtypes = [ctypes.c_int]
        R.nfref_struct_sizes.restype = ctypes.c_int
        R.nfref_l3_forward.argtypes = [_u8p, ctypes.c_size_t, _u8p]
        R.nfref_l3_forward.restype = ctypes.c_int
        R.nfref_l3_forward_batch.argtypes = [_u8p, ctypes.c_void_p, _u32p, ctypes.c_uint32, _u8p,
                                             ctypes.c_uint32, ctypes.c_int]
        R.nfref_l3_forward_batch.restype = None
        R.nfref_vlan.argtypes = [_u8p, _u32p, ctypes.c_uint32, ctypes.c_uint32]
        R.nfref_vlan.restype = ctypes.c_int
        R.nfref_vlan_batch.argtypes = [_u8p, ctypes.c_void_p, _u32p, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_int]
        R.nfref_vlan_batch.restype = None
        R.nfref_flow_key.argtypes = [_u8p, ctypes.c_size_t, _u8p]
        R.nfref_flow_key.restype = ctypes.c_uint32
        R.nfref_flow_keys_batch.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_uint32, _u8p, _u32p,
                                            ctypes.c_int]
        R.nfref_flow_keys_batch.restype = None
        _ref = R
    return _ref


# ---- convenience wrappers --------------------------------------------------------------

def update_frame(frame: bytes) -> tuple[bytes, int]:
    """Oracle update of one frame; returns (new bytes, status)."""
    buf = np.frombuffer(bytearray(frame) + bytearray(16), dtype=np.uint8).copy()
    st = lib().nfo_update(_ptr(buf), len(frame))
    return bytes(buf[: len(frame)]), st


def ref_update_frame(frame: bytes) -> bytes:
    """Reference update of one frame (64 bytes of slack after it, like a PacketBuffer)."""
    buf = np.frombuffer(bytearray(frame) + bytearray(64), dtype=np.uint8).copy()
    ref().nfref_update(_ptr(buf), len(frame))
    return bytes(buf[: len(frame)])


def l3_forward_frame(frame: bytes, nh: bytes | None) -> tuple[bytes, int]:
    """Oracle L3 forward of one frame (nh = 12 bytes {dst, src} or None); (bytes, status)."""
    buf = np.frombuffer(bytearray(frame) + bytearray(16), dtype=np.uint8).copy()
    h = None if nh is None else np.frombuffer(bytes(nh), dtype=np.uint8).copy()
    st = lib().nfo_l3_forward(_ptr(buf), len(frame), None if h is None else _ptr(h))
    return bytes(buf[: len(frame)]), st


def ref_l3_forward_frame(frame: bytes, nh: bytes | None) -> tuple[bytes, int]:
    """Reference L3 forward of one frame; (bytes, 1 if forwarded else 0)."""
    buf = np.frombuffer(bytearray(frame) + bytearray(64), dtype=np.uint8).copy()
    h = None if nh is None else np.frombuffer(bytes(nh), dtype=np.uint8).copy()
    fw = ref().nfref_l3_forward(_ptr(buf), len(frame), None if h is None else _ptr(h))
    return bytes(buf[: len(frame)]), fw


def l3_forward_batch(arena: np.ndarray, desc: np.ndarray, nh_index: np.ndarray,
                     table: np.ndarray) -> np.ndarray:
    n = len(desc)
    status = np.zeros(n, dtype=np.uint8)
    nh_index = np.ascontiguousarray(nh_index, dtype=np.uint32)
    table = np.ascontiguousarray(table, dtype=np.uint8).reshape(-1)
    lib().nfo_l3_forward_batch(_ptr(arena), arena.nbytes, desc.ctypes.data, _ptr(nh_index, _u32p),
                               n, _ptr(table) if table.size else None, table.size // 12,
                               _ptr(status))
    return status


VLAN_PUSH = 0x40000000
VLAN_POP = 0x80000000


def vlan_op(kind: str, vid: int = 0, prio: int = 0) -> int:
    """Edit word of include/nfcs.h (NFCS_VLAN_OP): 'push' / 'pop' / 'nop'."""
    k = {"push": VLAN_PUSH, "pop": VLAN_POP, "nop": 0}[kind]
    return k | ((prio & 7) << 13) | (vid & 0xFFF) if k == VLAN_PUSH else k


def vlan_window(n: int) -> int:
    """Bytes of a frame's buffer an edit of an n-byte frame can touch: round_up(max(n+4, 16), 16)."""
    return (max(n + 4, 16) + 15) // 16 * 16


def _vlan_buf(frame: bytes, cap: int) -> np.ndarray:
    size = max(cap, vlan_window(len(frame)))
    return np.frombuffer(bytes(frame) + bytes(size - len(frame)), dtype=np.uint8).copy()


def vlan_frame(frame: bytes, op: int, cap: int) -> tuple[bytes, int, bytes]:
    """Oracle push_vlan/pop_vlan + update_checksums of one frame in a zero-filled buffer of
    max(cap, vlan_window) bytes. Returns (new frame, status, buffer[:vlan_window(len)])."""
    buf = _vlan_buf(frame, cap)
    ln = np.array([len(frame)], dtype=np.uint32)
    st = lib().nfo_vlan(_ptr(buf), _ptr(ln, _u32p), cap, op)
    return bytes(buf[: int(ln[0])]), st, bytes(buf[: vlan_window(len(frame))])


def ref_vlan_frame(frame: bytes, op: int, cap: int) -> tuple[bytes, int, bytes]:
    """The reference's Packet::push_vlan / pop_vlan on the same buffer: (frame, ret, window)."""
    buf = _vlan_buf(frame, cap)
    ln = np.array([len(frame)], dtype=np.uint32)
    ok = ref().nfref_vlan(_ptr(buf), _ptr(ln, _u32p), cap, op)
    return bytes(buf[: int(ln[0])]), ok, bytes(buf[: vlan_window(len(frame))])


def vlan_batch(arena: np.ndarray, desc: np.ndarray, ops=None, caps=None, op_all: int = 0,
               cap_all: int = 0) -> np.ndarray:
    """Oracle batch (nfcs_vlan_device contract): arena and desc lengths updated in place;
    per-frame ops / caps arrays or uniform op_all / cap_all. Returns the status bytes."""
    n = len(desc)
    status = np.zeros(n, dtype=np.uint8)
    o = None if ops is None else np.ascontiguousarray(ops, dtype=np.uint32)
    c = None if caps is None else np.ascontiguousarray(caps, dtype=np.uint32)
    lib().nfo_vlan_batch(_ptr(arena), arena.nbytes, desc.ctypes.data,
                         None if o is None else _ptr(o, _u32p), op_all,
                         None if c is None else _ptr(c, _u32p), cap_all, n, _ptr(status))
    return status


def flow_key(frame: bytes) -> tuple[bytes, int]:
    """Oracle extract_flow_key + hash_flow of one frame: (64-byte record, hash)."""
    buf = np.frombuffer(bytes(frame) + bytes(16), dtype=np.uint8).copy()
    rec = np.zeros(64, dtype=np.uint8)
    h = lib().nfo_flow_key(_ptr(buf), len(frame), _ptr(rec))
    return bytes(rec), int(h)


def ref_flow_key(frame: bytes) -> tuple[bytes, int]:
    """Reference PacketClassifier::extract_flow_key + hash_flow: (64-byte record, hash)."""
    buf = np.frombuffer(bytes(frame) + bytes(64), dtype=np.uint8).copy()
    rec = np.zeros(64, dtype=np.uint8)
    h = ref().nfref_flow_key(_ptr(buf), len(frame), _ptr(rec))
    return bytes(rec), int(h)


def flow_keys_batch(arena: np.ndarray, desc: np.ndarray):
    n = len(desc)
    recs = np.zeros((n, 64), dtype=np.uint8)
    hashes = np.zeros(n, dtype=np.uint32)
    lib().nfo_flow_keys_batch(_ptr(arena), arena.nbytes, desc.ctypes.data, n, _ptr(recs),
                              _ptr(hashes, _u32p))
    return recs, hashes


def update_batch(arena: np.ndarray, desc: np.ndarray, nthreads: int = 1,
                 want_result: bool = True):
    n = len(desc)
    status = np.zeros(n, dtype=np.uint8)
    result = np.zeros(n, dtype=np.uint32) if want_result else None
    lib().nfo_update_batch(_ptr(arena), arena.nbytes, desc.ctypes.data, n, _ptr(status),
                           _ptr(result, _u32p) if want_result else None, nthreads)
    return status, result


def layout_config(config: int, seed: int, first: int, n: int, align: int = 16):
    desc = np.zeros(n, dtype=DESC_DTYPE)
    nbytes = lib().nfo_layout_config(config, seed, first, n, align, desc.ctypes.data)
    return desc, int(nbytes)


def gen_config(config: int, seed: int, first: int, n: int, align: int = 16):
    desc, nbytes = layout_config(config, seed, first, n, align)
    arena = np.zeros(max(nbytes, 16), dtype=np.uint8)
    lib().nfo_gen_config(config, seed, first, n, _ptr(arena), desc.ctypes.data)
    return arena, desc


def fuzz_frames(seed: int, first: int, n: int) -> list[bytes]:
    buf = np.zeros(9024, dtype=np.uint8)
    out = []
    L = lib()
    for i in range(first, first + n):
        ln = L.nfo_fuzz_frame(seed, i, _ptr(buf))
        out.append(bytes(buf[:ln]))
    return out


def pack_frames(frames: list[bytes], align: int = 16, room: int = 0):
    """Lay frames out in one arena with `align`-byte starts (16-byte chunk padding); each slot
    holds at least len + room bytes (room = 4 leaves tailroom for a VLAN push)."""
    assert align % 16 == 0
    n = len(frames)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    off = 0
    for i, f in enumerate(frames):
        desc[i] = (off // 16, len(f))
        off += (len(f) + room + align - 1) // align * align
    arena = np.zeros(max(off, 16), dtype=np.uint8)
    for i, f in enumerate(frames):
        o = int(desc[i]["off16"]) * 16
        arena[o: o + len(f)] = np.frombuffer(f, dtype=np.uint8)
    return arena, desc


def unpack_frames(arena: np.ndarray, desc: np.ndarray) -> list[bytes]:
    out = []
    for d in desc:
        o = int(d["off16"]) * 16
        out.append(bytes(arena[o: o + int(d["len"])]))
    return out


def digest(arena: np.ndarray, desc: np.ndarray, first: int = 0) -> int:
    return int(lib().nfo_digest(_ptr(arena), desc.ctypes.data, len(desc), first))


def config_digest(config: int, seed: int, first: int, n: int, nthreads: int = 8):
    din = ctypes.c_uint64()
    dout = ctypes.c_uint64()
    hist = (ctypes.c_uint64 * 256)()
    lib().nfo_config_digest(config, seed, first, n, nthreads, ctypes.byref(din),
                            ctypes.byref(dout), hist)
    return int(din.value), int(dout.value), {i: int(hist[i]) for i in range(256) if hist[i]}
