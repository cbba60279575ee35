"""Python host binding of the MI355X ed25519 verification engine (stellar-core_amd).

The product is the C-ABI library ``libstellar_sigverify.so`` built in-tree from
``csrc/`` (see ``include/stellar_sigverify.h``).  This module is a thin ctypes
binding used by the tests and ``bench.py``; the C++ integration surface that
mirrors the reference interface (``stellar::PubKeyUtils::verifySig`` /
``verifySigBatch``, /root/reference/src/crypto/SecretKey.{h,cpp}) lives in
``csrc/host/``.

There is deliberately no CPU fallback here: if the HIP library is missing or
no device is present, every entry point raises.

Import it as ``importlib.import_module("stellar-core_amd")`` (the directory
name follows the repository layout contract; it is not a valid identifier).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libstellar_sigverify.so")


VERIFY_KERNEL_SOURCES = ("sv_common.h", "fe25519.h", "fe_asm_gen.h", "ge25519.h", "sc25519.h", "lattice.h", "sha512_dev.h",
                         "verify_core.h", "quad.h", "sv_kparams.h", "sv_kernels.hip")

# kernel paths (include/stellar_sigverify.h)
PATH_AUTO, PATH_THROUGHPUT, PATH_LATENCY = 0, 1, 2


def kernel_source_digest() -> str:
    """SHA-256 over the verify kernel's device sources: ties profile-derived
    numbers (profiles/*_traffic.json) to the kernel they were measured on."""
    import hashlib
    h = hashlib.sha256()
    for name in VERIFY_KERNEL_SOURCES:
        h.update(name.encode())
        with open(os.path.join(_HERE, "csrc", name), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


HOSTLIB_PATH = os.path.join(_HERE, "libstellar_host.so")

SV_OK = 0
SV_ERRORS = {
    -1: "SV_ERR_INVALID_ARG",
    -2: "SV_ERR_NO_DEVICE",
    -3: "SV_ERR_HIP",
    -4: "SV_ERR_ALLOC",
    -5: "SV_ERR_NOT_INIT",
    -6: "SV_ERR_ALIGN",
    -7: "SV_ERR_KERNEL",
}

EXPORTED_SYMBOLS = (
    "sv_init", "sv_shutdown", "sv_device_count", "sv_last_error_string", "sv_version",
    "sv_ed25519_verify_batch", "sv_ed25519_verify_batch_fixed", "sv_ed25519_verify_device",
    "sv_ed25519_sign_device", "sv_timing_enable", "sv_kernel_time", "sv_kernel_time_reset",
    "sv_device_synchronize", "sv_verify_cache_keys", "sv_ed25519_verify_batch_keyed", "sv_sha256_batch",
    "sv_verify_cache_keys_device", "sv_sha256_device", "sv_set_kernel_path",
    "sv_ed25519_verify_batch_gather", "sv_ed25519_verify_batch_gather_cb", "sv_ed25519_verify_batch_cpu", "sv_ed25519_verify_cpu",
    "sv_set_device_map", "sv_set_min_shard", "sv_set_debug_flags", "sv_workspace_bytes", "sv_pinned_bytes",
    "sv_set_key_cache", "sv_key_cache_wait", "sv_key_cache_get_stats", "sv_set_key_tables",
    "sv_ed25519_verify_batch_gather_progress", "sv_host_feed_probe",
)

# test knobs (include/stellar_sigverify.h sv_set_debug_flags)
DBG_TRIVIAL_PAIR, DBG_MAX_WINDOWS, DBG_FAIL, DBG_PREP_ONLY, DBG_KEY_COLLIDE = 0x1, 0x2, 0x4, 0x8, 0x10
# throughput-path geometry: one signature per quad of lanes on every launch / never
DBG_QUAD, DBG_NO_QUAD = 0x20, 0x40
# three-wave cold octet: the tables' hand-over is dropped (its bounded wait runs out: every signature rejects)
DBG_DROP_HANDOVER = 0x80


class SigVerifyError(RuntimeError):
    """A device/allocation error.  Never a reject: the batch is unverified."""


class sv_opts(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("device", ctypes.c_int32),
                ("max_devices", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class FeedStats(ctypes.Structure):
    _fields_ = ([(f, ctypes.c_uint32) for f in ("struct_size", "slots", "threads_per_slot", "usable_cpus")]
                + [("seconds", ctypes.c_double), ("gpu_numa", ctypes.c_int32 * 16),
                   ("staging_numa", ctypes.c_int32 * 16), ("pinned_cpus", ctypes.c_uint32 * 16)])


class KeyCacheStats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in ("capacity", "keys", "warm_batches", "cold_batches", "keys_built",
                                                "evictions", "shared_launches", "table_launches", "table_keys",
                                                "table_clears", "table_slots")]


_lib: Optional[ctypes.CDLL] = None


def _share_hip_runtime_with_torch() -> None:
    # torch ships its own libamdhip64 (soname libamdhip64.so.7).  Importing it
    # first makes this library bind to that same runtime instead of loading a
    # second copy from /opt/rocm when torch is (or will be) in the process.
    if os.environ.get("SV_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SigVerifyError(
            "libstellar_sigverify.so not built (%s); run __graft_entry__.build() "
            "or make -C stellar-core_amd" % path)
    _share_hip_runtime_with_torch()
    lib = ctypes.CDLL(path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.sv_init.restype = ctypes.c_int
    lib.sv_device_count.restype = ctypes.c_int
    lib.sv_last_error_string.restype = ctypes.c_char_p
    lib.sv_version.restype = ctypes.c_char_p
    lib.sv_ed25519_verify_batch.argtypes = [vp, vp, vp, vp, vp, sz, vp, vp]
    lib.sv_ed25519_verify_batch_fixed.argtypes = [vp, vp, vp, ctypes.c_uint32, sz, vp, vp]
    lib.sv_ed25519_verify_device.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_uint32, sz, vp, vp, vp]
    lib.sv_ed25519_sign_device.argtypes = [ctypes.c_int, vp, vp, sz, vp, vp, vp]
    lib.sv_timing_enable.argtypes = [ctypes.c_int]
    lib.sv_kernel_time.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    lib.sv_device_synchronize.argtypes = [ctypes.c_int]
    lib.sv_verify_cache_keys.argtypes = [vp, vp, vp, vp, vp, sz, vp, vp]
    lib.sv_ed25519_verify_batch_keyed.argtypes = [vp, vp, vp, vp, vp, sz, vp, vp, vp]
    lib.sv_sha256_batch.argtypes = [vp, vp, vp, sz, vp, vp]
    lib.sv_verify_cache_keys_device.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_uint32, sz, vp, vp]
    lib.sv_sha256_device.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_uint32, sz, vp, vp]
    lib.sv_ed25519_verify_batch_gather.argtypes = [vp, vp, vp, vp, sz, vp, vp, vp]
    lib.sv_ed25519_verify_batch_cpu.argtypes = [vp, vp, vp, vp, vp, sz, vp, ctypes.c_int]
    lib.sv_ed25519_verify_cpu.argtypes = [vp, vp, vp, sz]
    lib.sv_set_device_map.argtypes = [vp, ctypes.c_int]
    lib.sv_set_min_shard.argtypes = [sz]
    lib.sv_set_debug_flags.argtypes = [ctypes.c_uint32]
    lib.sv_workspace_bytes.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]
    lib.sv_pinned_bytes.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]
    lib.sv_set_key_cache.argtypes = [sz]
    lib.sv_set_key_tables.argtypes = [ctypes.c_int, sz]
    lib.sv_key_cache_wait.argtypes = [ctypes.c_int]
    lib.sv_key_cache_get_stats.argtypes = [ctypes.c_int, ctypes.POINTER(KeyCacheStats)]
    lib.sv_lat_last_trace.argtypes = [ctypes.POINTER(ctypes.c_double)]
    lib.sv_host_feed_probe.argtypes = [vp, vp, vp, ctypes.c_uint32, sz, ctypes.c_uint32, ctypes.c_int,
                                       ctypes.POINTER(FeedStats)]
    _lib = lib
    return lib


def _check(rc: int) -> None:
    if rc != SV_OK:
        msg = _lib.sv_last_error_string().decode(errors="replace") if _lib else ""
        raise SigVerifyError("%s: %s" % (SV_ERRORS.get(rc, rc), msg))


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    # (__array_interface__ is several times cheaper than a.ctypes.data: the
    # 1k-batch latency path pays this per array)
    return ctypes.c_void_p(a.__array_interface__["data"][0])


# sv_opts.flags kernel-path requests (include/stellar_sigverify.h)
FLAG_PATH = {None: 0, "auto": 0, "throughput": 0x1, "latency": 0x2}


def _opts(device: int = -1, max_devices: int = 0, path=None):
    o = sv_opts(ctypes.sizeof(sv_opts), device, max_devices, FLAG_PATH[path] if isinstance(path, (str, type(None)))
                else int(path))
    return ctypes.byref(o)


def device_count() -> int:
    lib = load_library()
    n = lib.sv_device_count()
    if n < 0:
        _check(n)
    return n


def version() -> str:
    return load_library().sv_version().decode()


def _u8(a, shape_tail: int) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.uint8))
    return a.reshape(-1, shape_tail)


def verify_batch(pk, sig, msg, msg_off, msg_len, device: int = -1, max_devices: int = 0, path=None) -> np.ndarray:
    """Variable-length batch: message i = msg[msg_off[i]:msg_off[i]+msg_len[i]].

    Returns a uint8 verdict array (1 = valid), bit-identical to libsodium's
    crypto_sign_verify_detached on every row.  path: None / "auto",
    "throughput" or "latency" (sv_opts.flags; verdicts are identical)."""
    lib = load_library()
    pk = _u8(pk, 32)
    sig = _u8(sig, 64)
    n = pk.shape[0]
    if sig.shape[0] != n:
        raise ValueError("pk/sig row mismatch")
    msg = np.ascontiguousarray(np.asarray(msg, dtype=np.uint8).reshape(-1))
    if msg.size == 0:
        msg = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(np.asarray(msg_off, dtype=np.uint64))
    ln = np.ascontiguousarray(np.asarray(msg_len, dtype=np.uint32))
    if off.shape[0] != n or ln.shape[0] != n:
        raise ValueError("msg_off/msg_len length mismatch")
    if n and int((off + ln).max()) > msg.size:
        raise ValueError("message range out of bounds")
    out = np.zeros(n, np.uint8)
    _check(lib.sv_ed25519_verify_batch(_ptr(pk), _ptr(sig), _ptr(msg), _ptr(off), _ptr(ln), n, _ptr(out),
                                       _opts(device, max_devices, path)))
    return out


def _var_msgs(msg, msg_off, msg_len, n):
    msg = np.ascontiguousarray(np.asarray(msg, dtype=np.uint8).reshape(-1))
    if msg.size == 0:
        msg = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(np.asarray(msg_off, dtype=np.uint64))
    ln = np.ascontiguousarray(np.asarray(msg_len, dtype=np.uint32))
    if off.shape[0] != n or ln.shape[0] != n:
        raise ValueError("msg_off/msg_len length mismatch")
    if n and int((off + ln).max()) > msg.size:
        raise ValueError("message range out of bounds")
    return msg, off, ln


def cache_keys(pk, sig, msg, msg_off, msg_len, device: int = -1, max_devices: int = 0) -> np.ndarray:
    """n x 32 verify-cache keys BLAKE2b-256(pk || sig || msg) computed on the GPU
    (SecretKey.cpp:50-61), SURVEY §8 f4."""
    lib = load_library()
    pk, sig = _u8(pk, 32), _u8(sig, 64)
    n = pk.shape[0]
    msg, off, ln = _var_msgs(msg, msg_off, msg_len, n)
    keys = np.zeros((n, 32), np.uint8)
    _check(lib.sv_verify_cache_keys(_ptr(pk), _ptr(sig), _ptr(msg), _ptr(off), _ptr(ln), n, _ptr(keys),
                                    _opts(device, max_devices)))
    return keys


def verify_batch_keyed(pk, sig, msg, msg_off, msg_len, device: int = -1, max_devices: int = 0):
    """(verdicts, cache keys) from one staging of the batch."""
    lib = load_library()
    pk, sig = _u8(pk, 32), _u8(sig, 64)
    n = pk.shape[0]
    msg, off, ln = _var_msgs(msg, msg_off, msg_len, n)
    out = np.zeros(n, np.uint8)
    keys = np.zeros((n, 32), np.uint8)
    _check(lib.sv_ed25519_verify_batch_keyed(_ptr(pk), _ptr(sig), _ptr(msg), _ptr(off), _ptr(ln), n, _ptr(out),
                                             _ptr(keys), _opts(device, max_devices)))
    return out, keys


def sha256_batch(data, off, length, device: int = -1, max_devices: int = 0) -> np.ndarray:
    """n x 32 SHA-256 digests of data[off[i]:off[i]+length[i]] on the GPU
    (batch tx contents hashes, TransactionFrame.cpp:90-117), SURVEY §8 f4."""
    lib = load_library()
    n = len(off)
    data, o, ln = _var_msgs(data, off, length, n)
    out = np.zeros((n, 32), np.uint8)
    _check(lib.sv_sha256_batch(_ptr(data), _ptr(o), _ptr(ln), n, _ptr(out), _opts(device, max_devices)))
    return out


def verify_messages(pk, sig, messages: Sequence[bytes], **kw) -> np.ndarray:
    lens = np.array([len(m) for m in messages], np.uint32)
    off = np.zeros(len(messages), np.uint64)
    if len(messages) > 1:
        off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(messages), np.uint8) if messages else np.zeros(0, np.uint8)
    return verify_batch(pk, sig, buf, off, lens, **kw)


def verify_fixed(pk, sig, msg, msg_len: int = 32, device: int = -1, max_devices: int = 0, path=None) -> np.ndarray:
    """Fixed-length batch (msg is n x msg_len bytes); msg_len 32 = tx contents hashes."""
    lib = load_library()
    pk = _u8(pk, 32)
    sig = _u8(sig, 64)
    n = pk.shape[0]
    msg = np.ascontiguousarray(np.asarray(msg, dtype=np.uint8).reshape(-1))
    if msg.size != n * msg_len:
        raise ValueError("msg must hold n * msg_len bytes")
    if msg.size == 0:
        msg = np.zeros(1, np.uint8)
    out = np.zeros(n, np.uint8)
    _check(lib.sv_ed25519_verify_batch_fixed(_ptr(pk), _ptr(sig), _ptr(msg), msg_len, n, _ptr(out),
                                             _opts(device, max_devices, path)))
    return out


def verify_device(device: int, d_pk: int, d_sig: int, d_msg: int, n: int, d_verdict: int,
                  d_bitmap: int = 0, stream: int = 0, fixed_msg_len: int = 32,
                  d_msg_off: int = 0, d_msg_len: int = 0) -> None:
    """Device-resident batch (raw device pointers, e.g. torch tensor data_ptr())."""
    lib = load_library()
    _check(lib.sv_ed25519_verify_device(device, d_pk, d_sig, d_msg, d_msg_off or None, d_msg_len or None,
                                        fixed_msg_len, n, d_verdict, d_bitmap or None, stream or None))


def sign_device(device: int, d_seed: int, d_msg32: int, n: int, d_pk: int, d_sig: int, stream: int = 0) -> None:
    lib = load_library()
    _check(lib.sv_ed25519_sign_device(device, d_seed, d_msg32, n, d_pk, d_sig, stream or None))


def verify_batch_cpu(pk, sig, msg, msg_off, msg_len, threads: int = 0) -> np.ndarray:
    """The engine's CPU path (same algorithm, host build): what a caller runs
    when a GPU entry point fails, and what single verifySig calls use."""
    lib = load_library()
    pk, sig = _u8(pk, 32), _u8(sig, 64)
    n = pk.shape[0]
    msg, off, ln = _var_msgs(msg, msg_off, msg_len, n)
    out = np.zeros(n, np.uint8)
    _check(lib.sv_ed25519_verify_batch_cpu(_ptr(pk), _ptr(sig), _ptr(msg), _ptr(off), _ptr(ln), n, _ptr(out),
                                           int(threads)))
    return out


def verify_gather(items, keys: bool = False, device: int = -1, max_devices: int = 0):
    """Gather form: items = [(pk32, sig64, msg), ...] as bytes objects; the engine
    packs them straight from their buffers.  Returns verdicts (and cache keys)."""
    lib = load_library()
    n = len(items)
    bufs = [(bytes(p), bytes(s), bytes(m)) for p, s, m in items]
    P = (ctypes.c_char_p * max(1, n))(*[b[0] for b in bufs])
    S = (ctypes.c_char_p * max(1, n))(*[b[1] for b in bufs])
    M = (ctypes.c_char_p * max(1, n))(*[b[2] for b in bufs])
    L = np.array([len(b[2]) for b in bufs], np.uint32)
    out = np.zeros(n, np.uint8)
    kb = np.zeros((n, 32), np.uint8) if keys else None
    _check(lib.sv_ed25519_verify_batch_gather(ctypes.cast(P, ctypes.c_void_p), ctypes.cast(S, ctypes.c_void_p),
                                              ctypes.cast(M, ctypes.c_void_p), _ptr(L), n, _ptr(out),
                                              _ptr(kb) if keys else None, _opts(device, max_devices)))
    return (out, kb) if keys else out


def set_device_map(physical) -> None:
    """Device slots -> physical GPUs (e.g. [0, 0]: two slots on GPU 0); [] restores."""
    lib = load_library()
    arr = (ctypes.c_int * max(1, len(physical)))(*physical)
    _check(lib.sv_set_device_map(ctypes.cast(arr, ctypes.c_void_p), len(physical)))


def set_min_shard(n: int) -> None:
    _check(load_library().sv_set_min_shard(int(n)))


def set_debug_flags(flags: int) -> int:
    rc = load_library().sv_set_debug_flags(int(flags))
    if rc < 0:
        _check(rc)
    return rc


def workspace_bytes(device: int = 0) -> int:
    v = ctypes.c_size_t()
    _check(load_library().sv_workspace_bytes(device, ctypes.byref(v)))
    return v.value


def pinned_bytes(device: int = 0) -> int:
    v = ctypes.c_size_t()
    _check(load_library().sv_pinned_bytes(device, ctypes.byref(v)))
    return v.value


def set_kernel_path(path: int) -> int:
    """Process-wide default kernel path (PATH_AUTO / PATH_THROUGHPUT /
    PATH_LATENCY) for calls that do not request one; returns the previous."""
    lib = load_library()
    lib.sv_set_kernel_path.argtypes = [ctypes.c_int]
    rc = lib.sv_set_kernel_path(int(path))
    if rc < 0:
        _check(rc)
    return rc


def timing_enable(on: bool = True) -> None:
    _check(load_library().sv_timing_enable(1 if on else 0))


def kernel_time(device: int = 0):
    lib = load_library()
    ms, la, sg = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib.sv_kernel_time(device, ctypes.byref(ms), ctypes.byref(la), ctypes.byref(sg)))
    return ms.value, la.value, sg.value


def kernel_time_reset() -> None:
    _check(load_library().sv_kernel_time_reset())


def synchronize(device: int = 0) -> None:
    _check(load_library().sv_device_synchronize(device))


def set_key_cache(capacity: int) -> None:
    """Key-cache capacity of the warm-key latency path (0: off); clears it."""
    _check(load_library().sv_set_key_cache(int(capacity)))


def set_key_tables(mode: int, slots: int = 0) -> int:
    """Per-key tables of the throughput path: 0 off, 1 on, 2 auto (host
    batches whose keys repeat), -1 the SV_KEY_TABLES default; slots 0 keeps
    SV_KEY_TABLE_SLOTS / 2^19.  Returns the previous mode."""
    rc = load_library().sv_set_key_tables(int(mode), int(slots))
    if rc < -1:
        _check(rc)
    return rc


def key_cache_wait(device: int = 0) -> None:
    """Blocks until the device's queued key-table builds have finished."""
    _check(load_library().sv_key_cache_wait(device))


def key_cache_stats(device: int = 0) -> dict:
    st = KeyCacheStats()
    _check(load_library().sv_key_cache_get_stats(device, ctypes.byref(st)))
    return {f: int(getattr(st, f)) for f, _ in KeyCacheStats._fields_}


LAT_TRACE_FIELDS = ("plan_pack_us", "h2d_call_us", "launch_us", "d2h_rec_us", "build_us", "sync_us", "total_us", "warm")


def host_feed_probe(pk, sig, msg, msg_len: int, max_devices: int = 0, upload: bool = True) -> dict:
    """The host side of a multi-slot fixed-length batch without kernels
    (sv_host_feed_probe, include/stellar_sigverify.h): slices, each slot's
    staging workers, pack into pinned staging, optionally the H2D copies."""
    pk, sig, msg = (np.ascontiguousarray(x, dtype=np.uint8) for x in (pk, sig, msg))
    n = pk.reshape(-1, 32).shape[0]
    if sig.size != 64 * n or msg.size != msg_len * n:
        raise ValueError("pk/sig/msg row mismatch")
    st = FeedStats()
    st.struct_size = ctypes.sizeof(FeedStats)
    _check(load_library().sv_host_feed_probe(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, msg_len, n,
                                             max_devices, 1 if upload else 0, ctypes.byref(st)))
    G = st.slots
    return {"seconds": st.seconds, "slots": G, "threads_per_slot": st.threads_per_slot,
            "usable_cpus": st.usable_cpus, "gpu_numa": list(st.gpu_numa)[:G],
            "staging_numa": list(st.staging_numa)[:G], "pinned_cpus": list(st.pinned_cpus)[:G]}


def lat_last_trace() -> dict:
    """Host-side stages of this thread's last latency-lane batch
    (sv_lat_last_trace, include/stellar_sigverify.h), in microseconds."""
    buf = (ctypes.c_double * 8)()
    _check(load_library().sv_lat_last_trace(buf))
    return dict(zip(LAT_TRACE_FIELDS, list(buf)))
