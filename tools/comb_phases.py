#!/usr/bin/env python3
"""Developer tool: phase timeline of the warm-key comb kernel from the
stamps of variants/libsv_diag_phases.so (tools/build_comb_diag.sh):
s_memrealtime (100 MHz) at the phase boundaries of every wave of the last
1k SCP batch.  With --octet: the cold-key octet kernel (key cache off) from
variants/libsv_diag_ophases.so.
Usage: python tools/comb_phases.py [--octet] [library]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: F401,E402
import bench  # noqa: E402
from ab_lat_capi import Opts  # noqa: E402  (tools/ on sys.path via __file__'s dir)

TICK_US = 0.01  # s_memrealtime: 100 MHz


def stats(d):
    return "%7.2f %7.2f %7.2f" % (np.median(d), np.percentile(d, 90), d.max())


def octet_report(lib, n):
    st = np.zeros((2048, 2, 8), np.uint64)
    assert lib.sv_diag_octet_times(ctypes.c_void_p(st.ctypes.data), st.nbytes) == 0
    nwg = (n + 7) // 8  # 8 signatures per workgroup
    st = st[:nwg].astype(np.int64)
    t0 = st[:, :, 0].min()
    print("workgroups %d, first stamp -> last stamp %.1f us" % (nwg, (st[:, 0, 6].max() - t0) * TICK_US))
    w0 = st[:, 0, :]
    print("hash wave (us): median / p90 / max")
    for k, nm in enumerate(["load + SHA-512", "checks, mod L, lattice reduction", "digits",
                            "wait for the tables (decode wave)", "-A / -R chains (quads)",
                            "P_A + P_R, wait for [s]B"]):
        print("  %-36s %s" % (nm, stats((w0[:, k + 1] - w0[:, k]) * TICK_US)))
    print("  %-36s %s" % ("total", stats((w0[:, 6] - w0[:, 0]) * TICK_US)))
    w1 = st[:, 1, :]
    print("decode wave (us): median / p90 / max")
    for k, nm in enumerate(["square roots of A and R (quads)", "tables of -A / -R", "wait for the digits",
                            "[s]B (Horner, radix 2^16)", "wait for the hash wave"]):
        print("  %-36s %s" % (nm, stats((w1[:, k + 1] - w1[:, k]) * TICK_US)))


def main():
    octet = "--octet" in sys.argv
    argv = [a for a in sys.argv[1:] if a != "--octet"]
    dflt = "libsv_diag_ophases.so" if octet else "libsv_diag_phases.so"
    path = argv[0] if argv else os.path.join(REPO, "variants", dflt)
    sodium = bench.load_libsodium()
    pks, sigs, lmsgs, expect = bench.scp_latency_set(sodium)
    pk_a = np.ascontiguousarray(np.frombuffer(b"".join(pks), np.uint8).reshape(-1, 32))
    sg_a = np.ascontiguousarray(np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 64))
    m_len = np.array([len(m) for m in lmsgs], np.uint32)
    m_off = np.zeros(len(lmsgs), np.uint64)
    m_off[1:] = np.cumsum(m_len[:-1], dtype=np.uint64)
    m_buf = np.frombuffer(b"".join(lmsgs), np.uint8)
    n = len(m_len)
    args = [ctypes.c_void_p(a.ctypes.data) for a in (pk_a, sg_a, m_buf, m_off, m_len)]
    lib = ctypes.CDLL(path, mode=os.RTLD_LOCAL)
    lib.sv_set_key_cache.argtypes = [ctypes.c_size_t]
    assert lib.sv_init() == 0
    if octet:
        assert lib.sv_set_key_cache(0) == 0
    else:
        lib.sv_diag_comb_times.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    opts = ctypes.byref(Opts(ctypes.sizeof(Opts), 0, 0, 0))
    out = np.zeros(n, np.uint8)
    outp = ctypes.c_void_p(out.ctypes.data)
    for it in range(50):
        assert lib.sv_ed25519_verify_batch(*args, ctypes.c_size_t(n), outp, opts) == 0
        if it == 1:
            assert lib.sv_key_cache_wait(0) == 0
    assert np.array_equal(out, expect), "phase build: verdicts differ from libsodium"
    if octet:
        octet_report(lib, n)
        return
    st = np.zeros((1024, 4, 8), np.uint64)
    assert lib.sv_diag_comb_times(ctypes.c_void_p(st.ctypes.data), st.nbytes) == 0
    nwg = (n + 5) // 6  # SPW = 2: 6 signatures per workgroup
    st = st[:nwg].astype(np.int64)
    t0 = st[:, :, 0].min()
    span = (st[:, 1:, 7].max() - t0) * TICK_US
    print("workgroups %d, kernel span (first stamp -> last stamp) %.1f us" % (nwg, span))
    chain = st[:, 1:, :]
    names = ["hash (load + SHA-512)", "key slot + S digits", "B entry loads + first entry",
             "B sum, mod L, -A loads + sum", "tree", "barrier wait (decode wave)", "final check"]
    print("chain waves (per wave, us): median / p90 / max")
    for k, nm in enumerate(names):
        d = (chain[:, :, k + 1] - chain[:, :, k]).ravel() * TICK_US
        print("  %-30s %7.2f %7.2f %7.2f" % (nm, np.median(d), np.percentile(d, 90), d.max()))
    d = (chain[:, :, 7] - chain[:, :, 0]).ravel() * TICK_US
    print("  %-30s %7.2f %7.2f %7.2f" % ("chain wave total", np.median(d), np.percentile(d, 90), d.max()))
    dec = st[:, 0, :]
    d1 = (dec[:, 1] - dec[:, 0]) * TICK_US
    d2 = (dec[:, 2] - dec[:, 1]) * TICK_US
    print("decode wave: R decode %.2f / %.2f / %.2f, barrier wait %.2f / %.2f / %.2f" % (
        np.median(d1), np.percentile(d1, 90), d1.max(), np.median(d2), np.percentile(d2, 90), d2.max()))
    s0 = (st[:, :, 0] - t0).ravel() * TICK_US
    print("wave start offsets from the first wave: median %.2f p90 %.2f max %.2f us" % (
        np.median(s0), np.percentile(s0, 90), s0.max()))


if __name__ == "__main__":
    main()
