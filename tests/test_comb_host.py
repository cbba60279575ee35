"""CPU checks of the warm-key latency path (stellar-core_amd/csrc/comb.h).

* The comb equation and table layout: a host build of the path's algorithm
  (tests/native/host_core.cpp hc_comb_verify_batch: per-key tables of
  d * 16^j * (-A), base tables of e * 256^j * B, 96-entry sums, projective test
  against the decoded R) must give libsodium's verdict on every golden row.
* The host key index (csrc/keycache.h: open addressing with backward-shift
  deletion, CLOCK eviction, second-sighting admission when full) against a map
  model under random and colliding traffic.
The GPU kernels themselves are checked in tests/test_gpu_comb.py.
"""
import ctypes

import numpy as np
import pytest


@pytest.mark.parametrize("name", ["intree", "lattice_edge", "valid", "msglen", "adversarial"])
def test_comb_model_matches_golden(hostcore, golden, name):
    d = golden[name]
    n = len(d["verdict"])
    if name in ("valid", "adversarial"):
        n = min(n, 1500)  # (keeps the CPU suite short; the GPU test runs every row)
    pk = np.ascontiguousarray(d["pk"][:n])
    sig = np.ascontiguousarray(d["sig"][:n])
    msg = np.ascontiguousarray(d["msg"])
    off = np.ascontiguousarray(d["msg_off"][:n])
    ln = np.ascontiguousarray(d["msg_len"][:n])
    out = np.zeros(n, np.uint8)
    f = hostcore.hc_comb_verify_batch
    f.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_void_p]
    f(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, off.ctypes.data, ln.ctypes.data, n, out.ctypes.data)
    bad = np.nonzero(out != d["verdict"][:n])[0]
    assert len(bad) == 0, [(int(i), str(d["class_names"][d["cls"][i]])) for i in bad[:10]]


@pytest.mark.parametrize("seed,cap,ops,universe", [(1, 16, 20000, 40), (2, 64, 50000, 70), (3, 64, 50000, 1000),
                                                   (4, 1024, 100000, 1500), (5, 1, 5000, 3)])
def test_key_index_fuzz(hostcore, seed, cap, ops, universe):
    f = hostcore.hc_keyindex_fuzz
    f.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    assert f(seed, cap, ops, universe) == 0
