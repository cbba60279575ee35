"""The engine's CPU path (sv_ed25519_verify_batch_cpu / sv_ed25519_verify_cpu):
the same per-signature algorithm as the GPU kernels (verify_core.h, the
half-size equation of lattice.h) compiled for the host.  It is product code --
what a caller runs when a GPU entry point fails, and what single verifySig
calls use -- so it must give libsodium's verdicts on every fixture class.  No
GPU needed; the oracle is only the checker here (the fixtures' verdicts are
libsodium's own)."""
import ctypes

import numpy as np
import pytest

from conftest import oracle_verdicts


@pytest.mark.parametrize("name", ["intree", "valid", "msglen", "longmsg", "adversarial", "lattice_edge"])
def test_cpu_path_matches_golden(sv, golden, name):
    d = golden[name]
    out = sv.verify_batch_cpu(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"], threads=4)
    bad = np.nonzero(out != d["verdict"])[0]
    assert len(bad) == 0, [(int(i), str(d["class_names"][d["cls"][i]])) for i in bad[:10]]


def test_cpu_path_reference_expectations(sv, golden):
    d = golden["intree"]
    out = sv.verify_batch_cpu(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"])
    iacr = d["expect"] >= 0
    assert (out[iacr] == d["expect"][iacr]).all()
    assert out[12:].sum() == 0  # all 196 Zcash vectors rejected (CryptoTests.cpp:643-1644)


def test_cpu_single_matches_batch(sv, golden):
    lib = sv.load_library()
    d = golden["adversarial"]
    for i in range(0, len(d["verdict"]), 97):
        o, ln = int(d["msg_off"][i]), int(d["msg_len"][i])
        m = d["msg"][o:o + ln].tobytes()
        r = lib.sv_ed25519_verify_cpu(d["pk"][i].tobytes(), d["sig"][i].tobytes(), m if ln else None, ln)
        assert r == d["verdict"][i], i


def test_cpu_path_random_mutations_vs_oracle(sv, golden, oracle):
    """Fresh mutations of valid rows (not fixture rows): CPU path == oracle."""
    rng = np.random.default_rng(99)
    d = golden["valid"]
    rows = rng.choice(len(d["verdict"]), 96, replace=False)
    pk = d["pk"][rows].copy()
    sig = d["sig"][rows].copy()
    off = d["msg_off"][rows]
    ln = d["msg_len"][rows]
    for k in range(len(rows)):
        if k % 3 == 1:
            sig[k, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
        elif k % 3 == 2:
            pk[k, rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)
    dd = {"pk": pk, "sig": sig, "msg": d["msg"], "msg_off": off, "msg_len": ln, "verdict": np.zeros(len(rows))}
    out = sv.verify_batch_cpu(pk, sig, d["msg"], off, ln, threads=2)
    assert np.array_equal(out, oracle_verdicts(oracle, dd))


def test_cpu_path_empty_and_bad_args(sv):
    lib = sv.load_library()
    assert lib.sv_ed25519_verify_batch_cpu(None, None, None, None, None, 0, None, 0) == 0
    assert lib.sv_ed25519_verify_batch_cpu(None, None, None, None, None, 3, None, 0) == -1
    assert lib.sv_ed25519_verify_cpu(None, None, None, 0) == -1
