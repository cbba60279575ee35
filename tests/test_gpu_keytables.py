"""GPU parity of the per-key tables of the throughput path (csrc/keytab.h,
csrc/sv_kernels.hip sv_keyslot_kernel / sv_keybuild_kernel): with the tables
on, a key's decoded -A and its table are built once and reused by every later
signature of that key.  Verdicts must not change:
  * repeated signers (a checkpoint-like set) through the device API, first
    call (keys claimed and built) and again (every key already built), and
    against the same batch with the tables off;
  * every adversarial fixture class (small-order / non-canonical / off-curve
    keys are cached as rejecting keys) through the host API;
  * every key given the same fingerprint (test knob): one slot, every other
    key a mismatch that must fall back to decoding inline;
  * tables smaller than the key set: claims stop, the tables are cleared and
    refilled;
  * auto mode: a host batch with repeated keys uses the tables, one with
    distinct keys does not.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev(sv):
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture
def tables(sv, dev):
    # (the per-key tables serve the one-lane kernels: medium launches would
    # otherwise take the quad geometry, which decodes every key itself)
    prev = sv.set_key_tables(1)
    sv.set_debug_flags(sv.DBG_NO_QUAD)
    yield sv
    sv.set_key_tables(prev)
    sv.set_debug_flags(0)


def repeated_set(sv, dev, keys, reps, seed):
    """keys x reps signatures (row r signed by key r % keys), 1 % of rows corrupted."""
    n = keys * reps
    rng = np.random.default_rng(seed)
    kseeds = rng.integers(0, 256, (keys, 32), dtype=np.uint8)
    seeds = torch.from_numpy(np.tile(kseeds, (reps, 1))).to(dev)
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), n, pk.data_ptr(), sig.data_ptr(), st)
    torch.cuda.synchronize(dev)
    bad = np.unique(rng.integers(0, n, n // 100))
    bt = torch.from_numpy(bad).to(dev)
    sig[bt, torch.from_numpy(32 + bad % 32).to(dev)] ^= 0x02
    want = np.ones(n, np.uint8)
    want[bad] = 0
    return pk, sig, msgs, want


def verify_dev(sv, dev, pk, sig, msgs):
    n = pk.shape[0]
    out = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    sv.verify_device(0, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), n, out.data_ptr(), 0, st)
    torch.cuda.synchronize(dev)
    return out.cpu().numpy()


def test_repeated_signers_device_api(tables, dev):
    sv = tables
    pk, sig, msgs, want = repeated_set(sv, dev, 4096, 64, seed=1)
    s0 = sv.key_cache_stats(0)
    assert np.array_equal(verify_dev(sv, dev, pk, sig, msgs), want)  # keys claimed and built
    assert np.array_equal(verify_dev(sv, dev, pk, sig, msgs), want)  # every key built before
    s1 = sv.key_cache_stats(0)
    assert s1["table_launches"] >= s0["table_launches"] + 2
    assert 0 < s1["table_keys"] <= s1["table_slots"] // 2
    sv.set_key_tables(0)
    assert np.array_equal(verify_dev(sv, dev, pk, sig, msgs), want)  # tables off: the same verdicts
    assert sv.key_cache_stats(0)["table_launches"] == s1["table_launches"]


def test_adversarial_keys_cached_as_rejecting(tables, golden):
    sv = tables
    d = golden["adversarial"]
    m = len(d["verdict"])
    reps = -(-16384 // m)  # (throughput path: > 12288 rows)
    pk = np.tile(d["pk"], (reps, 1))
    sig = np.tile(d["sig"], (reps, 1))
    off = np.tile(d["msg_off"], reps)
    ln = np.tile(d["msg_len"], reps)
    want = np.tile(d["verdict"], reps)
    for _ in range(2):
        out = sv.verify_batch(pk, sig, d["msg"], off, ln, device=0, path="throughput")
        bad = np.nonzero(out != want)[0]
        assert len(bad) == 0, [(int(i), str(d["class_names"][d["cls"][i % m]])) for i in bad[:10]]


def test_fingerprint_collisions_fall_back(tables, dev):
    sv = tables
    pk, sig, msgs, want = repeated_set(sv, dev, 512, 64, seed=2)
    sv.set_debug_flags(sv.DBG_KEY_COLLIDE | sv.DBG_NO_QUAD)
    for _ in range(2):
        assert np.array_equal(verify_dev(sv, dev, pk, sig, msgs), want)


def test_small_tables_clear_and_refill(tables, dev):
    sv = tables
    sv.set_key_tables(1, 1024)  # claims stop at 512 keys
    pk, sig, msgs, want = repeated_set(sv, dev, 3000, 16, seed=3)
    c0 = sv.key_cache_stats(0)["table_clears"]
    for _ in range(4):
        assert np.array_equal(verify_dev(sv, dev, pk, sig, msgs), want)
    st = sv.key_cache_stats(0)
    assert st["table_slots"] == 1024
    assert st["table_clears"] > c0
    sv.set_key_tables(1, 0)


def test_auto_mode_uses_tables_for_repeated_host_keys(sv, dev):
    prev = sv.set_key_tables(2)
    prev_dbg = sv.set_debug_flags(sv.DBG_NO_QUAD)
    try:
        pk, sig, msgs, want = repeated_set(sv, dev, 512, 64, seed=4)
        P, S, M = pk.cpu().numpy(), sig.cpu().numpy(), msgs.cpu().numpy()
        t0 = sv.key_cache_stats(0)["table_launches"]
        assert np.array_equal(sv.verify_fixed(P, S, M, 32, device=0), want)
        t1 = sv.key_cache_stats(0)["table_launches"]
        assert t1 > t0
        # distinct keys: no tables
        pk2, sig2, msgs2, want2 = repeated_set(sv, dev, 32768, 1, seed=5)
        out = sv.verify_fixed(pk2.cpu().numpy(), sig2.cpu().numpy(), msgs2.cpu().numpy(), 32, device=0)
        assert np.array_equal(out, want2)
        assert sv.key_cache_stats(0)["table_launches"] == t1
    finally:
        sv.set_key_tables(prev)
        sv.set_debug_flags(prev_dbg)
