"""GPU parity for messages longer than 512 bytes.

Survey responses sign `xdr_to_opaque(response)` with an EncryptedBody of up to
64000 B (/root/reference/src/overlay/SurveyManager.cpp:388-393,423-425), and
nominate statements with many votes pass 512 B (HerderImpl.cpp:2414-2432,
Peer.cpp:963-970); all of them reach PubKeyUtils::verifySig.  The fixture
tests/golden/longmsg.npz (libsodium 1.0.18-signed, make_golden.py longmsg)
covers 513 B .. 64 KiB - 1; a 1 MiB message is signed here by the oracle.

Every kernel path is exercised: auto / throughput (prep + main) / latency
(octet) / warm comb, the keyed pass (BLAKE2b keys on the GPU), the gather entry
point, the device-resident variable-length form, and the host staging
pipeline with long messages on both sides of a staging-chunk boundary.  The
mixed-wave cases put one long message among 32-byte ones, so per-lane SHA-512
block loops diverge inside one wave (throughput), one quad (octet) and one
chain wave (comb).
"""
import hashlib
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(sv):
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    return 0


@pytest.fixture(params=["auto", "throughput", "quad", "latency"])
def path(request, sv):
    """The per-call path; "throughput" forces the one-lane kernels and "quad"
    one signature per quad of lanes (the throughput path's two geometries)."""
    geom = {"throughput": sv.DBG_NO_QUAD, "quad": sv.DBG_QUAD}.get(request.param, 0)
    prev = sv.set_debug_flags(geom)
    yield "throughput" if request.param == "quad" else request.param
    sv.set_debug_flags(prev)


def _rows(d, rows):
    """Sub-batch of a fixture (messages copied out, packed anew)."""
    msgs = [d["msg"][int(d["msg_off"][i]):int(d["msg_off"][i]) + int(d["msg_len"][i])].tobytes() for i in rows]
    return d["pk"][rows], d["sig"][rows], msgs, d["verdict"][rows]


def _pack(msgs):
    ln = np.array([len(m) for m in msgs], np.uint32)
    off = np.zeros(len(msgs), np.uint64)
    if len(msgs) > 1:
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(msgs) or b"\0", np.uint8)
    return buf, off, ln


def _mixed(golden, n, long_at):
    """n rows of libsodium-signed 32-byte messages (every 5th corrupted) with
    the long-message fixture's rows placed at positions long_at (cycling)."""
    v, lm = golden["valid"], golden["longmsg"]
    r32 = np.nonzero(v["msg_len"] == 32)[0]
    src = [r32[i % len(r32)] for i in range(n)]
    pk, sig, msgs, want = _rows(v, src)
    pk, sig, want = pk.copy(), sig.copy(), want.copy()
    sig[::5, 33] ^= 0x08
    want[::5] = 0
    lpk, lsig, lmsgs, lwant = _rows(lm, np.arange(len(lm["verdict"])))
    for j, pos in enumerate(long_at):
        k = j % len(lmsgs)
        pk[pos], sig[pos], msgs[pos], want[pos] = lpk[k], lsig[k], lmsgs[k], lwant[k]
    return pk, sig, msgs, want


def test_longmsg_fixture_every_path(sv, gpu, golden, path):
    d = golden["longmsg"]
    out = sv.verify_batch(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"], device=0, path=path)
    bad = np.nonzero(out != d["verdict"])[0]
    assert len(bad) == 0, [(int(i), int(d["msg_len"][i]), str(d["class_names"][d["cls"][i]])) for i in bad[:10]]
    assert int(d["verdict"].sum()) == 18 and int(d["msg_len"].max()) == 65535


@pytest.mark.parametrize("n,long_at", [(64, [17]), (64, [0, 63]), (257, [3, 64, 65, 200]), (1000, list(range(0, 1000, 97)))])
def test_one_long_lane_in_short_waves(sv, gpu, golden, path, n, long_at):
    pk, sig, msgs, want = _mixed(golden, n, long_at)
    buf, off, ln = _pack(msgs)
    out = sv.verify_batch(pk, sig, buf, off, ln, device=0, path=path)
    assert np.array_equal(out, want), np.nonzero(out != want)[0][:10]


def test_longmsg_warm_comb(sv, gpu, golden):
    """The fixture again once its keys are in the device key cache (the comb
    kernel hashes R||A||M on every lane of the chain wave), then a mixed
    short/long batch over the same warm keys."""
    from test_gpu_comb import _warm_up  # noqa: E402  (same process, same binding)
    sv.set_key_cache(8192)
    try:
        d = golden["longmsg"]
        assert _warm_up(sv, d, d["verdict"]) >= 1
        pk, sig, msgs, want = _mixed(golden, 300, [0, 1, 2, 64, 150, 299])
        buf, off, ln = _pack(msgs)
        dm = {"pk": pk, "sig": sig, "msg": buf, "msg_off": off, "msg_len": ln}
        _warm_up(sv, dm, want)
    finally:
        sv.set_key_cache(1024)


def test_longmsg_keyed_and_gather(sv, gpu, golden):
    d = golden["longmsg"]
    v, k = sv.verify_batch_keyed(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"])
    assert np.array_equal(v, d["verdict"])
    pk, sig, msgs, want = _rows(d, np.arange(len(d["verdict"])))
    for i in range(len(msgs)):
        assert k[i].tobytes() == hashlib.blake2b(pk[i].tobytes() + sig[i].tobytes() + msgs[i],
                                                 digest_size=32).digest(), i
    items = [(pk[i].tobytes(), sig[i].tobytes(), msgs[i]) for i in range(len(msgs))]
    gv, gk = sv.verify_gather(items, keys=True, device=0)
    assert np.array_equal(gv, want) and np.array_equal(gk, k)


def test_longmsg_device_api_variable_length(sv, gpu, golden):
    """sv_ed25519_verify_device with msg_off / msg_len in HBM (the catchup /
    tx-set form), one long row among short ones, both kernel paths by size."""
    dev = torch.device("cuda", 0)
    for n in (100, 20000):
        pk, sig, msgs, want = _mixed(golden, n, [n // 3, n - 1])
        buf, off, ln = _pack(msgs)
        t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (pk, sig, buf)]
        toff = torch.from_numpy(off.view(np.int64)).to(dev)
        tln = torch.from_numpy(ln.view(np.int32)).to(dev)
        tv = torch.full((n,), 9, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        sv.verify_device(0, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), n, tv.data_ptr(), stream=st,
                         fixed_msg_len=0, d_msg_off=toff.data_ptr(), d_msg_len=tln.data_ptr())
        torch.cuda.synchronize(dev)
        assert np.array_equal(tv.cpu().numpy(), want), n


def test_staging_chunk_boundary_with_long_messages(sv, gpu, golden):
    """A host batch of 70,000 rows runs as staging chunks of 65,536 (the ramp's
    first chunk, a quarter of 2^18) and the rest; long messages sit on both
    sides of the boundary and at the ends."""
    n = 70000
    at = [0, 1000, 65534, 65535, 65536, 65537, 69999]
    pk, sig, msgs, want = _mixed(golden, n, at)
    buf, off, ln = _pack(msgs)
    out = sv.verify_batch(pk, sig, buf, off, ln, device=0)
    assert np.array_equal(out, want), np.nonzero(out != want)[0][:10]


def test_one_mib_message(sv, gpu, oracle, path):
    """A 1 MiB message signed by the oracle's RFC 8032 signer (checker-side
    fixture), valid and with its last byte flipped, beside short rows."""
    seed = hashlib.sha256(b"MIB").digest()
    import ctypes
    pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    oracle.oracle_ed25519_seed_keypair(pk, sk, seed)
    m = hashlib.shake_256(b"MIB" + struct.pack("<Q", 1 << 20)).digest(1 << 20)
    s = ctypes.create_string_buffer(64)
    oracle.oracle_ed25519_sign(s, m, len(m), sk)
    bad = bytearray(m)
    bad[-1] ^= 1
    pks = np.frombuffer(pk.raw * 3, np.uint8).reshape(3, 32)
    sigs = np.frombuffer(s.raw * 3, np.uint8).reshape(3, 64)
    msgs = [m, bytes(bad), m[:32]]
    buf, off, ln = _pack(msgs)
    want = np.array([oracle.oracle_ed25519_verify(s.raw, x, len(x), pk.raw) == 0 for x in msgs], np.uint8)
    assert want.tolist() == [1, 0, 0]
    out = sv.verify_batch(pks, sigs, buf, off, ln, device=0, path=path)
    assert np.array_equal(out, want)
