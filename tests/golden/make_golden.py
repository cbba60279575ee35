#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the build container: verdicts come from libsodium 1.0.18
(/opt/conda/lib/libsodium.so.23.3.0, the version stellar-core's configure.ac
:284-289 accepts; its source is an empty submodule in the reference) through
ctypes, i.e. from the exact function PubKeyUtils::verifySig calls
(/root/reference/src/crypto/SecretKey.cpp:461-463).  Nothing here ships to the
GPU box except the .npz data it writes.

Fixture files (numpy .npz, allow_pickle=False):
  intree.npz     208 in-tree vectors parsed from the reference's own tests
                 (src/crypto/test/CryptoTests.cpp:518-625 IACR 2020/1244,
                 :643-1629 Zcash), with the reference's expected verdicts.
  valid.npz      deterministic valid set: seed_i = SHA-256("SVSEED"||u64le i),
                 msg_i = SHA-256("SVMSG"||u64le i)  
  msglen.npz     message lengths 0..512 (1- to 5-block SHA-512 paths, incl. the
                 128-384 B SCP statement range of config 4)
  longmsg.npz    messages of 513 B .. 64 KiB - 1 (survey responses carry an
                 EncryptedBody up to 64000 B, SurveyManager.cpp:388-393; large
                 SCP nominations, HerderImpl.cpp:2414-2432): valid rows, a byte
                 flipped in the first / last block, and signature mutations
                 (S + L, a flipped R or S bit, another key) over the same bytes
  adversarial.npz  mutation classes: bit flips in R/S/A/msg,
                 S+L / S+2L / S=L, small-order R and A (+/- bit 255),
                 non-canonical y>=p encodings, off-curve A, mixed-order
                 A = A'+T (T of order 2/4/8), random garbage.
  digests.json   SHA-256 digest of the valid-set stream pk||sig||msg for the
                 first 2^10, 2^16 and 2^20 signatures, so the GPU box can
                 regenerate the bench dataset and prove it is the same one.

Every fixture row carries (pk, sig, msg, libsodium verdict); the generator
also asserts the oracle (oracle/liboracle.so) agrees on every row.

Usage:  make -C oracle && python tests/golden/make_golden.py
"""
import ctypes
import hashlib
import json
import os
import re
import struct
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_TESTS = "/root/reference/src/crypto/test/CryptoTests.cpp"

sodium = ctypes.CDLL("/opt/conda/lib/libsodium.so.23")
assert sodium.sodium_init() >= 0
sodium.sodium_version_string.restype = ctypes.c_char_p
SODIUM_VERSION = sodium.sodium_version_string().decode()
oracle = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))

# ----------------------------------------------------------- curve helpers
P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)


def inv(x):
    return pow(x, P - 2, P)


def pt_add(p, q):
    (x1, y1), (x2, y2) = p, q
    t = D * x1 * x2 * y1 * y2 % P
    return ((x1 * y2 + x2 * y1) * inv(1 + t) % P, (y1 * y2 + x1 * x2) * inv(1 - t) % P)


def pt_mul(k, p):
    r, a = (0, 1), p
    while k:
        if k & 1:
            r = pt_add(r, a)
        a = pt_add(a, a)
        k >>= 1
    return r


def pt_enc(p):
    x, y = p
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def pt_dec(s):
    v = int.from_bytes(s, "little")
    y, sign = v & ((1 << 255) - 1), v >> 255
    if y >= P:
        return None
    x2 = (y * y - 1) * inv(D * y * y + 1) % P
    x = pow(x2, (P + 3) // 8, P)
    if (x * x - x2) % P:
        x = x * SQRTM1 % P
    if (x * x - x2) % P:
        return None
    if (x & 1) != sign:
        x = (P - x) % P
    return (x, y)


BY = 4 * inv(5) % P
B = pt_dec(BY.to_bytes(32, "little"))


def sha512_int(*parts):
    return int.from_bytes(hashlib.sha512(b"".join(parts)).digest(), "little")


# ------------------------------------------------------------ libsodium
def sod_keypair(seed):
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    assert sodium.crypto_sign_seed_keypair(pk, sk, seed) == 0
    return pk.raw, sk.raw


def sod_sign(msg, sk):
    sig = ctypes.create_string_buffer(64)
    sodium.crypto_sign_detached(sig, None, msg, ctypes.c_ulonglong(len(msg)), sk)
    return sig.raw


def sod_verify(sig, msg, pk):
    return int(sodium.crypto_sign_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0)


def orc_verify(sig, msg, pk):
    return int(oracle.oracle_ed25519_verify(sig, msg, ctypes.c_size_t(len(msg)), pk) == 0)


def seed_of(i):
    return hashlib.sha256(b"SVSEED" + struct.pack("<Q", i)).digest()


def msg_of(i):
    return hashlib.sha256(b"SVMSG" + struct.pack("<Q", i)).digest()


# ------------------------------------------------------------ fixture IO
class Rows:
    def __init__(self):
        self.pk, self.sig, self.msg, self.cls, self.expect = [], [], [], [], []
        self.classes = {}

    def add(self, cls, pk, sig, msg, expect=-1):
        assert len(pk) == 32 and len(sig) == 64
        cid = self.classes.setdefault(cls, len(self.classes))
        self.pk.append(pk)
        self.sig.append(sig)
        self.msg.append(msg)
        self.cls.append(cid)
        self.expect.append(expect)

    def save(self, name, share=False):
        """share: rows with identical message bytes point at one copy (msg_off),
        so signature-mutation rows over a long message cost no extra bytes."""
        n = len(self.pk)
        verdict = np.array([sod_verify(s, m, p) for p, s, m in zip(self.pk, self.sig, self.msg)], np.uint8)
        orc = np.array([orc_verify(s, m, p) for p, s, m in zip(self.pk, self.sig, self.msg)], np.uint8)
        assert (verdict == orc).all(), "oracle disagrees with libsodium at rows %s" % np.nonzero(verdict != orc)[0][:10]
        exp = np.array(self.expect, np.int8)
        has = exp >= 0
        assert (exp[has] == verdict[has]).all(), "libsodium disagrees with the reference's expected verdicts"
        lens = np.array([len(m) for m in self.msg], np.uint32)
        off = np.zeros(n, np.uint64)
        if share:
            at, parts, pos = {}, [], 0
            for i, m in enumerate(self.msg):
                if m not in at:
                    at[m] = pos
                    parts.append(m)
                    pos += len(m)
                off[i] = at[m]
            blob = b"".join(parts)
        else:
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            blob = b"".join(self.msg)
        np.savez_compressed(
            os.path.join(HERE, name),
            pk=np.frombuffer(b"".join(self.pk), np.uint8).reshape(n, 32),
            sig=np.frombuffer(b"".join(self.sig), np.uint8).reshape(n, 64),
            msg=np.frombuffer(blob or b"", np.uint8),
            msg_off=off, msg_len=lens, verdict=verdict,
            cls=np.array(self.cls, np.uint16), expect=exp,
            class_names=np.array(sorted(self.classes, key=self.classes.get)),
        )
        print("%-16s %6d rows, %5d accepted, classes=%d" % (name, n, int(verdict.sum()), len(self.classes)))


# ------------------------------------------------------------ sets
def intree():
    src = open(REF_TESTS).read()
    rows = Rows()
    iacr = src[src.index("IACR_2020_1244_TEST_VECTORS[12]"):src.index("TEST_CASE(\"Ed25519 test vectors from IACR")]
    ents = re.findall(r'Iacr20201244TestVector\{\s*"([0-9a-f]+)",\s*"([0-9a-f]+)",\s*((?:"[0-9a-f]+"\s*)+),\s*(true|false)', iacr)
    assert len(ents) == 12, len(ents)
    for msg, pk, sigparts, fail in ents:
        sig = "".join(re.findall(r'"([0-9a-f]+)"', sigparts))
        rows.add("iacr2020_1244", bytes.fromhex(pk), bytes.fromhex(sig), bytes.fromhex(msg), 0 if fail == "true" else 1)
    zc = src[src.index("ZCASH_TEST_VECTORS[196]"):src.index("TEST_CASE(\"Ed25519 test vectors from Zcash")]
    ents = re.findall(r'ZcashTestVector\{\s*"([0-9a-f]+)",\s*((?:"[0-9a-f]+"\s*)+),?\s*\}', zc)
    assert len(ents) == 196, len(ents)
    for pk, sigparts in ents:
        sig = "".join(re.findall(r'"([0-9a-f]+)"', sigparts))
        rows.add("zcash", bytes.fromhex(pk), bytes.fromhex(sig), b"Zcash", 0)
    rows.save("intree.npz")


def valid(n=1024):
    rows = Rows()
    for i in range(n):
        pk, sk = sod_keypair(seed_of(i))
        m = msg_of(i)
        rows.add("valid32", pk, sod_sign(m, sk), m, 1)
    # reference benchmark shape: 256-byte messages (SecretKey.cpp:182-189)
    for i in range(64):
        pk, sk = sod_keypair(seed_of(1_000_000 + i))
        m = hashlib.shake_256(b"SVMSG256" + struct.pack("<Q", i)).digest(256)
        rows.add("valid256", pk, sod_sign(m, sk), m, 1)
    rows.save("valid.npz")


def msglen():
    rows = Rows()
    for ln in range(0, 513):
        pk, sk = sod_keypair(seed_of(2_000_000 + ln))
        m = hashlib.shake_256(b"LEN" + struct.pack("<Q", ln)).digest(ln) if ln else b""
        s = sod_sign(m, sk)
        rows.add("msglen_valid", pk, s, m, 1)
        if ln:
            mm = bytearray(m)
            mm[ln // 2] ^= 0x40
            rows.add("msglen_flip", pk, s, bytes(mm), 0)
    rows.save("msglen.npz")


LONG_LENS = (513, 575, 576, 639, 640, 767, 768, 1023, 1024, 1025, 2047, 2048, 4095, 4096, 8191, 16384, 32768,
             65535)


def longmsg():
    """Messages past 512 B: every length is a valid libsodium signature, the
    same message with one byte flipped in its first and in its last SHA-512
    block (R||A||M: the first block holds M[0..63]), and over the valid bytes
    S + L, one flipped bit of R and of S, and a different signer's key."""
    rows = Rows()
    for k, ln in enumerate(LONG_LENS):
        pk, sk = sod_keypair(seed_of(4_000_000 + k))
        m = hashlib.shake_256(b"LONG" + struct.pack("<Q", ln)).digest(ln)
        s = sod_sign(m, sk)
        rows.add("long_valid", pk, s, m, 1)
        mm = bytearray(m); mm[ln - 1] ^= 0x01
        rows.add("long_flip_last", pk, s, bytes(mm), 0)
        if ln <= 4096:
            mm = bytearray(m); mm[0] ^= 0x80
            rows.add("long_flip_first", pk, s, bytes(mm), 0)
        S = int.from_bytes(s[32:], "little")
        rows.add("long_S_plus_L", pk, s[:32] + (S + L).to_bytes(32, "little"), m, 0)
        sb = bytearray(s); sb[7] ^= 0x10
        rows.add("long_flip_R", pk, bytes(sb), m, 0)
        sb = bytearray(s); sb[40] ^= 0x02
        rows.add("long_flip_S", pk, bytes(sb), m, 0)
        pk2, _ = sod_keypair(seed_of(4_100_000 + k))
        rows.add("long_other_key", pk2, s, m, 0)
    rows.save("longmsg.npz", share=True)


BLACKLIST = [
    bytes(32),
    b"\x01" + bytes(31),
    bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"),
    bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"),
    (P - 1).to_bytes(32, "little"),
    P.to_bytes(32, "little"),
    (P + 1).to_bytes(32, "little"),
]


def adversarial():
    rows = Rows()
    rng = np.random.default_rng(20250211)
    base = []
    for i in range(48):
        pk, sk = sod_keypair(seed_of(3_000_000 + i))
        m = msg_of(3_000_000 + i)
        base.append((pk, sk, m, sod_sign(m, sk)))
    # bit flips
    for k, (pk, sk, m, s) in enumerate(base[:16]):
        for bit in range(0, 256, 3 + k % 5):
            sb = bytearray(s); sb[bit // 8] ^= 1 << (bit % 8)
            rows.add("flip_R", pk, bytes(sb), m, 0)
            sb = bytearray(s); sb[32 + bit // 8] ^= 1 << (bit % 8)
            rows.add("flip_S", pk, bytes(sb), m)
            pb = bytearray(pk); pb[bit // 8] ^= 1 << (bit % 8)
            rows.add("flip_A", bytes(pb), s, m)
            mb = bytearray(m); mb[bit // 8] ^= 1 << (bit % 8)
            rows.add("flip_msg", pk, s, bytes(mb), 0)
    # S + kL, S = L, S = L - 1, S with high bits
    for pk, sk, m, s in base[:24]:
        S = int.from_bytes(s[32:], "little")
        for k in (1, 2, 3, 15):
            if S + k * L < 2**256:
                rows.add("S_plus_kL", pk, s[:32] + (S + k * L).to_bytes(32, "little"), m, 0)
        rows.add("S_eq_L", pk, s[:32] + L.to_bytes(32, "little"), m, 0)
        rows.add("S_eq_Lm1", pk, s[:32] + (L - 1).to_bytes(32, "little"), m)
        rows.add("S_top_bits", pk, s[:32] + (S | (0xF << 252)).to_bytes(32, "little"), m, 0)
        rows.add("S_bit252_only", pk, s[:32] + (S ^ (1 << 252)).to_bytes(32, "little"), m)
    # small-order R and A with and without bit 255
    pk0, sk0, m0, s0 = base[0]
    for enc in BLACKLIST:
        for hb in (0, 0x80):
            e = bytearray(enc); e[31] |= hb; e = bytes(e)
            rows.add("smallorder_R", pk0, e + s0[32:], m0, 0)
            rows.add("smallorder_A", e, s0, m0, 0)
            rows.add("smallorder_A_and_R", e, e + bytes(32), m0, 0)
    # non-canonical y >= p encodings (both sign bits) for A and R
    for k in range(0, 19):
        for hb in (0, 0x80):
            e = bytearray((P + k).to_bytes(32, "little")); e[31] |= hb; e = bytes(e)
            rows.add("noncanon_A", e, s0, m0, 0)
            rows.add("noncanon_R", pk0, e + s0[32:], m0, 0)
    # y in [2^255-19, 2^255) i.e. the top of the range, again both signs
    for k in range(1, 20):
        e = bytearray((2**255 - k).to_bytes(32, "little"))
        rows.add("noncanon_A_top", bytes(e), s0, m0, 0)
        e[31] |= 0x80
        rows.add("noncanon_A_top", bytes(e), s0, m0, 0)
    # off-curve A: random y with no square root
    cnt = 0
    while cnt < 96:
        y = int(rng.integers(0, 2**62)) * 2**190 + int(rng.integers(0, 2**62))
        y %= P
        if pt_dec(y.to_bytes(32, "little")) is None:
            enc = bytearray(y.to_bytes(32, "little")); enc[31] |= 0x80 * (cnt & 1)
            rows.add("offcurve_A", bytes(enc), s0, m0, 0)
            cnt += 1
    # x = 0 with the sign bit set for A (y = 1 and y = p-1): blacklisted after masking
    rows.add("x0_sign_A", (1 | (1 << 255)).to_bytes(32, "little"), s0, m0, 0)
    rows.add("x0_sign_A", ((P - 1) | (1 << 255)).to_bytes(32, "little"), s0, m0, 0)
    # mixed-order keys A = a'B + T, signed with a': accepted iff [h]T = O
    T8 = pt_dec(BLACKLIST[2])
    torsion = {8: T8, 4: pt_add(T8, T8), 2: pt_mul(4, T8)}
    acc_mixed = 0
    for i in range(512):
        order = (8, 4, 2)[i % 3]
        a = int.from_bytes(hashlib.sha256(b"MIXED" + struct.pack("<Q", i)).digest(), "little") % L
        A = pt_add(pt_mul(a, B), pt_mul(1 + (i % (order - 1)), torsion[order]) if order > 2 else torsion[2])
        Aenc = pt_enc(A)
        m = hashlib.sha256(b"MIXEDMSG" + struct.pack("<Q", i)).digest()
        r = sha512_int(b"NONCE", struct.pack("<Q", i)) % L
        Renc = pt_enc(pt_mul(r, B))
        h = sha512_int(Renc, Aenc, m) % L
        S = (r + h * a) % L
        sig = Renc + S.to_bytes(32, "little")
        rows.add("mixed_order_A_%d" % order, Aenc, sig, m)
        acc_mixed += sod_verify(sig, m, Aenc)
    # mixed-order R: R = rB + T8 with S computed for R (verifies iff never: R' is the prime-order part)
    for i in range(64):
        pk, sk, m, _ = base[i % len(base)]
        a_bytes = hashlib.sha512(sk[:32]).digest()[:32]
        a = int.from_bytes(a_bytes, "little")
        a &= ~7; a &= (1 << 254) - 1; a |= 1 << 254
        r = sha512_int(b"MIXR", struct.pack("<Q", i)) % L
        Renc = pt_enc(pt_add(pt_mul(r, B), pt_mul(1 + i % 7, T8)))
        h = sha512_int(Renc, pk, m) % L
        S = (r + h * a) % L
        rows.add("mixed_order_R", pk, Renc + S.to_bytes(32, "little"), m, 0)
    # sign-bit flips on A and R of valid signatures
    for pk, sk, m, s in base:
        pb = bytearray(pk); pb[31] ^= 0x80
        rows.add("signflip_A", bytes(pb), s, m, 0)
        sb = bytearray(s); sb[31] ^= 0x80
        rows.add("signflip_R", pk, bytes(sb), m, 0)
        rows.add("valid_ctrl", pk, s, m, 1)
    # random garbage
    for i in range(256):
        g = rng.integers(0, 256, 96, dtype=np.uint8).tobytes()
        rows.add("garbage", g[:32], g[32:], msg_of(i), 0)
    print("  mixed-order keys accepted by libsodium: %d / 512" % acc_mixed)
    rows.save("adversarial.npz")


def dataset_digests():
    """Digests of the deterministic valid-set stream pk||sig||msg."""
    out = {"scheme": "seed_i=SHA256('SVSEED'||u64le(i)), msg_i=SHA256('SVMSG'||u64le(i)), "
                     "digest=SHA256(concat_i pk_i||sig_i||msg_i)", "libsodium": SODIUM_VERSION}
    todo = [1 << 10, 1 << 16, 1 << 20]
    top = todo[-1]

    def work(lo):
        buf = bytearray()
        for i in range(lo, min(lo + 4096, top)):
            pk, sk = sod_keypair(seed_of(i))
            m = msg_of(i)
            buf += pk + sod_sign(m, sk) + m
        return bytes(buf)

    h = hashlib.sha256()
    done = 0
    with ThreadPoolExecutor(max_workers=8) as ex:
        for chunk in ex.map(work, range(0, top, 4096)):
            for k in range(0, len(chunk), 128):
                h.update(chunk[k:k + 128])
                done += 1
                if done in todo:
                    out[str(done)] = h.copy().hexdigest()
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("digests", out)


if __name__ == "__main__":
    print("libsodium", SODIUM_VERSION)
    which = sys.argv[1:] or ["intree", "valid", "msglen", "longmsg", "adversarial", "digests"]
    if "intree" in which: intree()
    if "valid" in which: valid()
    if "msglen" in which: msglen()
    if "longmsg" in which: longmsg()
    if "adversarial" in which: adversarial()
    if "digests" in which: dataset_digests()
