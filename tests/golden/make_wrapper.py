#!/usr/bin/env python3
"""Generate tests/golden/wrapper.json: fixtures that pin the C++ mirror of the
reference's signature WRAPPER logic, i.e. the layers above
crypto_sign_verify_detached, against the reference's own tests:

  pubkey_signature  src/transactions/test/SignatureUtilsTest.cpp:15-32: keys
                    SecretKey::fromSeed(sha256("NODE_SEED_" + i)), messages
                    sha256("HASH_" + i + j), i, j < 10; SignatureUtils::sign ->
                    SignatureUtils::verify must hold.
  hashx             SignatureUtilsTest.cpp:34-48: x = 'A' * i, i <= 64; the HASH_X
                    signer sha256(x) with signature x must verify.
  sign_tests        src/crypto/test/CryptoTests.cpp:272-297: a good signature of
                    "hello", the wrong message "helloo", and sig[4] ^= 1.  (The
                    reference draws its key pseudo-randomly; the key here is
                    fromSeed(sha256("sign tests")).)
  envelopes         src/transactions/test/TxEnvelopeTests.cpp:396-736: the outer
                    envelope cases (no signature, bad signature, wrong hint, signed
                    twice, unused signature) and the multisig cases (not enough
                    rights, success with two signatures, without master key,
                    account locked down, duplicate signature), each as the ledger
                    state the test builds (accounts, thresholds, signers) plus the
                    envelope, with the result code the reference test REQUIREs for
                    protocol >= 8 and, where the test states it, protocol 7.
                    Keys: fromSeed(sha256(name)).  Contents hashes: sha256 of the
                    case name (the checker only signs/verifies the 32-byte hash).
                    A few fee-bump cases follow the reference's logic
                    (FeeBumpTransactionFrame.cpp:173-197) with expectations derived
                    from it (marked "derived": no reference test states them).

Signatures come from libsodium 1.0.18 (/opt/conda/lib/libsodium.so.23) in this
container only; the JSON ships, nothing else.
Usage:  python tests/golden/make_wrapper.py
"""
import ctypes
import hashlib
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
sodium = ctypes.CDLL("/opt/conda/lib/libsodium.so.23")
assert sodium.sodium_init() >= 0

LOW, MED, HIGH = 1, 2, 3
ED25519, PRE_AUTH_TX, HASH_X, SIGNED_PAYLOAD = 0, 1, 2, 3


def keypair(seed):
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    assert sodium.crypto_sign_seed_keypair(pk, sk, seed) == 0
    return pk.raw, sk.raw


def sign(msg, sk):
    s = ctypes.create_string_buffer(64)
    sodium.crypto_sign_detached(s, None, msg, ctypes.c_ulonglong(len(msg)), sk)
    return s.raw


def verify(sig, msg, pk):
    return sodium.crypto_sign_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0


def sha256(b):
    return hashlib.sha256(b).digest()


def named(name):
    return keypair(sha256(name.encode()))


def dsig(pk, sk, h):
    return {"hint": pk[-4:].hex(), "sig": sign(h, sk).hex()}


def pubkey_signature():
    rows = []
    for i in range(10):
        pk, sk = keypair(sha256(b"NODE_SEED_" + str(i).encode()))
        for j in range(10):
            h = sha256(b"HASH_" + str(i).encode() + str(j).encode())
            s = sign(h, sk)
            assert verify(s, h, pk)
            rows.append({"pk": pk.hex(), "msg": h.hex(), "hint": pk[-4:].hex(), "sig": s.hex(), "expect": 1})
    return rows


def hashx():
    rows = []
    for i in range(65):
        x = b"A" * i
        key = sha256(x)
        rows.append({"key": key.hex(), "hint": key[-4:].hex(), "sig": x.hex(), "expect": 1})
    return rows


def sign_tests():
    pk, sk = keypair(sha256(b"sign tests"))
    s = sign(b"hello", sk)
    bad = bytearray(s)
    bad[4] ^= 1
    rows = [
        {"case": "good", "pk": pk.hex(), "sig": s.hex(), "msg": b"hello".hex(), "expect": 1},
        {"case": "bad message", "pk": pk.hex(), "sig": s.hex(), "msg": b"helloo".hex(), "expect": 0},
        {"case": "bad signature", "pk": pk.hex(), "sig": bytes(bad).hex(), "msg": b"hello".hex(), "expect": 0},
    ]
    for r in rows:
        assert verify(bytes.fromhex(r["sig"]), bytes.fromhex(r["msg"]), pk) == bool(r["expect"])
    return rows


def account(pk, master=1, low=0, med=0, high=0, signers=()):
    return {"id": pk.hex(), "thresholds": [master, low, med, high],
            "signers": [{"type": ED25519, "key": k.hex(), "weight": w} for k, w in signers]}


def envelopes():
    root_pk, root_sk = named("root")
    a_pk, a_sk = named("A")
    s1_pk, s1_sk = named("S1")
    s2_pk, s2_sk = named("S2")
    bogus_pk, bogus_sk = named("bogus")
    cases = []

    def case(name, accounts, source, ops, sigs, p_ge8, p7=None, ref="", fee_bump=None):
        c = {"name": name, "ref": ref, "accounts": accounts, "source": source.hex(), "hash": sha256(name.encode()).hex(),
             "ops": ops, "sigs": sigs, "expect": {"21": p_ge8, "8": p_ge8}}
        if p7 is not None:
            c["expect"]["7"] = p7
        if fee_bump:
            c["fee_bump"] = fee_bump
        cases.append(c)
        return c

    def h(name):
        return sha256(name.encode())

    root = account(root_pk)
    multisig = account(a_pk, 100, 10, 50, 100, [(s1_pk, 5), (s2_pk, 95)])
    op_med = [{"source": None, "level": MED}]  # createAccount / payment need MEDIUM
    op_high = [{"source": None, "level": HIGH}]  # setOptions with thresholds / signers needs HIGH
    R = "TxEnvelopeTests.cpp"
    # outer envelope (:396-500): root.tx({createAccount(a1)}) -- A does not exist
    case("no signature", [root], root_pk, op_med, [], {"code": -6}, {"code": 0}, R + ":399-416")
    case("bad signature", [root], root_pk, op_med,
         [{"hint": root_pk[-4:].hex(), "sig": bytes([123] * 32).hex()}], {"code": -6}, {"code": 0}, R + ":418-436")
    c = case("bad signature (wrong hint)", [root], root_pk, op_med, [], {"code": -6}, {"code": 0}, R + ":438-456")
    c["sigs"] = [{"hint": "01010101", "sig": sign(h(c["name"]), root_sk).hex()}]
    c = case("too many signatures (signed twice)", [root], root_pk, op_med, [], {"code": -10}, {"code": 0},
             R + ":458-476")
    c["sigs"] = [dsig(root_pk, root_sk, h(c["name"])), dsig(a_pk, a_sk, h(c["name"]))]
    c = case("too many signatures (unused signature)", [root], root_pk, op_med, [], {"code": -10}, {"code": 0},
             R + ":478-499")
    c["sigs"] = [dsig(root_pk, root_sk, h(c["name"])), dsig(bogus_pk, bogus_sk, h(c["name"]))]
    # multisig (:502-736): A: master 100, low 10, med 50, high 100, S1 weight 5, S2 weight 95
    accts = [root, multisig]

    def ms(name, ops, signers_, p_ge8, p7=None, lines="", accounts=None):
        c = case(name, accounts or accts, a_pk, ops, [], p_ge8, p7, R + ":" + lines)
        c["sigs"] = [dsig(pk, sk, h(name)) for pk, sk in signers_]
        return c

    ms("not enough rights (envelope)", op_med, [(s1_pk, s1_sk)], {"code": -6}, {"code": 0}, "515-538")
    ms("not enough rights (operation, together)", op_high, [(s2_pk, s2_sk)],
       {"code": -1, "failed_op": 0, "op_code": -1}, {"code": 0}, "540-565")
    ms("not enough rights (first thresholds)", op_high + op_high, [(s2_pk, s2_sk)],
       {"code": -1, "failed_op": 0, "op_code": -1}, {"code": 0}, "567-592")
    ms("not enough rights (first signer)", op_high + op_high, [(s2_pk, s2_sk)],
       {"code": -1, "failed_op": 0, "op_code": -1}, {"code": 0}, "594-619")
    ms("success two signatures, together", op_high, [(s1_pk, s1_sk), (s2_pk, s2_sk)], {"code": 0}, {"code": 0},
       "621-636")
    ms("success two signatures, first thresholds", op_high + op_high, [(s1_pk, s1_sk), (s2_pk, s2_sk)],
       {"code": 0}, {"code": 0}, "638-653")
    ms("success two signatures, first signer", op_high + op_high, [(s1_pk, s1_sk), (s2_pk, s2_sk)],
       {"code": 0}, {"code": 0}, "655-670")
    nomaster = account(a_pk, 0, 10, 50, 100, [(s1_pk, 5), (s2_pk, 95)])
    ms("without master key (good tx)", op_med, [(s2_pk, s2_sk)], {"code": 0}, None, "672-700",
       accounts=[root, nomaster])
    ms("without master key (master key is extra)", op_med, [(a_pk, a_sk), (s2_pk, s2_sk)], {"code": -10}, None,
       "672-700", accounts=[root, nomaster])
    c = case("account locked down", [account(root_pk, 0)], root_pk, op_med, [], {"code": -6}, None, R + ":702-709")
    c["sigs"] = [dsig(root_pk, root_sk, h(c["name"]))]
    c = ms("do not allow duplicate signature", op_med, [(s1_pk, s1_sk)] * 10, {"code": -6}, {"code": 0}, "711-735")
    # fee bump (derived from FeeBumpTransactionFrame.cpp:173-197, 267-287; protocol >= 13)
    for name, outer, p in [
        ("fee bump: valid outer and inner", [(root_pk, root_sk)], {"code": 1, "inner_code": 0}),
        ("fee bump: missing outer signature", [], {"code": -6}),
        ("fee bump: unused outer signature", [(root_pk, root_sk), (bogus_pk, bogus_sk)], {"code": -10}),
    ]:
        fb_hash = sha256(("FB " + name).encode())
        c = case(name, accts, a_pk, op_med, [], dict(p), None, "derived: FeeBumpTransactionFrame.cpp:173-197",
                 fee_bump={"hash": fb_hash.hex(), "fee_source": root_pk.hex(),
                           "sigs": [dsig(pk, sk, fb_hash) for pk, sk in outer]})
        c["sigs"] = [dsig(s2_pk, s2_sk, h(name))]  # inner: S2 (95) clears MED 50
        c["expect"].pop("8")
    name = "fee bump: inner not authorized"
    fb_hash = sha256(("FB " + name).encode())
    c = case(name, accts, a_pk, op_med, [], {"code": -13, "inner_code": -6}, None,
             "derived: FeeBumpTransactionFrame.cpp:173-197",
             fee_bump={"hash": fb_hash.hex(), "fee_source": root_pk.hex(), "sigs": [dsig(root_pk, root_sk, fb_hash)]})
    c["sigs"] = [dsig(s1_pk, s1_sk, h(name))]  # inner: S1 (5) < LOW 10
    c["expect"].pop("8")
    return cases


def main():
    out = {"libsodium": "1.0.18", "pubkey_signature": pubkey_signature(), "hashx": hashx(),
           "sign_tests": sign_tests(), "envelopes": envelopes()}
    with open(os.path.join(HERE, "wrapper.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrapper.json: %d pubkey, %d hashx, %d sign, %d envelope cases" % (
        len(out["pubkey_signature"]), len(out["hashx"]), len(out["sign_tests"]), len(out["envelopes"])))


if __name__ == "__main__":
    main()
