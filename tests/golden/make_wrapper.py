#!/usr/bin/env python3
"""Generate tests/golden/wrapper.json (and derived.json): fixtures that pin the C++ mirror of the
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
  envelopes         src/transactions/test/TxEnvelopeTests.cpp:98-395 (ed25519
                    payload signers, extraSigners), :396-736 (outer envelope and
                    multisig), :738-1637 (pre-auth / HASH_X / payload signers
                    standing in for keys, alone and in multisig) and
                    FeeBumpTransactionTests.cpp:117-216 (fee source missing, outer
                    signature missing / invalid / extra, inner unauthorized): each
                    as the ledger state the test builds (accounts, thresholds,
                    signers) plus the envelope, with the result code the test
                    REQUIREs for the protocol versions it states.  Keys:
                    fromSeed(sha256(name)).  Contents hashes: sha256 of the case
                    name (the checker only signs/verifies the 32-byte hash).  The
                    missing-op-source cases, which no reference test states, are
                    written to derived.json instead (their source lines cited).
  value_sigs        src/herder/test/HerderTests.cpp:2052-2115: StellarValue
                    signatures (HerderImpl.cpp:2440-2449 verifies the node's
                    signature over xdr(networkID, ENVELOPE_TYPE_SCPVALUE, txSetHash,
                    closeTime)): valid, missing signature, wrong signature, wrong
                    node ID.

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
    """signers: (pk, weight) pairs (ED25519) or signer dicts (signer())."""
    return {"id": pk.hex(), "thresholds": [master, low, med, high],
            "signers": [s if isinstance(s, dict) else {"type": ED25519, "key": s[0].hex(), "weight": s[1]}
                        for s in signers]}


def signer(kind, key, weight=1, payload=b""):
    return {"type": kind, "key": key.hex(), "weight": weight, "payload": payload.hex()}


def hint_of(b):
    """SignatureUtils::getHint (SignatureUtils.cpp:107-122): the last 4 bytes,
    or the bytes zero-padded when shorter."""
    return (b + bytes(4))[:4] if len(b) < 4 else b[-4:]


def payload_hint(pk, payload):
    """getSignedPayloadHint (SignatureUtils.cpp:93-105)."""
    return bytes(a ^ b for a, b in zip(hint_of(pk), hint_of(payload)))


def payload_sig(pk, sk, payload):
    return {"hint": payload_hint(pk, payload).hex(), "sig": sign(payload, sk).hex()}


def hashx_sig(x):
    return {"hint": sha256(x)[-4:].hex(), "sig": x.hex()}


def envelopes():
    root_pk, root_sk = named("root")
    a_pk, a_sk = named("A")
    s1_pk, s1_sk = named("S1")
    s2_pk, s2_sk = named("S2")
    bogus_pk, bogus_sk = named("bogus")
    cases = []

    def case(name, accounts, source, ops, sigs, p_ge8, p7=None, ref="", fee_bump=None, extra=(), protos=("21", "8")):
        c = {"name": name, "ref": ref, "accounts": accounts, "source": source.hex(), "hash": sha256(name.encode()).hex(),
             "ops": ops, "sigs": sigs, "expect": {p: p_ge8 for p in protos}}
        if p7 is not None:
            c["expect"]["7"] = p7
        if fee_bump:
            c["fee_bump"] = fee_bump
        if extra:
            c["extra"] = list(extra)
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
    # fee bump: src/transactions/test/FeeBumpTransactionTests.cpp, feeBumpUnsigned(acc, root, root, ...):
    # fee source A (created: master 1, thresholds 0), inner transaction from root (payment to root)
    FB = "FeeBumpTransactionTests.cpp:"
    fee_pk, fee_sk = named("fee bump A")

    def fb(name, outer, inner_signed, p, lines, fee_exists=True, outer_hash=None):
        fb_hash = sha256(("FB " + name).encode())
        signed_over = outer_hash or fb_hash
        accs = [root, account(fee_pk)] if fee_exists else [root]
        c = case(name, accs, root_pk, op_med, [], dict(p), None, FB + lines, protos=("21", "13"),
                 fee_bump={"hash": fb_hash.hex(), "fee_source": fee_pk.hex(),
                           "sigs": [dsig(pk, sk, signed_over) for pk, sk in outer]})
        c["sigs"] = [dsig(root_pk, root_sk, h(name))] if inner_signed else []
        return c

    fb("fee bump: fee source does not exist", [(fee_pk, fee_sk)], True, {"code": -8}, "117-128", fee_exists=False)
    fb("fee bump: bad signatures, signature missing", [], True, {"code": -6}, "130-145")
    # signed in the wrong order: the outer signature covers another fee-bump hash
    fb("fee bump: bad signatures, signature invalid", [(fee_pk, fee_sk)], True, {"code": -6}, "147-164",
       outer_hash=sha256(b"fee bump signed before its inner signature"))
    fb("fee bump: extra signatures", [(fee_pk, fee_sk), (root_pk, root_sk)], True, {"code": -10}, "177-195")
    fb("fee bump: inner transaction invalid, transaction level", [(fee_pk, fee_sk)], False,
       {"code": -13, "inner_code": -6}, "197-216")
    fb("fee bump: valid outer and inner", [(fee_pk, fee_sk)], True, {"code": 1, "inner_code": 0},
       "43-60 (the valid fee bump every other section starts from)")
    payload_and_extra_signer_cases(root_pk, root_sk, case, h)
    alternative_signature_cases(root_pk, root_sk, s1_pk, s1_sk, case, h)
    return cases


def payload_and_extra_signer_cases(root_pk, root_sk, case, h):
    """TxEnvelopeTests.cpp:98-256 (ed25519 payload signer) and :257-395
    (extraSigners), protocol >= 19.  a1 = root.create("a1"): master weight 1,
    thresholds 0.  transactionWithV2Precondition(a1, ...) is a payment signed by
    a1 (TxTests.cpp:676-722)."""
    R = "TxEnvelopeTests.cpp:"
    a1_pk, a1_sk = named("a1 payload")
    root = account(root_pk)
    pay = [{"source": None, "level": MED}]

    def on_a1(signers_):
        return [root, account(a1_pk, signers=signers_)]

    for label, payload, lines in [("3 byte payload", b"a12", "158-161"), ("4 byte payload", b"a123", "162-165"),
                                  ("5 byte payload", b"a1234", "166-169")]:
        name = "payload signer: " + label
        case(name, on_a1([signer(SIGNED_PAYLOAD, root_pk, 1, payload)]), a1_pk, pay,
             [payload_sig(root_pk, root_sk, payload)], {"code": 0}, None, R + lines + ",120-141", protos=("21",))
    # payload = tx2's contents hash; the same signature then signs tx2 itself
    h2 = h("payload signer: payload is tx (tx2)")
    case("payload signer: payload is tx", on_a1([signer(SIGNED_PAYLOAD, root_pk, 1, h2)]), a1_pk, pay,
         [payload_sig(root_pk, root_sk, h2)], {"code": 0}, None, R + "170-180,120-156", protos=("21",))
    c = case("payload signer: payload is tx (tx2)", [root, account(a1_pk)], root_pk, pay,
             [{"hint": root_pk[-4:].hex(), "sig": sign(h2, root_sk).hex()}], {"code": 0}, None,
             R + "143-155", protos=("21",))
    c["hash"] = h2.hex()
    aaa = b"aaa"
    for sub, extra_sig, p in [("success", True, {"code": 0}), ("fail", False, {"code": -6})]:
        name = "payload signer in extra signers: " + sub
        sigs = [dsig(a1_pk, a1_sk, h(name))] + ([payload_sig(root_pk, root_sk, aaa)] if extra_sig else [])
        case(name, [root, account(a1_pk)], a1_pk, pay, sigs, p, None, R + "181-205", protos=("21",),
             extra=[signer(SIGNED_PAYLOAD, root_pk, 1, aaa)])
    zero = bytes(32)
    name = "payload signer with zeroed out ed25519"
    case(name, [root, account(a1_pk, 1, 255, 0, 0, [signer(SIGNED_PAYLOAD, zero, 1, aaa)])], a1_pk, pay,
         [payload_sig_hint(zero, aaa, root_sk), dsig(a1_pk, a1_sk, h(name))], {"code": -6}, None, R + "206-231",
         protos=("21",))
    # extraSigners (:257-395): rootSigner = root's ed25519 key, hashXSigner = sha256("hashx")
    rs = signer(ED25519, root_pk)
    hx = signer(HASH_X, sha256(b"hashx"))
    for label, extra, with_sigs, p, lines in [
            ("one extra signer: success", [rs], ["root"], {"code": 0}, "271-280"),
            ("one extra signer: fail", [rs], [], {"code": -6}, "281-285"),
            ("one extra hashx signer: success", [hx], ["hashx"], {"code": 0}, "287-296"),
            ("one extra hashx signer: fail", [hx], [], {"code": -6}, "297-301"),
            ("two extra signers: success", [rs, hx], ["root", "hashx"], {"code": 0}, "303-315"),
            ("two extra signers: fail", [rs, hx], ["root"], {"code": -6}, "316-320")]:
        name = "extraSigners: " + label
        sigs = [dsig(a1_pk, a1_sk, h(name))]
        for w in with_sigs:
            sigs.append(dsig(root_pk, root_sk, h(name)) if w == "root" else hashx_sig(b"hashx"))
        case(name, [root, account(a1_pk)], a1_pk, pay, sigs, p, None, R + lines, protos=("21",), extra=extra)
    name = "extraSigners: signer overlap with default account signer"
    case(name, [root], root_pk, pay, [dsig(root_pk, root_sk, h(name))], {"code": 0}, None, R + "343-349",
         protos=("21",), extra=[rs])
    for sub, present, p, lines in [("signature present", True, {"code": 0}, "357-361"),
                                   ("signature missing", False, {"code": -6}, "362-366")]:
        name = "extraSigners: signer overlap with added account signer: " + sub
        sigs = [dsig(a1_pk, a1_sk, h(name))] + ([dsig(root_pk, root_sk, h(name))] if present else [])
        case(name, [root, account(a1_pk, signers=[(root_pk, 100)])], a1_pk, pay, sigs, p, None,
             R + "350-367", protos=("21",), extra=[rs])
    name = "extraSigners: signer overlap with added account signer - both signers used"
    case(name, [root, account(a1_pk, signers=[(root_pk, 100)])], a1_pk,
         [{"source": root_pk.hex(), "level": MED}],
         [dsig(a1_pk, a1_sk, h(name)), dsig(root_pk, root_sk, h(name))], {"code": 0}, None, R + "368-379",
         protos=("21",), extra=[rs])
    name = "extraSigners: preauth signer"
    case(name, [root, account(a1_pk)], a1_pk, pay, [dsig(a1_pk, a1_sk, h(name)), dsig(a1_pk, a1_sk, h(name))],
         {"code": -6}, None, R + "380-392", protos=("21",),
         extra=[signer(PRE_AUTH_TX, h("root.tx({}) of the preauth section"))])


def payload_sig_hint(pk_for_hint, payload, sk):
    """A payload signature by sk whose hint is computed for another key."""
    return {"hint": payload_hint(pk_for_hint, payload).hex(), "sig": sign(payload, sk).hex()}


def alternative_signature_cases(root_pk, root_sk, s1_pk, s1_sk, case, h):
    """TxEnvelopeTests.cpp:738-1676, "alternative signatures": the same account
    scenarios with a pre-auth (hash tx), HASH_X (x with embedded zeros) or
    ed25519 signed-payload signer standing in for a key.  a1 = root.create("A")
    (master 1, thresholds 0); the multisig sections first set master 100,
    thresholds 10 / 50 / 100 and S1 at weight 95 (:1094-1100).  Result codes as
    the tests REQUIRE for protocol >= 10 (and 7 where stated); the signer
    removals the tests also check are ledger state, not signature checks."""
    R = "TxEnvelopeTests.cpp:"
    a1_pk, a1_sk = named("A alternative")
    root = account(root_pk)
    x = bytes([97, 98, 99, 0, 100, 101, 102, 0, 0, 0, 103, 104, 105, 106, 107, 108,
               65, 66, 67, 0, 68, 69, 70, 0, 0, 0, 71, 72, 73, 74, 75, 76])
    pay = [{"source": None, "level": MED}]
    alts = [("hash tx", 0), ("hash x", 0), ("payload signer", 19)]

    def alt_signer(kind, name, weight, corrupt=False):
        if kind == "hash tx":
            k = bytearray(h(name))
            if corrupt:
                k[0] ^= 1
            return signer(PRE_AUTH_TX, bytes(k), weight)
        if kind == "hash x":
            k = bytearray(sha256(x))
            if corrupt:
                k[0] ^= 1
            return signer(HASH_X, bytes(k), weight)
        k = bytearray(root_pk)
        if corrupt:
            k[0] ^= 1
        return signer(SIGNED_PAYLOAD, bytes(k), weight, x)

    def alt_sigs(kind):
        if kind == "hash tx":
            return []
        if kind == "hash x":
            return [hashx_sig(x)]
        return [payload_sig(root_pk, root_sk, x)]

    for kind, minp in alts:
        protos = ("21",) if minp >= 19 else ("21", "10")

        def alt_case(label, accounts_of, source, ops, pre_sigs, p, p7, lines):
            name = "alternative %s: %s" % (kind, label)
            accts = accounts_of(name)
            c = case(name, accts, source, ops, [], p, p7 if minp < 7 else None, R + lines, protos=protos)
            c["sigs"] = [s(name) if callable(s) else s for s in pre_sigs] + alt_sigs(kind)
            return c

        alt_case("invalid signature", lambda n: [root, account(a1_pk, signers=[alt_signer(kind, n, 1, True)])],
                 a1_pk, pay, [], {"code": -6}, {"code": 0}, "837-877")
        alt_case("too many signatures (signed by owner)",
                 lambda n: [root, account(a1_pk, signers=[alt_signer(kind, n, 1)])], a1_pk, pay,
                 [lambda n: dsig(a1_pk, a1_sk, h(n))], {"code": -10}, {"code": 0}, "879-915")
        alt_case("success", lambda n: [root, account(a1_pk, signers=[alt_signer(kind, n, 1)])], a1_pk, pay, [],
                 {"code": 0}, {"code": 0}, "917-950")
        # merge source account before payment (:952-1058): b1 is merged away before the
        # payment applies -- the op source (checkSignatureNoAccount: b1's key never
        # signed) or the transaction source goes missing
        b1_pk, _ = named("b1 alternative")
        for sub, src, ops, p, lines in [
                ("merge op source account", a1_pk, [{"source": b1_pk.hex(), "level": MED},
                                                    {"source": root_pk.hex(), "level": MED}],
                 {"code": -1}, "1010-1021,1049-1052"),
                ("merge tx source account", b1_pk, [{"source": a1_pk.hex(), "level": MED},
                                                    {"source": root_pk.hex(), "level": MED}],
                 {"code": -8}, "1010-1019,1054-1057")]:
            name = "alternative %s: %s" % (kind, sub)
            c = case(name, [account(root_pk, signers=[alt_signer(kind, name, 1)]),
                            account(a1_pk, signers=[alt_signer(kind, name, 1)])], src, ops, alt_sigs(kind), p,
                     None, R + lines, protos=("21",))
            c["apply_only"] = True  # (b1 existed at validation; the test states the apply outcome)
        ms = lambda n, w: [root, account(a1_pk, 100, 10, 50, 100, [(s1_pk, 95), alt_signer(kind, n, w)])]
        alt_case("multisig: not enough rights (envelope)", lambda n: ms(n, 5), a1_pk, pay, [], {"code": -6},
                 {"code": 0}, "1102-1136")
        alt_case("multisig: not enough rights (envelope), same signer on tx and op source account",
                 lambda n: [account(root_pk, signers=[alt_signer(kind, n, 5)]),
                            account(a1_pk, 100, 10, 50, 100, [(s1_pk, 95), alt_signer(kind, n, 5)])],
                 a1_pk, [{"source": root_pk.hex(), "level": MED}], [], {"code": -6}, {"code": 0}, "1138-1184")
        alt_case("multisig: not enough rights (operation)", lambda n: ms(n, 95), a1_pk,
                 [{"source": None, "level": HIGH}], [], {"code": -1, "failed_op": 0, "op_code": -1}, {"code": 0},
                 "1215-1252")
        if minp < 10:
            c = alt_case("multisig: signatures removed from multiple accounts even though transaction failed",
                         lambda n: [account(root_pk, signers=[alt_signer(kind, n, 1)]),
                                    account(a1_pk, 100, 10, 50, 100, [(s1_pk, 95), alt_signer(kind, n, 1)])],
                         a1_pk, [{"source": root_pk.hex(), "level": MED}],
                         [lambda n: dsig(s1_pk, s1_sk, h(n)), lambda n: dsig(s1_pk, s1_sk, h(n))], {"code": -10},
                         None, "1316-1352")
            c["expect"] = {"10": {"code": -10}, "9": {"code": -10}}
        c = alt_case("multisig: success signature", lambda n: [root, account(a1_pk, 100, 10, 100, 100,
                                                                             [(s1_pk, 95), alt_signer(kind, n, 5)])],
                     a1_pk, pay, [lambda n: dsig(s1_pk, s1_sk, h(n))], {"code": 0}, {"code": 0}, "1513-1546")
        alt_case("in op source account signers",
                 lambda n: [account(root_pk, signers=[alt_signer(kind, n, 1)]),
                            account(a1_pk, signers=[alt_signer(kind, n, 1)])], root_pk,
                 [{"source": a1_pk.hex(), "level": MED}], [], {"code": 0}, {"code": 0}, "1549-1580")
        alt_case("in multiple ops source account signers",
                 lambda n: [account(root_pk, signers=[alt_signer(kind, n, 1)]),
                            account(a1_pk, signers=[alt_signer(kind, n, 1)])], root_pk,
                 [{"source": a1_pk.hex(), "level": MED}] * 2, [], {"code": 0}, {"code": 0}, "1581-1612")
    name = "alternative: empty X"
    c = case(name, [root, account(a1_pk, 100, 10, 50, 100, [(s1_pk, 95), signer(HASH_X, sha256(x), 5)])], a1_pk,
             pay, [dsig(s1_pk, s1_sk, h(name)), hashx_sig(x)], {"code": 0}, None, R + "1614-1637",
             protos=("21", "10"))
    # missing operation source account, both modes: OperationFrame::checkSignature
    # with forApply = false (TransactionFrame.cpp:1130-1131 passes false on apply too) checks a
    # missing op-source account by its own key (checkSignatureNoAccount, :186-207)
    m_pk, m_sk = named("missing op source")
    bogus_pk, bogus_sk = named("bogus op source")
    for sub, who, p in [("signed by the missing account's key", ["root", "m"], {"code": 0}),
                        ("not signed by it", ["root"], {"code": -1, "failed_op": 0, "op_code": -1}),
                        ("with an extra signature", ["root", "m", "bogus"], {"code": -10})]:
        name = "missing op source account: " + sub
        keys = {"root": (root_pk, root_sk), "m": (m_pk, m_sk), "bogus": (bogus_pk, bogus_sk)}
        case(name, [root], root_pk, [{"source": m_pk.hex(), "level": MED}],
             [dsig(keys[k][0], keys[k][1], h(name)) for k in who], p, None,
             "derived: OperationFrame.cpp:186-207, TransactionFrame.cpp:1130-1131 (no reference test states it)",
             protos=("21",))


def value_sigs():
    """HerderTests.cpp:2052-2115 through verifySig (HerderImpl.cpp:2440-2449)."""
    import struct
    node_pk, node_sk = named("herder node")
    network_id = sha256(b"Test SDF Network ; September 2015")
    ENVELOPE_TYPE_SCPVALUE = 4
    tx_set_hash = sha256(b"txSet0")
    close_time = 1700000000
    msg = network_id + struct.pack(">i", ENVELOPE_TYPE_SCPVALUE) + tx_set_hash + struct.pack(">Q", close_time)
    assert len(msg) == 76
    s = sign(msg, node_sk)
    bad = bytearray(s)
    bad[0] ^= 1
    wrong_node = bytearray(node_pk)
    wrong_node[0] ^= 1
    rows = [("valid", node_pk, s, 1, "2068-2077"), ("missing signature", node_pk, b"", 0, "2096-2100"),
            ("wrong signature", node_pk, bytes(bad), 0, "2101-2105"),
            ("wrong signature 2", bytes(wrong_node), s, 0, "2106-2110")]
    out = []
    for name, pk, sig, expect, lines in rows:
        assert (len(sig) == 64 and verify(sig, msg, pk)) == bool(expect)
        out.append({"case": name, "ref": "HerderTests.cpp:" + lines, "pk": pk.hex(), "sig": sig.hex(),
                    "msg": msg.hex(), "expect": expect})
    return out


def main():
    env = envelopes()
    # reference-pinned cases only in wrapper.json; the cases no reference test
    # states (their source lines cited) go to derived.json
    out = {"libsodium": "1.0.18", "pubkey_signature": pubkey_signature(), "hashx": hashx(),
           "sign_tests": sign_tests(), "envelopes": [c for c in env if not c["ref"].startswith("derived")],
           "value_sigs": value_sigs()}
    derived = {"libsodium": "1.0.18", "envelopes": [c for c in env if c["ref"].startswith("derived")]}
    with open(os.path.join(HERE, "wrapper.json"), "w") as f:
        json.dump(out, f, indent=0)
    with open(os.path.join(HERE, "derived.json"), "w") as f:
        json.dump(derived, f, indent=0)
    print("derived.json: %d envelope cases" % len(derived["envelopes"]))
    print("wrapper.json: %d pubkey, %d hashx, %d sign, %d envelope cases, %d value signatures" % (
        len(out["pubkey_signature"]), len(out["hashx"]), len(out["sign_tests"]), len(out["envelopes"]),
        len(out["value_sigs"])))


if __name__ == "__main__":
    main()
