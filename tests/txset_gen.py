"""Synthetic transaction sets for the SignatureChecker path (BASELINE config 3).

Each tx has 1..20 ED25519 signers (weights and a threshold that force k
signatures), its signatures shuffled so the hint matching
(SignatureUtils.cpp:127-136) is exercised, and ~1% of txs carry a signature
from a wrong key whose DecoratedSignature hint is forged to collide with a
real signer's hint.  Some txs also mix in PRE_AUTH_TX / HASH_X /
ED25519_SIGNED_PAYLOAD signers and unused extra signatures so every branch of
SignatureChecker.cpp:30-158 is reached.

`replay` is an independent Python restatement of the greedy checker used as
the CPU reference for the C++ mirror.
"""
import ctypes
import hashlib
import struct

import numpy as np

ED25519, PRE_AUTH_TX, HASH_X, SIGNED_PAYLOAD = 0, 1, 2, 3


class svh_signer(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint8), ("key", ctypes.c_uint8 * 32), ("weight", ctypes.c_uint32),
                ("payload_len", ctypes.c_uint32), ("payload", ctypes.c_uint8 * 64)]


class svh_decorated_sig(ctypes.Structure):
    _fields_ = [("hint", ctypes.c_uint8 * 4), ("sig_len", ctypes.c_uint32), ("sig", ctypes.c_uint8 * 64)]


class svh_tx(ctypes.Structure):
    _fields_ = [("contents_hash", ctypes.c_uint8 * 32), ("protocol", ctypes.c_uint32),
                ("needed_weight", ctypes.c_int32), ("nsigs", ctypes.c_uint32), ("sig_off", ctypes.c_uint32),
                ("nsigners", ctypes.c_uint32), ("signer_off", ctypes.c_uint32)]


def hint_of(b):
    return bytes(b[-4:]) if len(b) >= 4 else bytes(b) + bytes(4 - len(b))


def payload_hint(key, payload):
    a, b = hint_of(key), hint_of(payload) if payload else bytes(4)
    return bytes(x ^ y for x, y in zip(a, b))


def generate(n_tx, sign_fn, seed=7, protocol=21, extra_types=True):
    """sign_fn(list of (seed32, msg bytes)) -> list of (pk32, sig64)."""
    rng = np.random.default_rng(seed)
    txs = []
    requests = []
    for t in range(n_tx):
        h = hashlib.sha256(b"TX" + struct.pack("<QQ", seed, t)).digest()
        k = int(rng.integers(1, 21))
        need = int(rng.integers(1, k + 1))
        keys = [hashlib.sha256(b"ACCT" + struct.pack("<QQQ", seed, t, j)).digest() for j in range(k)]
        tx = {"hash": h, "k": k, "need_sigs": need, "seeds": keys, "signers": [], "sigs": [], "protocol": protocol}
        for j in range(k):
            requests.append((keys[j], h))
        txs.append(tx)
    signed = sign_fn(requests)
    pos = 0
    for t, tx in enumerate(txs):
        k = tx["k"]
        pairs = signed[pos:pos + k]
        pos += k
        # each signer weight 1, threshold = need_sigs: exactly need_sigs valid signatures required
        for j in range(k):
            tx["signers"].append({"type": ED25519, "key": pairs[j][0], "weight": 1, "payload": b""})
        chosen = list(rng.choice(k, tx["need_sigs"], replace=False))
        sigs = [{"hint": hint_of(pairs[j][0]), "sig": pairs[j][1]} for j in chosen]
        r = rng.random()
        if r < 0.01 and k > 1:
            # wrong key, forged colliding hint (signature of another signer's key)
            victim = chosen[0]
            other = (victim + 1) % k
            sigs[0] = {"hint": hint_of(pairs[victim][0]), "sig": pairs[other][1]}
        elif r < 0.03:
            sigs.append({"hint": b"\x00\x01\x02\x03", "sig": bytes(64)})  # unused extra signature
        elif r < 0.05:
            sigs.append({"hint": hint_of(pairs[chosen[0]][0]), "sig": pairs[chosen[0]][1][:63]})  # short
        if extra_types and r > 0.95:
            pre = tx["hash"]
            tx["signers"].append({"type": PRE_AUTH_TX, "key": pre, "weight": 1, "payload": b""})
            x = rng.bytes(int(rng.integers(1, 64)))
            hx = hashlib.sha256(x).digest()
            tx["signers"].append({"type": HASH_X, "key": hx, "weight": 1, "payload": b""})
            sigs.append({"hint": hint_of(hx), "sig": x})
            tx["protocol"] = 19 if r > 0.99 else protocol
        if extra_types and 0.90 < r <= 0.95:
            # signed payload signer: key j signs the payload
            payload = rng.bytes(int(rng.integers(1, 65)))
            j = int(rng.integers(0, k))
            tx["signers"].append({"type": SIGNED_PAYLOAD, "key": pairs[j][0], "weight": 2, "payload": payload,
                                  "_seed": tx["seeds"][j]})
            tx["need_payload"] = (tx["seeds"][j], payload)
        order = rng.permutation(len(sigs))
        tx["sigs"] = [sigs[i] for i in order]
        tx["needed"] = tx["need_sigs"]
        if r > 0.998:
            tx["protocol"] = 7
    return txs


def add_payload_signatures(txs, sign_var_fn):
    """Sign the signed-payload payloads (variable-length) with sign_var_fn([(seed, msg)])."""
    reqs = [tx["need_payload"] for tx in txs if "need_payload" in tx]
    out = sign_var_fn(reqs) if reqs else []
    i = 0
    for tx in txs:
        if "need_payload" in tx:
            seed, payload = tx["need_payload"]
            pk, sig = out[i]
            i += 1
            tx["sigs"].append({"hint": payload_hint(pk, payload), "sig": sig})


def to_ctypes(txs):
    n_sig = sum(len(t["sigs"]) for t in txs)
    n_sgn = sum(len(t["signers"]) for t in txs)
    T = (svh_tx * len(txs))()
    S = (svh_decorated_sig * max(1, n_sig))()
    G = (svh_signer * max(1, n_sgn))()
    si = gi = 0
    for i, tx in enumerate(txs):
        T[i].contents_hash[:] = list(tx["hash"])
        T[i].protocol = tx["protocol"]
        T[i].needed_weight = tx["needed"]
        T[i].nsigs, T[i].sig_off = len(tx["sigs"]), si
        T[i].nsigners, T[i].signer_off = len(tx["signers"]), gi
        for s in tx["sigs"]:
            S[si].hint[:] = list(s["hint"])
            S[si].sig_len = len(s["sig"])
            S[si].sig[:len(s["sig"])] = list(s["sig"])
            si += 1
        for g in tx["signers"]:
            G[gi].type = g["type"]
            G[gi].key[:] = list(g["key"])
            G[gi].weight = g["weight"]
            G[gi].payload_len = len(g["payload"])
            G[gi].payload[:len(g["payload"])] = list(g["payload"])
            gi += 1
    return T, S, G


def replay(txs, verify):
    """Independent restatement of SignatureChecker.cpp:30-158; verify(pk, sig, msg) -> bool."""
    ok, used_all = [], []
    for tx in txs:
        if tx["protocol"] == 7:
            ok.append(1)
            used_all.append(1)
            continue
        sigs = tx["sigs"]
        used = [False] * len(sigs)
        by = {ED25519: [], PRE_AUTH_TX: [], HASH_X: [], SIGNED_PAYLOAD: []}
        for g in tx["signers"]:
            by[g["type"]].append(g)
        total = 0
        clamp = (lambda w: min(w, 255)) if tx["protocol"] >= 10 else (lambda w: w)
        done = False
        for g in by[PRE_AUTH_TX]:
            if g["key"] == tx["hash"]:
                total += clamp(g["weight"])
                if total >= tx["needed"]:
                    done = True
                    break

        def verify_all(signers, fn):
            nonlocal total
            for i, s in enumerate(sigs):
                for g in list(signers):
                    if fn(s, g):
                        used[i] = True
                        total += clamp(g["weight"])
                        if total >= tx["needed"]:
                            return True
                        signers.remove(g)
                        break
            return False

        def v_hashx(s, g):
            return s["hint"] == hint_of(g["key"]) and hashlib.sha256(s["sig"]).digest() == g["key"]

        def v_ed(s, g):
            return s["hint"] == hint_of(g["key"]) and len(s["sig"]) == 64 and verify(g["key"], s["sig"], tx["hash"])

        def v_sp(s, g):
            return (s["hint"] == payload_hint(g["key"], g["payload"]) and len(s["sig"]) == 64
                    and verify(g["key"], s["sig"], g["payload"]))

        if not done:
            done = (verify_all(by[HASH_X], v_hashx) or verify_all(by[ED25519], v_ed)
                    or verify_all(by[SIGNED_PAYLOAD], v_sp))
        ok.append(1 if done else 0)
        used_all.append(1 if all(used) else 0)
    return np.array(ok, np.uint8), np.array(used_all, np.uint8)


# ---------------------------------------------------------------------------
# Transaction-level replay (tests/golden/wrapper.json "envelopes"): an
# independent Python restatement of the reference's signature checks of one
# envelope -- TransactionFrame.cpp:268-321 (checkSignature /
# checkSignatureNoAccount / checkExtraSigners), :1091-1156 (processSignatures),
# :1247-1262 (commonValid), OperationFrame.cpp:173-209 and
# FeeBumpTransactionFrame.cpp:138-197 -- over ONE checker per envelope whose
# used-signature marks persist across its calls (SignatureChecker.cpp:30-158).

TX_NO_ACCOUNT, TX_BAD_AUTH, TX_BAD_AUTH_EXTRA, TX_FAILED = -8, -6, -10, -1
OP_BAD_AUTH, OP_NO_ACCOUNT = -1, -2


class Checker:
    def __init__(self, protocol, contents_hash, sigs, verify):
        self.protocol, self.hash, self.sigs, self.verify = protocol, contents_hash, sigs, verify
        self.used = [False] * len(sigs)

    def check(self, signers, needed):
        if self.protocol == 7:
            return True
        by = {ED25519: [], PRE_AUTH_TX: [], HASH_X: [], SIGNED_PAYLOAD: []}
        for g in signers:
            by[g["type"]].append(g)
        clamp = (lambda w: min(w, 255)) if self.protocol >= 10 else (lambda w: w)
        total = 0
        for g in by[PRE_AUTH_TX]:
            if g["key"] == self.hash:
                total += clamp(g["weight"])
                if total >= needed:
                    return True

        def run(signers_, match):
            nonlocal total
            for i, s in enumerate(self.sigs):
                for g in list(signers_):
                    if match(s, g):
                        self.used[i] = True
                        total += clamp(g["weight"])
                        if total >= needed:
                            return True
                        signers_.remove(g)
                        break
            return False

        def hx(s, g):
            return s["hint"] == hint_of(g["key"]) and hashlib.sha256(s["sig"]).digest() == g["key"]

        def ed(s, g):
            return s["hint"] == hint_of(g["key"]) and len(s["sig"]) == 64 and self.verify(g["key"], s["sig"], self.hash)

        def sp(s, g):
            return (self.protocol >= 19 and s["hint"] == payload_hint(g["key"], g["payload"]) and len(s["sig"]) == 64
                    and self.verify(g["key"], s["sig"], g["payload"]))

        return run(by[HASH_X], hx) or run(by[ED25519], ed) or run(by[SIGNED_PAYLOAD], sp)

    def all_used(self):
        return self.protocol == 7 or all(self.used)


def _signers_of(acc):
    out = []
    if acc["thresholds"][0]:
        out.append({"type": ED25519, "key": acc["id"], "weight": acc["thresholds"][0], "payload": b""})
    return out + [dict(g) for g in acc["signers"]]


def replay_envelope(case, protocol, for_apply, verify):
    """{"code", "inner_code", "failed_op", "op_code"} of one wrapper.json case."""
    def b(x):
        return bytes.fromhex(x) if isinstance(x, str) else x

    accounts = {}
    for a in case["accounts"]:
        accounts[b(a["id"])] = {"id": b(a["id"]), "thresholds": a["thresholds"],
                                "signers": [{"type": g["type"], "key": b(g["key"]), "weight": g.get("weight", 1),
                                             "payload": b(g.get("payload", ""))} for g in a["signers"]]}
    sigs = [{"hint": b(d["hint"]), "sig": b(d["sig"])} for d in case["sigs"]]

    def check_tx():
        r = {"code": 0, "inner_code": 0, "failed_op": -1, "op_code": 0}
        ck = Checker(protocol, b(case["hash"]), sigs, verify)
        src = accounts.get(b(case["source"]))
        if src is None:
            r["code"] = TX_NO_ACCOUNT
            return r
        if not ck.check(_signers_of(src), src["thresholds"][1]):
            r["code"] = TX_BAD_AUTH
            return r
        extra = [{"type": g["type"], "key": b(g["key"]), "weight": 1, "payload": b(g.get("payload", ""))}
                 for g in case.get("extra", [])]
        if protocol >= 19 and extra and not ck.check(extra, len(extra)):
            r["code"] = TX_BAD_AUTH
            return r
        if for_apply and protocol < 10:
            return r
        for i, op in enumerate(case["ops"]):
            oid = b(op["source"]) if op.get("source") else b(case["source"])
            acc = accounts.get(oid)
            if acc is not None:
                ok, opc = ck.check(_signers_of(acc), acc["thresholds"][op["level"]]), OP_BAD_AUTH
            elif not op.get("source"):
                ok, opc = False, OP_NO_ACCOUNT
            else:
                ok = ck.check([{"type": ED25519, "key": oid, "weight": 1, "payload": b""}], 0)
                opc = OP_BAD_AUTH
            if not ok and r["code"] != TX_FAILED:
                r.update(code=TX_FAILED, failed_op=i, op_code=opc)
                if not for_apply:
                    return r
        if r["code"] == TX_FAILED:
            return r
        if not ck.all_used():
            r["code"] = TX_BAD_AUTH_EXTRA
        return r

    fb = case.get("fee_bump")
    if not fb:
        return check_tx()
    r = {"code": 0, "inner_code": 0, "failed_op": -1, "op_code": 0}
    if protocol < 13:
        r["code"] = -12
        return r
    fee = accounts.get(b(fb["fee_source"]))
    if fee is None:
        r["code"] = TX_NO_ACCOUNT
        return r
    ck = Checker(protocol, b(fb["hash"]), [{"hint": b(d["hint"]), "sig": b(d["sig"])} for d in fb["sigs"]], verify)
    if not ck.check(_signers_of(fee), fee["thresholds"][1]):
        r["code"] = TX_BAD_AUTH
        return r
    if not ck.all_used():
        r["code"] = TX_BAD_AUTH_EXTRA
        return r
    inner = check_tx()
    r.update(code=1 if inner["code"] == 0 else -13, inner_code=inner["code"], failed_op=inner["failed_op"],
             op_code=inner["op_code"])
    return r
