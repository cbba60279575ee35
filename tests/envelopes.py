"""Builders for the transaction-level C surface (include/stellar_host.h
svh_check_envelopes): numpy structured arrays laid out exactly like the C
structs, so large envelope sets (a catchup checkpoint) are built without a
Python loop per field."""
import ctypes

import numpy as np

SIGNER = np.dtype([("type", "u1"), ("key", "u1", 32), ("pad", "u1", 3), ("weight", "<u4"), ("payload_len", "<u4"),
                   ("payload", "u1", 64)])
DSIG = np.dtype([("hint", "u1", 4), ("sig_len", "<u4"), ("sig", "u1", 64)])
ACCOUNT = np.dtype([("account_id", "u1", 32), ("thresholds", "u1", 4), ("nsigners", "<u4"), ("signer_off", "<u4")])
OP = np.dtype([("has_source", "u1"), ("level", "u1"), ("source", "u1", 32), ("pad", "u1", 2)])
ENVELOPE = np.dtype([("contents_hash", "u1", 32), ("source", "u1", 32), ("nsigs", "<u4"), ("sig_off", "<u4"),
                     ("nops", "<u4"), ("op_off", "<u4"), ("nextra", "<u4"), ("extra_off", "<u4"),
                     ("fee_bump", "<u4"), ("fee_bump_hash", "u1", 32), ("fee_source", "u1", 32),
                     ("nouter", "<u4"), ("outer_off", "<u4")])
RESULT = np.dtype([("code", "<i4"), ("inner_code", "<i4"), ("failed_op", "<i4"), ("op_code", "<i4")])
assert SIGNER.itemsize == 108 and DSIG.itemsize == 72 and ACCOUNT.itemsize == 44
assert OP.itemsize == 36 and ENVELOPE.itemsize == 164 and RESULT.itemsize == 16


def _b(h):
    return np.frombuffer(bytes.fromhex(h), np.uint8)


class EnvelopeSet:
    """Accumulates accounts / envelopes into the flat arrays the C call takes."""

    def __init__(self):
        self.signers, self.sigs, self.ops, self.accounts, self.envs = [], [], [], [], []
        self.account_index = {}

    def _signer(self, s):
        r = np.zeros(1, SIGNER)[0]
        r["type"] = s.get("type", 0)
        r["key"] = _b(s["key"])
        r["weight"] = s.get("weight", 1)
        p = bytes.fromhex(s.get("payload", ""))
        r["payload_len"] = len(p)
        r["payload"][:len(p)] = np.frombuffer(p, np.uint8)
        self.signers.append(r)

    def _sig(self, d):
        r = np.zeros(1, DSIG)[0]
        r["hint"] = _b(d["hint"])
        s = bytes.fromhex(d["sig"])
        r["sig_len"] = len(s)
        r["sig"][:len(s)] = np.frombuffer(s, np.uint8)
        self.sigs.append(r)

    def account(self, a):
        if a["id"] in self.account_index:
            return
        r = np.zeros(1, ACCOUNT)[0]
        r["account_id"] = _b(a["id"])
        r["thresholds"] = a["thresholds"]
        r["signer_off"] = len(self.signers)
        r["nsigners"] = len(a["signers"])
        for s in a["signers"]:
            self._signer(s)
        self.account_index[a["id"]] = len(self.accounts)
        self.accounts.append(r)

    def envelope(self, source, chash, sigs, ops, extra=(), fee_bump=None):
        e = np.zeros(1, ENVELOPE)[0]
        e["contents_hash"] = _b(chash)
        e["source"] = _b(source)
        e["sig_off"], e["nsigs"] = len(self.sigs), len(sigs)
        for d in sigs:
            self._sig(d)
        e["op_off"], e["nops"] = len(self.ops), len(ops)
        for o in ops:
            r = np.zeros(1, OP)[0]
            r["level"] = o["level"]
            if o.get("source"):
                r["has_source"] = 1
                r["source"] = _b(o["source"])
            self.ops.append(r)
        e["extra_off"], e["nextra"] = len(self.signers), len(extra)
        for s in extra:
            self._signer(s)
        if fee_bump:
            e["fee_bump"] = 1
            e["fee_bump_hash"] = _b(fee_bump["hash"])
            e["fee_source"] = _b(fee_bump["fee_source"])
            e["outer_off"], e["nouter"] = len(self.sigs), len(fee_bump["sigs"])
            for d in fee_bump["sigs"]:
                self._sig(d)
        self.envs.append(e)

    def arrays(self):
        def arr(lst, dt):
            return np.array(lst, dt) if lst else np.zeros(1, dt)
        return (arr(self.envs, ENVELOPE), arr(self.sigs, DSIG), arr(self.ops, OP), arr(self.signers, SIGNER),
                arr(self.accounts, ACCOUNT))


def check_envelopes(host, envs, sigs, ops, signers, accounts, n, naccounts, protocol, prefetch=0, for_apply=0):
    res = np.zeros(max(1, n), RESULT)
    pairs = ctypes.c_uint64()
    vp = ctypes.c_void_p
    rc = host.svh_check_envelopes(vp(envs.ctypes.data), ctypes.c_size_t(n), vp(sigs.ctypes.data), vp(ops.ctypes.data),
                                  vp(signers.ctypes.data), vp(accounts.ctypes.data), ctypes.c_size_t(naccounts),
                                  ctypes.c_uint32(protocol), prefetch, for_apply, vp(res.ctypes.data),
                                  ctypes.byref(pairs))
    assert rc == 0, host.svh_last_error_string()
    return res[:n], pairs.value


def case_set(case):
    """One wrapper.json envelope case as its own EnvelopeSet."""
    es = EnvelopeSet()
    for a in case["accounts"]:
        es.account(a)
    es.envelope(case["source"], case["hash"], case["sigs"], case["ops"], extra=case.get("extra", ()),
                fee_bump=case.get("fee_bump"))
    return es
