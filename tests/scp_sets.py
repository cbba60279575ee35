"""SCP-shaped verification sets for the latency-path GPU tests: 100
validator keys (oracle-signed), 0..400-byte messages, ~30 % of rows mutated
(an R bit, an S bit or the message), verdicts from the oracle."""
import ctypes

import numpy as np

from conftest import oracle_verdicts


def scp_set(oracle, n, seed):
    rng = np.random.default_rng(seed)
    keys = []
    for v in range(100):
        seedb = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        pkb, skb = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
        oracle.oracle_ed25519_seed_keypair(pkb, skb, seedb)
        keys.append((pkb.raw, skb.raw))
    pk = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    msgs, lens = [], []
    for i in range(n):
        pkb, skb = keys[int(rng.integers(0, 100))]
        m = rng.integers(0, 256, int(rng.integers(0, 401)), dtype=np.uint8).tobytes()
        sb = ctypes.create_string_buffer(64)
        oracle.oracle_ed25519_sign(sb, m, len(m), skb)
        s = bytearray(sb.raw)
        kind = int(rng.integers(0, 10))
        if kind == 0:
            s[int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))  # R bit
        elif kind == 1:
            s[32 + int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))  # S bit
        elif kind == 2 and m:
            m = bytes([m[0] ^ 1]) + m[1:]
        pk[i] = np.frombuffer(pkb, np.uint8)
        sig[i] = np.frombuffer(bytes(s), np.uint8)
        msgs.append(m)
        lens.append(len(m))
    ln = np.array(lens, np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(msgs), np.uint8) if sum(lens) else np.zeros(1, np.uint8)
    d = {"pk": pk, "sig": sig, "msg": buf, "msg_off": off, "msg_len": ln}
    d["verdict"] = oracle_verdicts(oracle, d, rows=range(n))
    return d
