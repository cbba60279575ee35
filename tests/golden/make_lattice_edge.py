#!/usr/bin/env python3
"""Generate tests/golden/lattice_edge.npz: rows aimed at the half-size
verification path (stellar-core_amd/csrc/lattice.h).

Runs ONLY in the build container (libsodium 1.0.18 through ctypes gives every
verdict, exactly as make_golden.py).  Classes:
  lat_bits131 / lat_bits131_bad   valid signatures whose reduced pair (c0, c1)
                                  has max bit length 131 = 4*33-1: the signed
                                  radix-16 top digit is +8 (carry case); and the
                                  same rows with one S bit flipped
  lat_w34                         pairs of >= 132 bits (34+ windows)
  lat_tb_even                     Euclid ends on an even t: the balanced
                                  (r_{i-1} - k r_i) vector is used
  torsion_AR_accept               mixed-order A = aB + T_A and R = rB + T_R with
                                  T_R = -[h] T_A: libsodium ACCEPTS (the
                                  torsion cancels); exercises the mod-8L
                                  lattice (a mod-L pair would get these wrong)
  torsion_AR_reject               same keys, T_R != -[h] T_A: rejected
The classification below restates the reduction in Python integers; it only
selects rows (the verdicts are libsodium's).

Usage:  make -C oracle && python tests/golden/make_lattice_edge.py
"""
import hashlib
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as G  # noqa: E402  (libsodium + curve helpers; no work at import)

L, N8 = G.L, 8 * G.L


def lattice(h):
    """(c0, c1, tb_even) as lattice.h computes them (exact-integer Euclid)."""
    a, ta, b, tb = N8, 0, h, 1
    while b >= 1 << 128:
        q = a // b
        a, ta, b, tb = b, tb, a - q * b, ta - q * tb
    if tb % 2:
        return b, tb, False
    k = max(0, (a - abs(ta)) // (b + abs(tb)))
    return a - k * b, ta - k * tb, True


def bits(c0, c1):
    return max(c0.bit_length(), abs(c1).bit_length())


def hram(sig, pk, m):
    return G.sha512_int(sig[:32], pk, m) % L


def main():
    rows = G.Rows()
    want = {"lat_bits131": 24, "lat_w34": 16, "lat_tb_even": 16}
    got = {k: 0 for k in want}
    i = 0
    while any(got[k] < want[k] for k in want) and i < 400000:
        seed = hashlib.sha256(b"LATSEED" + struct.pack("<Q", i)).digest()
        m = hashlib.sha256(b"LATMSG" + struct.pack("<Q", i)).digest()
        i += 1
        pk, sk = G.sod_keypair(seed)
        sig = G.sod_sign(m, sk)
        c0, c1, even = lattice(hram(sig, pk, m))
        nb = bits(c0, c1)
        cls = None
        if nb == 131 and got["lat_bits131"] < want["lat_bits131"]:
            cls = "lat_bits131"
        elif nb >= 132 and got["lat_w34"] < want["lat_w34"]:
            cls = "lat_w34"
        elif even and got["lat_tb_even"] < want["lat_tb_even"]:
            cls = "lat_tb_even"
        if cls is None:
            continue
        got[cls] += 1
        rows.add(cls, pk, sig, m, 1)
        if cls == "lat_bits131":
            bad = bytearray(sig)
            bad[32 + (i % 31)] ^= 1 << (i % 8)
            rows.add("lat_bits131_bad", pk, bytes(bad), m, 0)
    print("searched %d signatures: %s" % (i, got))

    T8 = G.pt_dec(G.BLACKLIST[2])
    torsion = [(0, 1)]
    for _ in range(7):
        torsion.append(G.pt_add(torsion[-1], T8))  # torsion[j] = [j] T8
    acc = rej = 0
    j = 0
    while acc < 48 or rej < 48:
        a = int.from_bytes(hashlib.sha256(b"TORA" + struct.pack("<Q", j)).digest(), "little") % L
        ta = 1 + j % 7                      # T_A = [ta] T8 (order 8, 4 or 2)
        Aenc = G.pt_enc(G.pt_add(G.pt_mul(a, G.B), torsion[ta]))
        m = hashlib.sha256(b"TORM" + struct.pack("<Q", j)).digest()
        r = G.sha512_int(b"TORR", struct.pack("<Q", j)) % L
        rB = G.pt_mul(r, G.B)
        j += 1
        for tr in range(8):                 # T_R = [tr] T8
            Renc = G.pt_enc(G.pt_add(rB, torsion[tr]))
            h = G.sha512_int(Renc, Aenc, m) % L
            S = (r + h * a) % L
            sig = Renc + S.to_bytes(32, "little")
            if (tr + h * ta) % 8 == 0:
                if acc < 48:
                    rows.add("torsion_AR_accept", Aenc, sig, m, 1)
                    acc += 1
            elif rej < 48 and tr != 0:
                rows.add("torsion_AR_reject", Aenc, sig, m, 0)
                rej += 1
    rows.save("lattice_edge.npz")


if __name__ == "__main__":
    main()
