#!/usr/bin/env python3
"""Generates stellar-core_amd/csrc/fe_asm_gen.h: each GF(2^255-19) product /
square of fe25519.h (radix 2^25.5, column-major, carry folded into the next
column's first mad) as ONE gfx950 inline-asm statement.

Why one statement: LLVM's gfx950 hazard recognizer assumes every inline-asm
statement may write a 16-bit dst-sel destination and pads the next
instruction with an s_nop whenever it reads what the statement wrote (one
wait state, 4 issue cycles); split into per-column statements a product paid
up to 10 of them.  Inside one statement the dependent chain issues back to
back (dependent v_mad_u64_u32 chains run at the independent rate:
profiles/r02/ubench_valu_rates_dep.txt).  Doublings use v_add_u32 x, x (full
rate) instead of shifts (half rate on gfx950).

Fixed scratch: the column accumulators alternate between v[0:1] and v[2:3]
(declared clobbered), so the low half of a column can be masked into the
output limb by a 32-bit v_and_b32.  The lowest VGPRs are allocatable in every
kernel; high ones are not (a kernel without launch bounds gets 128, and a
clobbered register outside the budget is only warned about, then written
anyway).  Carry-out SGPR pairs rotate over s[88:95] (never read).

    python tools/gen_fe_asm.py > stellar-core_amd/csrc/fe_asm_gen.h
"""
PAIRS = ["s[94:95]", "s[92:93]", "s[90:91]", "s[88:89]"]
ACC = [("v[0:1]", "v0", "v1"), ("v[2:3]", "v2", "v3")]
WIDTH = [26 if i % 2 == 0 else 25 for i in range(10)]
MASK = ["0x3ffffff" if w == 26 else "0x1ffffff" for w in WIDTH]
CLOB = ", ".join('"v%d"' % r for r in range(0, 4)) + ", " + ", ".join('"s%d"' % r for r in range(88, 96))


def product(name, terms_of_col, temps, inputs, doc, sig=None, sconst=()):
    """terms_of_col[k] = list of (a_operand, b_operand) names; temps = list of
    (name, instruction text producing it); sig: explicit parameter list."""
    lines = []
    for _, text in temps:
        lines.append(text)
    mad = 0
    for k in range(10):
        cur = ACC[k % 2]
        prev = ACC[(k - 1) % 2]
        for t, (a, b) in enumerate(terms_of_col[k]):
            if t == 0:
                addend = "0" if k == 0 else cur[0]
                if k > 0:
                    # carry of column k-1 (in prev) into cur, then mask prev's low half
                    lines.append("v_lshrrev_b64 %s, %d, %s" % (cur[0], WIDTH[k - 1], prev[0]))
                    lines.append("v_and_b32 %%[o%d], %s, %s" % (k - 1, MASK[k - 1], prev[1]))
            else:
                addend = cur[0]
            lines.append("v_mad_u64_u32 %s, %s, %%[%s], %%[%s], %s" % (cur[0], PAIRS[mad % 4], a, b, addend))
            mad += 1
    # close column 9: c9 = acc >> 25 (in the other pair), limb 9 masked
    cur, oth = ACC[9 % 2], ACC[0]
    lines.append("v_lshrrev_b64 %s, 25, %s" % (oth[0], cur[0]))
    lines.append("v_and_b32 %%[o9], %s, %s" % (MASK[9], cur[1]))
    # wrap: h0 = o0 + 19 c9 (c9 < 2^38: low word by a mad, high word by a
    # 24-bit mad), o0 = h0 mod 2^26, o1 += h0 >> 26 (< 2^18)
    lines.append("v_mov_b32 %s, %%[o0]" % cur[1])
    lines.append("v_mov_b32 %s, 0" % cur[2])
    lines.append("v_mad_u64_u32 %s, %s, %s, 19, %s" % (cur[0], PAIRS[mad % 4], oth[1], cur[0]))
    lines.append("v_mad_u32_u24 %s, %s, 19, %s" % (cur[2], oth[2], cur[2]))
    lines.append("v_and_b32 %%[o0], %s, %s" % (MASK[0], cur[1]))
    lines.append("v_alignbit_b32 %s, %s, %s, 26" % (oth[1], cur[2], cur[1]))
    lines.append("v_add_u32 %%[o1], %%[o1], %s" % oth[1])
    outs = ['[o%d] "=&v"(o[%d])' % (k, k) for k in range(10)] + ['[%s] "=&v"(%s)' % (n, n) for n, _ in temps]
    ins = ['[%s] "v"(%s)' % (n, e) for n, e in inputs] + ['[%s] "s"(%s)' % (n, e) for n, e in sconst]
    body = "\n".join('      "%s\\n"' % l for l in lines)
    out = []
    out.append("// %s" % doc)
    params = sig or ", ".join("const fe& " + v for v in sorted({e.split('.')[0] for _, e in inputs}))
    out.append("SV_HD void %s(fe& h, %s) {" % (name, params))
    out.append("  uint32_t o[10];")
    for n, _ in temps:
        out.append("  uint32_t %s;" % n)
    out.append("  asm(")
    out.append(body)
    out.append("      : " + ", ".join(outs))
    out.append("      : " + ", ".join(ins))
    out.append("      : %s);" % CLOB)
    out.append("  SV_UNROLL for (int i = 0; i < 10; ++i) h.v[i] = o[i];")
    out.append("}")
    return "\n".join(out)


def gen_mul(dbl, pre19=False):
    """pre19: the 19-multiples of g's limbs 1..9 come in as g19 (fe19), so a g
    shared by two products is pre-multiplied once (ge_p1p1_to_p3's T)."""
    inputs = [("f%d" % i, "f.v[%d]" % i) for i in range(10)] + [("g%d" % j, "g.v[%d]" % j) for j in range(10)]
    temps = []
    for j in range(1, 10):
        if pre19:
            inputs.append(("t19_%d" % j, "g19.v[%d]" % (j - 1)))
        else:
            temps.append(("t19_%d" % j, "v_mul_lo_u32 %%[t19_%d], %%[g%d], 19" % (j, j)))
    fa = {}
    fb = {}
    for i in range(10):
        if dbl:
            temps.append(("a2_%d" % i, "v_add_u32 %%[a2_%d], %%[f%d], %%[f%d]" % (i, i, i)))
            fa[i] = "a2_%d" % i
        else:
            fa[i] = "f%d" % i
    for i in range(1, 10, 2):
        temps.append(("b_%d" % i, "v_add_u32 %%[b_%d], %%[%s], %%[%s]" % (i, fa[i], fa[i])))
        fb[i] = "b_%d" % i
    cols = []
    for k in range(10):
        col = []
        for i in range(10):
            j = (k - i) % 10
            a = fb[i] if (i % 2 and j % 2) else fa[i]
            b = "t19_%d" % j if i + j >= 10 else "g%d" % j
            col.append((a, b))
        cols.append(col)
    name = ("fe_mul2_asm" if dbl else "fe_mul_asm") if not pre19 else "fe_mul_g19_asm"
    doc = "h = %sf g (fe_mul_cm<%s>)" % ("2 " if dbl else "", "true" if dbl else "false")
    if pre19:
        doc += ", g19 = 19 g[1..9] given"
        return product(name, cols, temps, inputs, doc, sig="const fe& f, const fe& g, const fe19& g19")
    return product(name, cols, temps, inputs, doc)


# Operand multiples a squaring derives (limb, multiplier), chosen by a small
# integer program (minimum count of v_add_u32 / v_lshlrev_b32 / v_mul_lo_u32
# such that every term f_i f_j (i <= j, factor 2 for i != j, 2 for odd * odd,
# 19 for a wrapped column, 2 for DBL) is one product of two available 32-bit
# operands within the input bound): 13 instead of 20 for fe_sq, 16 instead
# of 30 for fe_sq2.
SQ_DERIVED = {
    # fe_sq: inputs <= M3 (even limbs 3 2^26, odd 3 2^25, + slack)
    False: [(0, 2), (1, 2), (2, 2), (3, 2), (4, 2), (5, 2), (5, 38), (6, 19), (7, 2), (7, 38), (8, 2), (8, 19), (9, 38)],
    # fe_sq2: inputs <= R (the doubling's Z, a product output)
    True: [(0, 2), (0, 4), (1, 2), (1, 4), (2, 2), (3, 2), (3, 4), (4, 2), (5, 2), (5, 76), (6, 2), (6, 38), (7, 2),
           (7, 76), (8, 38), (9, 76)],
}
SQ_BOUND = {False: (3 * 2**26 + 2**12, 3 * 2**25 + 2**12), True: (2**26 + 2**11, 2**25 + 2**17)}


def limb_bound(i, bound):
    return bound[i % 2]


def gen_sq(dbl):
    inputs = [("f%d" % i, "f.v[%d]" % i) for i in range(10)]
    bound = SQ_BOUND[dbl]
    avail = {(i, 1): "f%d" % i for i in range(10)}
    sconst = []
    temps = []
    for (i, m) in SQ_DERIVED[dbl]:  # (listed in derivation order)
        assert m * limb_bound(i, bound) < 2**32, (i, m)
        n = "m%d_%d" % (m, i)
        if m % 2 == 0 and (i, m // 2) in avail:
            src = avail[(i, m // 2)]
            temps.append((n, "v_add_u32 %%[%s], %%[%s], %%[%s]" % (n, src, src)))
        elif m & (m - 1) == 0:
            temps.append((n, "v_lshlrev_b32 %%[%s], %d, %%[f%d]" % (n, m.bit_length() - 1, i)))
        elif m <= 64:  # (an inline constant)
            temps.append((n, "v_mul_lo_u32 %%[%s], %%[f%d], %d" % (n, i, m)))
        else:  # VOP3 takes no literal: the constant comes in an SGPR
            k = "k%d" % m
            if (k, "%du" % m) not in sconst:
                sconst.append((k, "%du" % m))
            temps.append((n, "v_mul_lo_u32 %%[%s], %%[f%d], %%[%s]" % (n, i, k)))
        avail[(i, m)] = n
    cols = [[] for _ in range(10)]
    for i in range(10):
        for j in range(i, 10):
            k = (i + j) % 10
            mult = (2 if i != j else 1) * (2 if (i % 2 and j % 2) else 1) * (19 if i + j >= 10 else 1) * (2 if dbl else 1)
            pick = None
            for (p, q) in ((i, j), (j, i)):
                for (pp, a), an in sorted(avail.items()):
                    if pp != p or mult % a:
                        continue
                    b = mult // a
                    if (q, b) in avail:
                        pick = (an, avail[(q, b)])
                        break
                if pick:
                    break
            assert pick, (i, j, mult)
            cols[k].append(pick)
    name = "fe_sq2_asm" if dbl else "fe_sq_asm"
    doc = "h = %sf^2 (fe_sq_cm<%s>)" % ("2 " if dbl else "", "true" if dbl else "false")
    return product(name, cols, temps, inputs, doc, sconst=sconst)


def main():
    print("// GENERATED by tools/gen_fe_asm.py -- do not edit.  Device-only field")
    print("// products as single inline-asm statements (see the generator's docstring);")
    print("// included by fe25519.h for device builds.  Same arithmetic and bounds as")
    print("// fe_mul_cm / fe_sq_cm there, which the host build and tests/ exercise.")
    print("#pragma once")
    print()
    for f in (gen_mul(False), gen_mul(True), gen_sq(False), gen_sq(True), gen_mul(False, pre19=True)):
        print(f)
        print()


if __name__ == "__main__":
    main()
