"""Static ISA census of a gfx950 kernel: instruction classes per loop body.

usage: python tools/isa_loops.py <file.s> <kernel-substring>
  (file.s from: hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S csrc/sv_kernels.hip)

Prints, for the kernel, the whole-function class counts and, for every
backward branch (a loop), the class counts of the instructions between its
target label and the branch.  Developer tool; nothing in the product uses it.
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mad_u64_u32"):
        return "mad64"
    if "_dpp" in op or op.startswith("v_mov_b32_dpp"):
        return "dpp"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith(("v_lshrrev_b64", "v_lshlrev_b64", "v_lshl_add_u64", "v_add_u64", "v_ashrrev_i64")):
        return "v64"
    if op.startswith(("v_mul_lo", "v_mul_hi", "v_mul_u32", "v_mad_u32")):
        return "vmul32"
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu32"
    return "other"


def main():
    path, kname = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l)]
    k = [i for i in starts if kname in lines[i]]
    if not k:
        sys.exit("kernel not found")
    s = k[0]
    e = next((i for i in starts if i > s), len(lines))
    body = lines[s:e]
    ins = []
    labels = {}
    for l in body:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        m = re.match(r"^\s*([vsgdb][a-z_0-9]+)(\s+(.*))?$", l)
        if m and not l.strip().startswith(";"):
            ins.append((m.group(1), m.group(3) or ""))
    tot = Counter(classify(op) for op, _ in ins)
    print("kernel", lines[s].split(":")[0], "instructions", len(ins))
    print("  ", dict(sorted(tot.items(), key=lambda x: -x[1])))
    for idx, (op, args) in enumerate(ins):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = args.strip().split()[0] if args.strip() else ""
            if tgt in labels and labels[tgt] <= idx:
                seg = ins[labels[tgt]: idx + 1]
                c = Counter(classify(o) for o, _ in seg)
                print("loop %s [%d..%d] %d instr: %s" % (tgt, labels[tgt], idx, len(seg),
                                                        dict(sorted(c.items(), key=lambda x: -x[1]))))


if __name__ == "__main__":
    main()
