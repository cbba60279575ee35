#!/usr/bin/env python3
"""Developer tool: resolve compile-time switches whose value is fixed, in place.

    python tools/unifdef.py -DSV_X=1 -USV_Y file...

Every #if / #ifdef / #ifndef / #elif / #else / #endif group whose condition is
decided by the given macros (-D name=value: defined with that value; -U name:
undefined) is resolved: the taken branch is kept without its directives, the
others are dropped.  A condition that still depends on other macros is kept,
simplified when that is exact (e.g. `defined(__HIP_DEVICE_COMPILE__) && SV_X`
with SV_X = 1 becomes `defined(__HIP_DEVICE_COMPILE__)`): the truth table over
the remaining macros (each 0 or 1) must equal the simplified form's.  A
condition mixing a fixed macro with a macro that is not a 0/1 switch is left
untouched and reported.  Used to remove the retired alternates from the
product kernels; the code objects before and after must be identical
(tools/codeobj_digest.sh)."""
import itertools
import re
import sys

DIRECTIVE = re.compile(r"^(\s*)#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$")
IDENT = re.compile(r"[A-Za-z_][A-Za-z_0-9]*")


def strip_comment(s):
    s = re.sub(r"/\*.*?\*/", " ", s)
    return s.split("//")[0].strip()


class Expr:
    """A preprocessor condition evaluated with fixed and free macros."""

    def __init__(self, text, known):
        self.text = text
        self.known = known
        t = strip_comment(text)
        t = re.sub(r"defined\s*\(\s*([A-Za-z_]\w*)\s*\)", r"__DEF__(\1)", t)
        t = re.sub(r"defined\s+([A-Za-z_]\w*)", r"__DEF__(\1)", t)
        self.free = sorted({m for m in IDENT.findall(t) if m not in known and m not in ("__DEF__",)})
        py = t.replace("&&", " and ").replace("||", " or ")
        py = re.sub(r"!(?!=)", " not ", py)
        py = re.sub(r"__DEF__\((\w+)\)", r"__DEF__('\1')", py)
        self.py = re.sub(r"(?<!')\b([A-Za-z_]\w*)\b(?!')", lambda m: m.group(1) if m.group(1) in (
            "and", "or", "not", "__DEF__") else "__VAL__('%s')" % m.group(1), py)

    def value(self, free_vals):
        def dfn(m):
            if m in self.known:
                return self.known[m] is not None
            return bool(free_vals[m])

        def val(m):
            if m in self.known:
                v = self.known[m]
                return 0 if v is None else v
            return free_vals[m]
        return bool(eval(self.py, {"__DEF__": dfn, "__VAL__": val}))

    def table(self):
        return [self.value(dict(zip(self.free, bits))) for bits in itertools.product((0, 1), repeat=len(self.free))]

    def decided(self):
        """True / False when the fixed macros decide it, else None."""
        t = self.table()
        if all(t):
            return True
        if not any(t):
            return False
        return None

    def simplified(self):
        """An equivalent condition over the free macros only, or None."""
        if not any(m in strip_comment(self.text) for m in self.known):
            return self.text.strip()
        t = self.table()
        uses_defined = {m: bool(re.search(r"defined\s*\(?\s*%s\b" % m, self.text)) for m in self.free}
        lits = []
        for m in self.free:
            pos = "defined(%s)" % m if uses_defined[m] else m
            lits += [pos, "!" + pos]
        cands = list(lits)
        for a, b in itertools.combinations(lits, 2):
            cands += ["%s && %s" % (a, b), "%s || %s" % (a, b)]
        for c in cands:
            e = Expr(c, {})
            e.free = self.free
            if e.table() == t:
                return c
        return None


def parse(lines):
    """Nested list: plain lines (str) and groups [(kind, cond, indent, body), ...]."""
    root, stack = [], []
    cur = root
    for ln in lines:
        m = DIRECTIVE.match(ln)
        if not m:
            cur.append(ln)
            continue
        ind, kind, rest = m.group(1), m.group(2), m.group(3)
        if kind in ("if", "ifdef", "ifndef"):
            if kind == "ifdef":
                cond = "defined(%s)" % strip_comment(rest)
            elif kind == "ifndef":
                cond = "!defined(%s)" % strip_comment(rest)
            else:
                cond = rest.strip()
            grp = {"branches": [[cond, ind, [], ln]]}
            cur.append(grp)
            stack.append((cur, grp))
            cur = grp["branches"][-1][2]
        elif kind in ("elif", "else"):
            parent, grp = stack[-1]
            grp["branches"].append([rest.strip() if kind == "elif" else None, ind, [], ln])
            cur = grp["branches"][-1][2]
        else:  # endif
            parent, grp = stack.pop()
            grp["endif"] = ln
            cur = parent
    assert not stack, "unbalanced conditionals"
    return root


def emit(nodes, known, out, report):
    for nd in nodes:
        if isinstance(nd, str):
            out.append(nd)
            continue
        kept = []  # (cond or None for #else, indent, body, original line)
        for cond, ind, body, orig in nd["branches"]:
            if cond is None:
                kept.append((None, ind, body, orig))
                break
            e = Expr(cond, known)
            d = e.decided()
            if d is False:
                continue
            if d is True:
                kept.append((None, ind, body, orig))
                break
            if not any(re.search(r"\b%s\b" % re.escape(m), strip_comment(cond)) for m in known):
                kept.append((orig, ind, body, orig))  # (no fixed macro in it: the line as it was)
                continue
            s = e.simplified()
            if s is None:
                report.append("kept unsimplified: " + orig.strip())
                s = cond
            kept.append((s, ind, body, orig))
        if not kept:
            continue
        if kept[0][0] is None:  # decided: the branch's lines without directives
            emit(kept[0][2], known, out, report)
            continue
        for k, (cond, ind, body, orig) in enumerate(kept):
            directive = DIRECTIVE.match(orig).group(2)
            if cond is None:
                out.append(orig if directive == "else" else "%s#else" % ind)
            elif cond == orig:  # untouched line; an #elif that now opens the group becomes #if
                if k == 0 and directive == "elif":
                    out.append("%s#if %s" % (ind, orig_cond(orig)))
                else:
                    out.append(orig)
            else:
                out.append("%s#%s %s" % (ind, "if" if k == 0 else "elif", cond))
            emit(body, known, out, report)
        out.append(nd["endif"])


def orig_cond(line):
    m = DIRECTIVE.match(line)
    return m.group(3).strip() if m and m.group(2) in ("if", "elif") else None


def main():
    known, files = {}, []
    for a in sys.argv[1:]:
        if a.startswith("-D"):
            k, _, v = a[2:].partition("=")
            known[k] = int(v, 0) if v else 1
        elif a.startswith("-U"):
            known[a[2:]] = None
        else:
            files.append(a)
    for f in files:
        lines = open(f).read().split("\n")
        out, report = [], []
        emit(parse(lines), known, out, report)
        open(f, "w").write("\n".join(out))
        for r in report:
            print("%s: %s" % (f, r))


if __name__ == "__main__":
    main()
