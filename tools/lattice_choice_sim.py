"""Could a better choice of the lattice pair put more signatures in 32 windows?

lattice.h stops the Euclid reduction of (8L, h) at the first remainder below
2^128 (with an odd-c1 fix-up); 32 windows hold scalars of <= 127 bits, so a
lane needs 32 windows for ~37 % of h (profiles/r06/windows/window_hist.txt).
This searches every a*v1 + b*v2 (|a|, |b| <= 4, c1 odd) around the
Lagrange-reduced basis for the pair with the fewest bits and prints both
distributions: the share at <= 127 bits only moves from ~37 % to ~41 %, as the
lattice volume predicts (det 8L ~ 2^255: the box |c0|, |c1| < 2^127 of area
2^256 holds one nonzero +-pair on average, half of them with c1 even).
Output: profiles/r06/windows/lattice_choice_sim.txt.  (Plain Python integers;
no engine code.)
"""
import random, collections
L = 2**252 + 27742317777372353535851937790883648493
N8 = 8*L
def current(h):
    a, ta, b, tb = N8, 0, h, 1
    while b >= 1 << 128:
        q = a // b
        a, ta, b, tb = b, tb, a - q * b, ta - q * tb
    if tb % 2:
        return b, tb
    k = max(0, (a - abs(ta)) // (b + abs(tb)))
    return a - k * b, ta - k * tb
def bits(v): return max(abs(v[0]).bit_length(), abs(v[1]).bit_length())
def reduced(h):
    # Lagrange-Gauss reduction of basis (N8, 0), (h, 1) in max-norm-ish (use euclidean)
    u = (N8, 0); v = (h, 1)
    def n2(x): return x[0]*x[0] + x[1]*x[1]
    if n2(u) < n2(v): u, v = v, u
    while True:
        # u longer; reduce u by v
        d = n2(v)
        m = (u[0]*v[0] + u[1]*v[1])
        q = (2*m + d) // (2*d)
        u = (u[0]-q*v[0], u[1]-q*v[1])
        if n2(u) >= n2(v):
            return v, u
        u, v = v, u
def best(h, R=4):
    v1, v2 = reduced(h)
    bestv = None
    for a in range(-R, R+1):
        for b in range(-R, R+1):
            if a == 0 and b == 0: continue
            c = (a*v1[0]+b*v2[0], a*v1[1]+b*v2[1])
            if c[1] % 2 == 0: continue
            if bestv is None or bits(c) < bits(bestv): bestv = c
    return bestv
random.seed(1)
cur = collections.Counter(); bst = collections.Counter()
N=20000
for _ in range(N):
    h = random.randrange(L)
    c = current(h); assert (c[0] - c[1]*h) % N8 == 0 and c[1] % 2
    cur[bits(c)] += 1
    b = best(h); assert (b[0] - b[1]*h) % N8 == 0 and b[1] % 2
    bst[bits(b)] += 1
for k in sorted(set(cur)|set(bst)):
    print(k, cur[k]/N, bst[k]/N)
print("<=127 current", sum(v for k,v in cur.items() if k<=127)/N, "best", sum(v for k,v in bst.items() if k<=127)/N)
