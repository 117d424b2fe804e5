"""LDS bank-conflict model of the region-major transpose buffer of k_zline (csrc/zline.hip,
round 5), same gfx950 rules as tools/lds_sim.py (ds_read_b128: 4 lane groups of 16, banks
(a/4) mod 64; ds_write_b128: 8 groups of 8 contiguous lanes, banks (a/4) mod 32).

Layout: row pair j lives in region (m, n2) = (j mod 5, -2j mod 11) at complex offset
A[m] + n2*PS; inside a region, slot a*11 + b (a < 10, b < 11; plus the two odd-row
self-conjugate slots a = 10, b = 0/1) sits at TAU[a] + SIG[b].  Every access of the slice loop
is then a per-lane base plus a compile-time register offset (no per-element index math).

Usage: python tools/lds_sim2.py            (search a family of layouts, print the best)
       python tools/lds_sim2.py show PS TA SG A1 A2 A3 A4   (one layout, per-site table)
"""
import itertools
import random
import sys
from collections import defaultdict

RG = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
      [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
RG += [[l + 32 for l in g] for g in RG]
WG = [list(range(8 * i, 8 * i + 8)) for i in range(8)]


def cyc(addrs, write):
    groups, nb = (WG, 32) if write else (RG, 64)
    tot = 0
    for g in groups:
        banks = defaultdict(set)
        for ln in g:
            a = addrs[ln]
            if a is None:
                continue
            for d in range(4):
                banks[(4 * a + d) % nb].add(a)
        tot += max([len(v) for v in banks.values()] or [1])
    return tot


def roles(w, lane):
    l = min(lane // 11, 4)
    s = lane - 11 * l
    return l, s, min(s, 10), min(s, 9), min(5 * w + l, 55), min(5 * w + l, 54)


def zslot(x):
    return (x % 10) * 11 + x % 11


def elem_a(n1, n2):
    return (11 * n1 + 10 * n2) % 110


def elem_b(k2, k1):
    return (11 * k1 + 100 * k2) % 110


class Layout:
    def __init__(self, PS, A, TAU, SIG, REV=False):
        self.PS, self.A, self.TAU, self.SIG, self.REV = PS, A, TAU, SIG, REV

    def reg(self, m, n2):
        return self.A[m] + n2 * self.PS

    def region_of_pair(self, j):
        return self.reg(j % 5, (-2 * j) % 11)

    def sl(self, slot):
        a, b = divmod(slot, 11)
        return self.TAU[a] + self.SIG[b]

    def ze(self, c):
        return self.sl(zslot(c))

    def zo(self, c):   # odd row of column c in the y->x direction
        if c == 0:
            return self.sl(110)
        if c == 55:
            return self.sl(111)
        return self.sl(zslot(110 - c))

    def xq(self, c, q):   # y-line exchange slot q of column c
        n1, k2 = divmod(q, 11)
        if n1 < 5:
            return self.reg(n1, k2) + self.ze(c)
        return self.reg(n1 - 5, 10 - k2 if self.REV else k2) + self.zo(c)

    def yaddr(self, c, y):   # T element (row y, column c), y -> x direction
        j = y >> 1
        return self.region_of_pair(j) + (self.zo(c) if y & 1 else self.ze(c))

    def all_slots(self):
        out = []
        for j in range(55):
            base = self.region_of_pair(j)
            for s in range(112):
                out.append(base + self.sl(s))
        return out

    def valid(self, limit):
        s = self.all_slots()
        return len(set(s)) == len(s) and min(s) >= 0 and max(s) < limit


def simulate(L, per_site=False):
    sites = defaultdict(lambda: [0, 0, 0])

    def site(name, write, nreg, fn, waves=range(12)):
        for w in waves:
            for r in range(nreg):
                addrs = [fn(w, ln, r) for ln in range(64)]
                sites[name][0] += cyc(addrs, write)
                sites[name][1] += 1
                sites[name][2] = write

    X = range(11)
    R = lambda w, ln: roles(w, ln)
    # P1 (y-C2R of column c): DFT-10 outputs n1 -> exchange, DFT-11 inputs, sink rows
    site("P1 dft10 -> E", True, 10, lambda w, ln, n1: L.xq(R(w, ln)[4], n1 * 11 + R(w, ln)[2]))
    site("P1 E -> dft11", False, 11, lambda w, ln, k2: L.xq(R(w, ln)[4], R(w, ln)[3] * 11 + k2))
    site("P1 sink -> T", True, 11, lambda w, ln, n2: L.yaddr(R(w, ln)[4], elem_a(R(w, ln)[3], n2)))

    # P3 (x-C2R of row pair j): two reads per bin register, then its own exchange
    def p3(w, ln, q):
        l, s, sb, sa, c, j = R(w, ln)
        k1, which = divmod(q, 2)
        x = elem_b(sb, k1)
        base = L.region_of_pair(j)
        if which == 0:
            return base + L.sl(zslot(x))
        sl = 110 if x == 0 else 111 if x == 55 else zslot((110 - x) % 110)
        return base + L.sl(sl)
    site("P3 T read", False, 20, p3, X)
    xr = lambda w, ln: L.region_of_pair(R(w, ln)[5])
    site("P3 dft10 -> E", True, 10, lambda w, ln, n1: xr(w, ln) + L.sl(n1 * 11 + R(w, ln)[2]), X)
    site("P3 E -> dft11", False, 11, lambda w, ln, k2: xr(w, ln) + L.sl(R(w, ln)[3] * 11 + k2), X)
    site("P5 dft11 -> E", True, 11, lambda w, ln, k2: xr(w, ln) + L.sl(R(w, ln)[3] * 11 + k2), X)
    site("P5 E -> dft10", False, 10, lambda w, ln, n1: xr(w, ln) + L.sl(n1 * 11 + R(w, ln)[2]), X)
    site("P5 sink -> T", True, 10, lambda w, ln, k1: xr(w, ln) + L.sl(k1 * 11 + R(w, ln)[2]), X)

    # P7: column c of pair y >> 1 (Z_j(c), Z_j(110 - c))
    def p7(w, ln, q):
        l, s, sb, sa, c, j = R(w, ln)
        n2, which = divmod(q, 2)
        y = elem_a(sa, n2)
        base = L.region_of_pair(y >> 1)
        return base + L.sl(zslot(c if which == 0 else (110 - c) % 110))
    site("P7 T read", False, 22, p7)
    site("P9 dft11 -> E", True, 11, lambda w, ln, k2: L.xq(R(w, ln)[4], R(w, ln)[3] * 11 + k2))
    site("P9 E -> dft10", False, 10, lambda w, ln, n1: L.xq(R(w, ln)[4], n1 * 11 + R(w, ln)[2]))

    tr = sum(v[0] for v in sites.values() if not v[2])
    tw = sum(v[0] for v in sites.values() if v[2])
    if per_site:
        for k, (cy, n, wr) in sites.items():
            base = 8 if wr else 4
            print(f"{k:16s} {'W' if wr else 'R'} instr {n:4d} cycles {cy:6d}  per-instr {cy / n:5.2f} (free {base})")
        print(f"read cycles {tr} write cycles {tw} total {tr + tw} per slice per WG")
    return tr + tw, tr, tw


LIMIT = (163840 - 61600) // 16   # complex slots left beside the resident w


def family(PS, TA, SG, A):
    TAU = [a * TA for a in range(11)]
    SIG = [b * SG for b in range(11)]
    return Layout(PS, A, TAU, SIG)


def search(trials=400, seed=1):
    rnd = random.Random(seed)
    best = None
    cands = []
    # region-contiguous: slot stride 1, TA in {11, 12}, PS in [112, 116], A = m*11*PS + pads
    for PS in range(112, 117):
        for TA in (11, 12):
            if TA * 10 + 2 > PS:
                continue
            for _ in range(trials // 10):
                pads = [0] + sorted(rnd.sample(range(0, LIMIT - 55 * PS + 1), 4)) if LIMIT - 55 * PS >= 4 else [0] * 5
                A = [m * 11 * PS + pads[m] for m in range(5)]
                cands.append((PS, TA, 1, A))
    # slot-major: regions interleaved (PS = 1, A[m] = m*11 + pad), slot stride SG >= 55
    for SG in range(55, 58):
        for TA in (11 * SG, 11 * SG + 1, 11 * SG + 2, 11 * SG + 3):
            for _ in range(trials // 20):
                A = [0] + [m * 11 + rnd.randrange(0, 3) for m in range(1, 5)]
                cands.append((1, TA, SG, A))
    seen = set()
    for PS, TA, SG, A in cands:
        key = (PS, TA, SG, tuple(A))
        if key in seen:
            continue
        seen.add(key)
        L = family(PS, TA, SG, A)
        if not L.valid(LIMIT):
            continue
        tot, tr, tw = simulate(L)
        if best is None or tot < best[0]:
            best = (tot, tr, tw, key)
            print(f"total {tot} (r {tr} w {tw}) PS {PS} TA {TA} SG {SG} A {A}", flush=True)
    return best


def climb(seed, iters=1500):
    rnd = random.Random(seed)
    PS = rnd.choice([113, 115, 117, 119, 121, 1])
    if PS == 1:
        SG = rnd.choice([55, 56, 57])
        P = dict(PS=1, A=[m * 11 for m in range(5)], TAU=[a * 11 * SG for a in range(11)],
                 SIG=[b * SG for b in range(11)], REV=rnd.random() < 0.5)
    else:
        P = dict(PS=PS, A=[m * 11 * PS for m in range(5)], TAU=[a * 11 for a in range(11)],
                 SIG=list(range(11)), REV=rnd.random() < 0.5)
    mk = lambda P: Layout(P["PS"], P["A"], P["TAU"], P["SIG"], P["REV"])
    cur = simulate(mk(P))[0] if mk(P).valid(LIMIT) else 10 ** 9
    for it in range(iters):
        Q = {k: (list(v) if isinstance(v, list) else v) for k, v in P.items()}
        r = rnd.random()
        if r < 0.25:
            m = rnd.randrange(1, 5); Q["A"][m] += rnd.choice([-3, -2, -1, 1, 2, 3])
        elif r < 0.5:
            a = rnd.randrange(1, 11); d = rnd.choice([-2, -1, 1, 2])
            for t in range(a, 11): Q["TAU"][t] += d
        elif r < 0.75:
            b = rnd.randrange(1, 11); d = rnd.choice([-2, -1, 1, 2])
            for t in range(b, 11): Q["SIG"][t] += d
        elif r < 0.9:
            Q["PS"] += rnd.choice([-2, -1, 1, 2])
        else:
            Q["REV"] = not Q["REV"]
        L = mk(Q)
        if Q["PS"] < 1 or not L.valid(LIMIT):
            continue
        v = simulate(L)[0]
        if v <= cur:
            if v < cur:
                print(seed, it, v, Q, flush=True)
            cur, P = v, Q
    return cur, P


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "climb":
    import multiprocessing as mp
    with mp.Pool(8) as pool:
        res = pool.starmap(climb, [(s, int(sys.argv[2])) for s in range(8)])
    for v, P in sorted(res, key=lambda t: t[0]):
        print("FINAL", v, P)
    sys.exit(0)

if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "show":
        PS, TA, SG = map(int, sys.argv[2:5])
        A = [0] + list(map(int, sys.argv[5:9]))
        L = family(PS, TA, SG, A)
        print("valid", L.valid(LIMIT))
        simulate(L, per_site=True)
    else:
        search(int(sys.argv[1]) if len(sys.argv) > 1 else 400)
