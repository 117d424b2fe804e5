"""Vectorised form of tools/lds_sim2.py (same accesses, same gfx950 bank rules) and a
simulated-annealing search over the region-major layout parameters of k_zline's transpose
buffer: A[m] (region block bases), PS (region stride per n2), TAU[a] / SIG[b] (separable slot
placement inside a region), XMAP (y-line exchange slot q -> region/side map) and REV (the
odd side of the y exchange walks the regions backwards).

Usage: python tools/lds_anneal.py check          (fast model == lds_sim2 on random layouts)
       python tools/lds_anneal.py anneal SEED ITERS
"""
import math
import random
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import lds_sim2 as S  # noqa: E402

LIMIT = S.LIMIT
RGA = np.array(S.RG)      # read groups (4 x 16 lanes)
WGA = np.array(S.WG)      # write groups (8 x 8 lanes)


def zsl(x):
    return divmod(S.zslot(x), 11)


def zo_ab(c):
    if c == 0:
        return (10, 0)
    if c == 55:
        return (10, 1)
    return zsl(110 - c)


def pair_region(j):
    return j % 5, (-2 * j) % 11


def xq_terms(c, q, xmap, rev):
    """(m, n2, a, b) of the y-line exchange slot q of column c"""
    n1, k2 = divmod(q, 11)
    if xmap == 0:
        m, side = (n1, 0) if n1 < 5 else (n1 - 5, 1)
    else:
        m, side = n1 >> 1, n1 & 1
    n2 = (10 - k2) if (rev and side) else k2
    a, b = zsl(c) if side == 0 else zo_ab(c)
    return m, n2, a, b


def y_terms(c, y):
    m, n2 = pair_region(y >> 1)
    a, b = zo_ab(c) if y & 1 else zsl(c)
    return m, n2, a, b


def build(xmap, rev):
    """per access site: (write?, terms[instr, lane, 4]); terms = -1 where no access"""
    sites = []

    def site(write, nreg, fn, waves=range(12)):
        rows = []
        for w in waves:
            for r in range(nreg):
                rows.append([fn(w, ln, r) for ln in range(64)])
        sites.append((write, np.array(rows, dtype=np.int64)))

    R = S.roles
    X = range(11)
    site(True, 10, lambda w, ln, n1: xq_terms(R(w, ln)[4], n1 * 11 + R(w, ln)[2], xmap, rev))
    site(False, 11, lambda w, ln, k2: xq_terms(R(w, ln)[4], R(w, ln)[3] * 11 + k2, xmap, rev))
    site(True, 11, lambda w, ln, n2: y_terms(R(w, ln)[4], S.elem_a(R(w, ln)[3], n2)))

    def p3(w, ln, q):
        l, s, sb, sa, c, j = R(w, ln)
        k1, which = divmod(q, 2)
        x = S.elem_b(sb, k1)
        m, n2 = pair_region(j)
        if which == 0:
            return (m, n2) + zsl(x)
        ab = (10, 0) if x == 0 else (10, 1) if x == 55 else zsl((110 - x) % 110)
        return (m, n2) + ab
    site(False, 20, p3, X)
    xr = lambda w, ln: pair_region(R(w, ln)[5])
    site(True, 10, lambda w, ln, n1: xr(w, ln) + (n1, R(w, ln)[2]), X)
    site(False, 11, lambda w, ln, k2: xr(w, ln) + (R(w, ln)[3], k2), X)
    site(True, 11, lambda w, ln, k2: xr(w, ln) + (R(w, ln)[3], k2), X)
    site(False, 10, lambda w, ln, n1: xr(w, ln) + (n1, R(w, ln)[2]), X)
    site(True, 10, lambda w, ln, k1: xr(w, ln) + (k1, R(w, ln)[2]), X)

    def p7(w, ln, q):
        l, s, sb, sa, c, j = R(w, ln)
        n2, which = divmod(q, 2)
        y = S.elem_a(sa, n2)
        return pair_region(y >> 1) + zsl(c if which == 0 else (110 - c) % 110)
    site(False, 22, p7)
    site(True, 11, lambda w, ln, k2: xq_terms(R(w, ln)[4], R(w, ln)[3] * 11 + k2, xmap, rev))
    site(False, 10, lambda w, ln, n1: xq_terms(R(w, ln)[4], n1 * 11 + R(w, ln)[2], xmap, rev))
    names = ["P1 dft10->E", "P1 E->dft11", "P1 sink->T", "P3 T read", "P3 dft10->E", "P3 E->dft11",
             "P5 dft11->E", "P5 E->dft10", "P5 sink->Z", "P7 T read", "P9 dft11->E", "P9 E->dft10"]
    return list(zip(names, sites))


_CACHE = {}


def tables(xmap, rev):
    key = (xmap, rev)
    if key not in _CACHE:
        _CACHE[key] = build(xmap, rev)
    return _CACHE[key]


def group_cycles(addr, groups, nb):
    """addr[instr, 64] -> sum over instrs and groups of the max bank multiplicity"""
    g = addr[:, groups]                          # [instr, ngroups, glen]
    g = np.sort(g, axis=2)
    uniq = np.ones(g.shape, dtype=bool)
    uniq[:, :, 1:] = g[:, :, 1:] != g[:, :, :-1]
    res = g % nb
    onehot = (res[..., None] == np.arange(nb)) & uniq[..., None]
    cnt = onehot.sum(axis=2)                     # [instr, ngroups, nb]
    return int(np.maximum(cnt.max(axis=2), 1).sum())


def evaluate(P, per_site=False):
    A = np.array(P["A"]); TAU = np.array(P["TAU"]); SIG = np.array(P["SIG"])
    tot = 0
    out = []
    for name, (write, t) in tables(P["XMAP"], P["REV"]):
        addr = A[t[..., 0]] + t[..., 1] * P["PS"] + TAU[t[..., 2]] + SIG[t[..., 3]]
        if write:
            cy = group_cycles(addr, WGA, 8) * 1   # 8-lane groups, 8 16-B chunks per row
            cy = cy  # 1 cycle per group pass -> 8 per conflict-free instr
        else:
            cy = group_cycles(addr, RGA, 16)
        out.append((name, write, t.shape[0], cy))
        tot += cy
    if per_site:
        for name, write, n, cy in out:
            base = 8 if write else 4
            print(f"{name:14s} {'W' if write else 'R'} instr {n:4d} cycles {cy:6d} per-instr {cy / n:5.2f} (free {base})")
        print("total", tot)
    return tot


def valid(P):
    A = np.array(P["A"]); TAU = np.array(P["TAU"]); SIG = np.array(P["SIG"])
    slots = [(a, b) for a in range(10) for b in range(11)] + [(10, 0), (10, 1)]
    ab = np.array([TAU[a] + SIG[b] for a, b in slots])
    regs = np.array([A[m] + n2 * P["PS"] for m in range(5) for n2 in range(11)])
    allv = (regs[:, None] + ab[None, :]).ravel()
    return allv.min() >= 0 and allv.max() < LIMIT and np.unique(allv).size == allv.size


def check():
    rnd = random.Random(3)
    for _ in range(3):
        PS = rnd.choice([113, 115])
        P = dict(PS=PS, A=[m * 11 * PS + rnd.randrange(0, 10) * (m > 0) for m in range(5)],
                 TAU=[a * 11 for a in range(11)], SIG=list(range(11)), XMAP=0, REV=rnd.random() < .5)
        P["TAU"][10] = 110 + rnd.randrange(0, 2)
        L = S.Layout(P["PS"], P["A"], P["TAU"], P["SIG"], P["REV"])
        ref = S.simulate(L)[0]
        fast = evaluate(P)
        print(ref, fast, "OK" if ref == fast else "MISMATCH")


def anneal(seed, iters):
    rnd = random.Random(seed)
    while True:
        PS = rnd.choice([113, 115, 117, 1, 3])
        if PS < 10:
            SG = rnd.choice([55, 57, 59])
            P = dict(PS=PS, A=[m * 11 * PS for m in range(5)], TAU=[a * 11 * SG for a in range(11)],
                     SIG=[b * SG for b in range(11)], XMAP=rnd.randrange(2), REV=False)
        else:
            P = dict(PS=PS, A=[m * 11 * PS for m in range(5)], TAU=[a * 11 for a in range(11)],
                     SIG=list(range(11)), XMAP=rnd.randrange(2), REV=False)
        if valid(P):
            break
    cur = evaluate(P)
    best, bestP = cur, P
    T0 = 400.0
    for it in range(iters):
        T = T0 * (1 - it / iters) + 1
        Q = {k: (list(v) if isinstance(v, list) else v) for k, v in P.items()}
        r = rnd.random()
        if r < 0.2:
            m = rnd.randrange(1, 5); Q["A"][m] += rnd.choice([-4, -3, -2, -1, 1, 2, 3, 4])
        elif r < 0.4:
            a = rnd.randrange(0, 11); Q["TAU"][a] += rnd.choice([-3, -2, -1, 1, 2, 3])
        elif r < 0.55:
            a = rnd.randrange(1, 11); d = rnd.choice([-2, -1, 1, 2])
            for t in range(a, 11): Q["TAU"][t] += d
        elif r < 0.7:
            b = rnd.randrange(0, 11); Q["SIG"][b] += rnd.choice([-3, -2, -1, 1, 2, 3])
        elif r < 0.8:
            b = rnd.randrange(1, 11); d = rnd.choice([-2, -1, 1, 2])
            for t in range(b, 11): Q["SIG"][t] += d
        elif r < 0.9:
            Q["PS"] += rnd.choice([-2, -1, 1, 2])
        elif r < 0.95:
            pass   # REV breaks the lane-base + compile-time form of the y exchange reads
        else:
            Q["XMAP"] = 1 - Q["XMAP"]
        if Q["PS"] < 1 or min(Q["TAU"]) < 0 or min(Q["SIG"]) < 0 or not valid(Q):
            continue
        v = evaluate(Q)
        if v <= cur or rnd.random() < math.exp((cur - v) / T):
            P, cur = Q, v
            if v < best:
                best, bestP = v, Q
                print(seed, it, best, bestP, flush=True)
    return best, bestP


if __name__ == "__main__":
    if sys.argv[1] == "check":
        check()
    elif sys.argv[1] == "anneal":
        b, P = anneal(int(sys.argv[2]), int(sys.argv[3]))
        print("FINAL", b, P)
