"""LDS bank-conflict model of the z-step's accesses (k_zline MODE 2, csrc/zline.hip), per the
gfx950 rules of MI355X_MICROARCH.md §LDS: ds_read_b128 in 4 lane groups of 16 (banks (a/4) mod 64),
ds_write_b128 in 8 groups of 8 contiguous lanes (banks (a/4) mod 32).  Prints, per access site,
the LDS-array cycles per wave-instruction summed over the site's registers and the 12 waves
(conflict-free: 4 per read, 8 per write).  Usage: python tools/lds_sim.py [RS] [old|new]
("old": the round-2 placement; "new": tcol/xoff/zoff of zline.hip)"""
import sys
from collections import defaultdict

RS = int(sys.argv[1]) if len(sys.argv) > 1 else 57
NEW = (sys.argv[2] if len(sys.argv) > 2 else "new") == "new"
WR = 10 * RS
TSZ = 110 * RS
RG = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
      [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
RG += [[l + 32 for l in g] for g in RG]
WG = [list(range(8 * i, 8 * i + 8)) for i in range(8)]


def cyc(addrs, write):
    """addrs: lane -> complex slot (16 B) or None; LDS-array cycles of one b128 instruction"""
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


def mod110(e):
    return e - 110 if e >= 110 else e


def zslot(x):
    return (x % 10) * 11 + x % 11


def tcol(c):
    return (c >> 1) + (c & 1) * 28 if NEW else c


def xoff(l):
    return 110 * l + ((0, 0, 11, 12, 16)[l] if NEW else 0)


def zoff(l):
    return 110 * l + (0, 6, 7, 8, 11)[l] if NEW else 114 * l


sites = defaultdict(lambda: [0, 0, 0])   # name -> [cycles, instrs, write]


def site(name, write, nreg, fn, waves=range(12)):
    for w in waves:
        for r in range(nreg):
            addrs = [fn(w, ln, r) for ln in range(64)]
            sites[name][0] += cyc(addrs, write)
            sites[name][1] += 1
            sites[name][2] = write


def run():
    X = range(11)
    ycol = lambda w, ln: tcol(roles(w, ln)[4])
    # P1: y-C2R, column c, E = sT + c, ES = RS
    site("P1 w-lds read", False, 10,
         lambda w, ln, k1: TSZ + k1 * 385 + roles(w, ln)[4] * 11 + roles(w, ln)[2], range(7))
    site("P1 dft10 -> E", True, 10, lambda w, ln, n1: ycol(w, ln) + (n1 * 11 + roles(w, ln)[2]) * RS)
    site("P1 E -> dft11", False, 11,
         lambda w, ln, k2: ycol(w, ln) + (min(roles(w, ln)[2], 9) * 11 + k2) * RS)
    site("P1 sink -> T", True, 11,
         lambda w, ln, n2: mod110(11 * min(roles(w, ln)[2], 9) + 10 * n2) * RS + ycol(w, ln))

    # P3: x-C2R of row pair j (x-waves)
    def p3r(w, ln, q):
        l, s, sb, sa, c, j = roles(w, ln)
        k1, hi_row = divmod(q, 2)
        xb = 110 - 10 * sb if sb else 0
        x = mod110(xb + 11 * k1)
        cc = 110 - x if x >= 56 else x
        return 2 * j * RS + hi_row * RS + tcol(cc)
    site("P3 T rows read", False, 20, p3r, X)
    ex = lambda w, l: WR * min(w, 10) + xoff(l)
    site("P3 dft10 -> E", True, 10, lambda w, ln, n1: ex(w, roles(w, ln)[0]) + n1 * 11 + roles(w, ln)[2], X)
    site("P3 E -> dft11", False, 11,
         lambda w, ln, k2: ex(w, roles(w, ln)[0]) + min(roles(w, ln)[2], 9) * 11 + k2, X)
    # P5: x-R2C
    site("P5 dft11 -> E", True, 11,
         lambda w, ln, k2: ex(w, roles(w, ln)[0]) + min(roles(w, ln)[2], 9) * 11 + k2, X)
    site("P5 E -> dft10", False, 10, lambda w, ln, n1: ex(w, roles(w, ln)[0]) + n1 * 11 + roles(w, ln)[2], X)
    site("P5 sink -> T", True, 10,
         lambda w, ln, k1: WR * min(w, 10) + zoff(roles(w, ln)[0]) + k1 * 11 + roles(w, ln)[2], X)

    # P7: two-for-one column loads
    def p7(w, ln, q):
        l, s, sb, sa, c, j = roles(w, ln)
        n2, which = divmod(q, 2)
        wv = (sa + n2) % 11   # pair (11 sa + 10 n2) mod 110 >> 1 = line sa >> 1 of wave wv
        z = zslot(c) if which == 0 else zslot(0 if c == 0 else 110 - c)
        return WR * wv + zoff(sa >> 1) + z
    site("P7 T cols read", False, 22, p7)
    # P9: y-R2C
    site("P9 dft11 -> E", True, 11,
         lambda w, ln, k2: ycol(w, ln) + (min(roles(w, ln)[2], 9) * 11 + k2) * RS)
    site("P9 E -> dft10", False, 10, lambda w, ln, n1: ycol(w, ln) + (n1 * 11 + roles(w, ln)[2]) * RS)


run()
tr = tw = 0
for k, (cy, n, wr) in sites.items():
    base = 8 if wr else 4
    print(f"{k:18s} {'W' if wr else 'R'} instr {n:4d} cycles {cy:6d}  per-instr {cy / n:5.2f} (free {base})")
    if wr:
        tw += cy
    else:
        tr += cy
print(f"RS={RS} {'new' if NEW else 'old'} read cycles {tr} write cycles {tw} per slice per WG")
