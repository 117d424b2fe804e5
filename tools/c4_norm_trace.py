#!/usr/bin/env python3
"""Engine per-filter norms of d_res = crop(D{1}) on a C4-shaped problem after 1, 2, 3, ...
outer iterations (each a fresh run from the same init, or from one perturbed at relative size
$C4_TRACE_EPS; the engine's norms to $C4_TRACE_JSON), beside the oracle's trace from
tools/norm_offset.py --json (its d1_norms_per_outer): where the two part, and how fast.
  python tools/c4_norm_trace.py <oracle.json> [iters ...] > gpurun_out/c4trace.txt   (GPU)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    g = json.load(open(sys.argv[1]))
    its = [int(x) for x in sys.argv[2:]] or list(range(1, len(g["d1_norms_per_outer"]) + 1))
    from ccsc_code_iccv2017_amd import learners as E
    from ccsc_code_iccv2017_amd import synth
    sb, K, n, psf = tuple(g["sb"]), g["K"], g["n"], g["psf"]
    b = synth.clips_3d(n, sb, K=K, psf=psf, device="cpu")
    r = psf // 2
    sp = [s + 2 * r for s in sb]
    dump = {}
    for it in its:
        rng = np.random.default_rng(44)
        init = {"d": rng.standard_normal((psf,) * 3 + (K,)), "z": rng.standard_normal(sp + [K, n])}
        eps = float(os.environ.get("C4_TRACE_EPS", "0"))
        if eps:   # sensitivity: the same run from an init perturbed at relative size eps
            init["d"] = init["d"] * (1 + eps * np.random.default_rng(7).standard_normal(init["d"].shape))
        d_e, *_ = E.admm_learn_conv3D_large(b, [psf] * 3 + [K], 1.0, 1.0, it, 0.0, "none", init)
        e = np.sqrt((d_e ** 2).sum(axis=(0, 1, 2)))
        o = np.array(g["d1_norms_per_outer"][it - 1]) if it <= len(g["d1_norms_per_outer"]) else None
        line = f"outer {it:2d}: engine {e.min():.9f} .. {e.max():.9f}"
        if o is not None:
            rel = np.abs(e - o) / o
            line += f"   oracle {o.min():.9f} .. {o.max():.9f}   max rel diff {rel.max():.3e}"
        print(line, flush=True)
        dump[it] = e.tolist()
    if os.environ.get("C4_TRACE_JSON"):
        json.dump(dump, open(os.environ["C4_TRACE_JSON"], "w"))


if __name__ == "__main__":
    main()
