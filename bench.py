#!/usr/bin/env python3
"""Benchmark: consensus-ADMM CSC learner on MI355X (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W
  (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

Workload (BASELINE.json configs[1], "C2"): 2D dzParallel learning of K = 100
filters 11x11 on n = 10,000 synthetic contrast-normalised 100x100 patches,
ni = 100 patches per block (100 consensus blocks), sharded over the ranks.
One *step* = one outer ADMM iteration (D precompute + 5 d-iterations + Z
precompute + 10 z-iterations, tol = 0 so the inner counts are fixed; the
objective is not evaluated, matching the reference's tim_vals, dP:122 vs :127).

metric = outer iterations/s x patches of the whole node (strong scaling: the
10^4 patches are split over the N GPUs).  Inputs are resident in HBM before
the timed region.  One JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
ZKERNEL_PREFIX = "ccsc::k_z"   # the dominant kernel: one z-iteration over the local patches
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_zsplit.json")   # tools/pmc_summary.py --json


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_threads():
    """Threads the CPU baseline may use: the CPUs this process is allowed to run on,
    bounded by the job's declared CPU share (OMP_NUM_THREADS; the GPU box grants 16
    CPUs per GPU although nproc shows the whole machine)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    return min(avail, int(share)) if share.isdigit() and int(share) > 0 else avail


def cpu_baseline(args):
    """SURVEY.md §8(d) CPU baseline: the float64 NumPy/SciPy port of the learner with
    C1's constants (2D dParallel, rho_D = 500, 10 d-its, rho_Z = 50, threshold
    lambda / 50, 10 z-its; K = 100 11x11, 100x100 patches, ni = 100), median of 2 outer
    iterations (tol = 0, objective excluded), on ONE block of ni = 100 patches -- a C1
    outer iteration is 10 such blocks (per-block precompute, d-solves and z-steps; the
    consensus mean between them is 12,100 values), so C1 patch-iters/s = 10 ni /
    (10 t_block) = ni / t_block.  The reference MATLAB cannot run here."""
    from oracle.ccsc_port import DzPort
    from ccsc_code_iccv2017_amd import synth

    threads = cpu_threads()
    ni = 100
    b = synth.images_2d(ni, device="cpu", seed=2017 + 0)
    rng = np.random.default_rng(11)
    d0 = rng.standard_normal((11, 11, 100))
    z0 = rng.standard_normal((110, 110, 100, ni))
    port = DzPort(b, d0, z0, 1.0, ni=ni, rho_d=500.0, rho_z=50.0, theta_div=50.0, max_it_d=10,
                  max_it_z=10, workers=threads, replicate_z0=False)
    ts = []
    try:
        from threadpoolctl import threadpool_limits
        limit = threadpool_limits(limits=threads)   # BLAS / LAPACK threads
    except ImportError:
        import contextlib
        limit = contextlib.nullcontext()
    with limit:
        for _ in range(2):
            t0 = time.perf_counter()
            port.outer()
            ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))
    return {
        "value": ni / dt,
        "unit": "patch-iters/s",
        "cores": threads,
        "kind": "port",
        "nproc": os.cpu_count(),
        "cpu_model": cpu_model(),
        "sample": f"C1 (2D dParallel: rho_D=500, 10 d-its, rho_Z=50, lambda/50, 10 z-its; K=100 "
                  f"11x11, 100x100 synthetic local-CN patches) on ONE block of ni={ni} patches, "
                  f"median of 2 outer iterations ({', '.join(f'{t:.1f}' for t in ts)} s); a C1 "
                  f"outer iteration is 10 such blocks, so C1 patch-iters/s = ni / t_block; "
                  f"oracle/ccsc_port.py float64, scipy.fft + BLAS on {threads} threads "
                  f"(nproc {os.cpu_count()}), host CPU '{cpu_model()}'",
    }


ZLINE_WAVES_PER_PATCH = 12


def pmc_traffic(n_local):
    """HBM bytes per launch of the dominant z-step kernel from the committed rocprofv3
    PMC passes (FETCH_SIZE doubled for 16-B streaming loads on gfx950 and WRITE_SIZE,
    both kB per dispatch; MI355X_MICROARCH.md "HBM"), scaled to this run's patch count
    when the profile was taken at another n, plus the SQ pass of the same kernel (VALU /
    LDS activity, wave waits) that says what bounds it.  Returns (bytes, source, kernel,
    stale, sq): stale is True when the kernel sources changed since the summary was
    taken (tools/pmc_summary.py records their hash).  (None, ...) without a summary."""
    from tools.pmc_summary import source_hash
    try:
        d = json.load(open(PMC_SUMMARY))
    except (OSError, ValueError):
        return None, None, None, None, None
    cands = [(v.get("avg_s", 0) * v.get("dispatches", 0), name, v) for name, v in d.items()
             if name.startswith(ZKERNEL_PREFIX) and isinstance(v, dict)]
    if not cands:
        return None, None, None, None, None
    _, name, k = max(cands)
    stale = d.get("src_sha256") != source_hash()
    sq = sq_limits(k)
    if "FETCH_SIZE" not in k or "WRITE_SIZE" not in k:
        return None, os.path.relpath(PMC_SUMMARY, ROOT), name, stale, sq
    # patches per profiled dispatch: one 12-wave workgroup per patch (zline.hip), so a
    # two-stream z-phase's half launches (rocprofv3 serialises them under --pmc) count as
    # halves; without the SQ pass, the profile's whole patch count
    disp = k["SQ_WAVES"] / ZLINE_WAVES_PER_PATCH if k.get("SQ_WAVES") else d.get("n_local", n_local)
    per = (2.0 * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024.0 * n_local / disp
    return per, os.path.relpath(PMC_SUMMARY, ROOT), name, stale, sq


def sq_limits(k):
    """What bounds the kernel, from its SQ counters (per dispatch): SIMD-cycle shares of
    VALU and LDS issue, and the wave-lifetime shares spent parked (s_waitcnt /
    barrier) or issue-stalled.  SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* / SQ_WAIT_* count
    quad-cycles; the clock is GRBM_GUI_ACTIVE / 8 XCDs / kernel time
    (MI355X_MICROARCH.md, cycle constants and DVFS)."""
    need = ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_ANY",
            "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE")
    if any(c not in k for c in need) or not k.get("sq_avg_s"):
        return None
    t = k["sq_avg_s"]
    clk = k["GRBM_GUI_ACTIVE"] / 8.0 / t
    simd_cycles = t * clk * 1024.0            # 256 CUs x 4 SIMDs
    wc = k["SQ_WAVE_CYCLES"]
    return {
        "clock_GHz": clk / 1e9,
        "valu_busy": 4.0 * k["SQ_ACTIVE_INST_VALU"] / simd_cycles,
        "lds_busy": 4.0 * k["SQ_ACTIVE_INST_LDS"] / simd_cycles,
        "wave_parked": k["SQ_WAIT_ANY"] / wc,
        "wave_issue_stalled": k["SQ_WAIT_INST_ANY"] / wc,
        "valu_insts_per_wave": k.get("SQ_INSTS_VALU", float("nan")) / max(k.get("SQ_WAVES", 1), 1),
        # LDS bank-conflict cycles per LDS issue cycle, and the LDS share with them counted
        # (lds_busy counts issue only)
        "lds_conflict_per_issue": (k["SQ_LDS_BANK_CONFLICT"] / k["SQ_ACTIVE_INST_LDS"]
                                   if "SQ_LDS_BANK_CONFLICT" in k and k["SQ_ACTIVE_INST_LDS"] else None),
        "lds_busy_incl_conflicts": (4.0 * (k["SQ_ACTIVE_INST_LDS"] + k["SQ_LDS_BANK_CONFLICT"]) / simd_cycles
                                    if "SQ_LDS_BANK_CONFLICT" in k else None),
    }


def limiter(frac_dram, sq):
    """The measured bound: HBM when the DRAM traffic runs at >= 60% of peak, else the
    busiest issue pipe if it is busy >= 50% of the SIMD cycles, else latency (waves
    parked on memory / barriers)."""
    if frac_dram is not None and frac_dram >= 0.6:
        return "hbm"
    if sq is None:
        return "unmeasured"
    if max(sq["valu_busy"], sq["lds_busy"]) >= 0.5:
        return "valu" if sq["valu_busy"] >= sq["lds_busy"] else "lds"
    return "latency"


def step_alg_bytes(n, K, ni, P, F, mid, miz, s=8, V=1):
    """algorithmic bytes of one outer iteration (precompute + max_it_d
    d-iterations + max_it_z z-iterations), c = 2 s, N = n / ni blocks.  Its z-iteration
    counts every stage's operands through HBM (prox, R2C, solve, C2R), which the fused
    z-steps never move, so it is a staged model, not a floor."""
    c = 2 * s
    N = n // ni
    s_app = min(c * F * K * (K + 1) // 2, c * F * (ni * K + ni * (ni + 1) // 2))
    z_it = n * K * (4 * s * P + 4 * c * F) + n * c * F * V
    d_it = N * (4 * s * P * V * K + 5 * c * F * V * K + s_app)
    pre = N * (c * F * K * ni + c * F * V * ni + s_app + c * F * V * K)
    return pre + mid * d_it + miz * z_it


def step_compulsory_bytes(n, K, ni, P, F, mid, miz, woodbury, V=1, four_d=False, s=8):
    """Compulsory HBM bytes of one outer iteration of a consensus learner: every kernel
    class reads its inputs once and writes its outputs once, with the z-iteration fused
    (DESIGN.md §7):
      z-iteration  the state a = z + y read and written once per (patch, filter) slice
                   (2 s P), plus per patch the z-solve's own operands: w read + written and
                   B^ read (3 c F; the closed form of dP:278-303), or for 4D the view
                   correlation E per slice (c F, L4:310-347);
      precompute   per block the R2C of the state into Z^ (ni K (s P + c F)), the Gram's
                   reads of Z^ and B^ and its writes of the factor and h (dP:221-237);
      d-iteration  per block §8(d)'s stages (dual update + R2C, d-solve over the factor,
                   C2R): 4 s P V K + 5 c F V K + the factor.
    The factor is K(K+1)/2 packed per f (Cholesky) or ni K + ni(ni+1)/2 (Woodbury)."""
    c = 2 * s
    N = n // ni
    fac = c * F * (ni * K + ni * (ni + 1) // 2) if woodbury else c * F * (K * (K + 1) // 2)
    pre = N * (ni * K * (s * P + c * F) + c * F * K * ni + c * F * V * ni + fac + c * F * V * K)
    d_it = N * (4 * s * P * V * K + 5 * c * F * V * K + fac)
    z_it = n * K * 2 * s * P + (n * K * c * F if four_d else 3 * n * c * F)
    return pre + mid * d_it + miz * z_it


def hs23_compulsory_bytes(n, K, W, P, F, mid, miz, s=8):
    """Compulsory bytes of one outer iteration of the 2-3D learner (L23:86-226, C3): the
    precompute fft2(z) + Gram (L23:100, 289-295), then per inner iteration (each of the
    max_it_d D- and max_it_z Z-iterations, objective included: L23:132,195) the synthesis
    sum_k d^_k z^_k (reads z^ and d^), the masked data prox/dual on the W-channel side
    (its spectrum in, d{1} and M.*b read, d{1} written, xi1 out: 2 c F + 3 s P per
    channel), the variable's prox/dual (3 s P + c F per variable slice), the solve's
    right-hand side reads, its output spectrum and the C2R of the variable (c F + s P),
    and the objective's synthesis (z^, d^ again)."""
    c = 2 * s
    Kp = K * (K + 1) // 2
    pre = n * K * (s * P + c * F) + n * K * c * F + c * F * Kp
    synth = n * K * c * F + W * K * c * F
    data = n * W * (2 * c * F + 3 * s * P)
    d_it = (synth + data + W * K * (3 * s * P + c * F) + n * K * c * F + n * W * c * F
            + c * F * Kp + W * K * (2 * c * F + s * P) + synth)
    z_it = (synth + data + n * K * (3 * s * P + c * F) + n * W * c * F
            + n * K * (2 * c * F + s * P) + synth)
    return pre + mid * d_it + miz * z_it


# the other BASELINE.json configs (C2 is the headline workload above): name, variant, b
# shape, kernel size, lambda, synthetic data kind (SURVEY.md §8d sizes; C4/C5 take n = 64)
CONFIGS = [
    ("C1", "2D dParallel, K=100 11x11, n=1000 100x100 patches, 10 blocks", "DPAR",
     (100, 100, 1000), [11, 11, 100], 1.0, "normal"),
    ("C3", "2-3D hyperspectral (admm_learn), K=100 11x11x31, n=64 100x100x31 cubes", "HS23",
     (100, 100, 31, 64), [11, 11, 31, 100], 1.0, "uniform"),
    ("C4", "3D video, K=49 11x11x11, n=64 64x64x32 clips (ni=8, Woodbury)", "L3D",
     (64, 64, 32, 64), [11, 11, 11, 49], 0.1, "normal"),
    ("C5", "4D light field, K=49 11x11x5x5, n=64 64x64 5x5-view patches (ni=8)", "L4D",
     (64, 64, 5, 5, 64), [11, 11, 5, 5, 49], 1.0, "normal"),
]


def config_bytes(p, b_shape, ks):
    """(§8(d) bytes, compulsory bytes) of one outer iteration of a resolved problem."""
    from ccsc_code_iccv2017_amd import _lib as L
    r = ks[0] // 2
    X, Y = b_shape[0] + 2 * r, b_shape[1] + 2 * r
    Xh = X // 2 + 1
    n, K, mid, miz = p.n, p.K, p.max_it_d, p.max_it_z
    if p.variant == L.CCSC_HS23:
        W = b_shape[2]
        return None, hs23_compulsory_bytes(n, K, W, X * Y, Xh * Y, mid, miz)
    T = b_shape[2] + 2 * r if p.variant == L.CCSC_L3D else 1
    V = p.views[0] * p.views[1]
    P, F = X * Y * T, Xh * Y * T
    wb = p.dfactor == L.DFACTOR["woodbury"]
    return (step_alg_bytes(n, K, p.ni, P, F, mid, miz, V=V),
            step_compulsory_bytes(n, K, p.ni, P, F, mid, miz, wb, V=V,
                                  four_d=p.variant == L.CCSC_L4D))


def run_config(ctx, key, label, variant, b_shape, ks, lam, kind, steps=3):
    """One untimed warm-up outer iteration, then `steps` outer iterations timed one by one
    (objective excluded where the learner allows it; C3 evaluates it every inner
    iteration, as the reference's rollback test needs), each synchronised through the
    session's own sync; the figure is their median (not one iteration)."""
    from ccsc_code_iccv2017_amd import learners as E
    from ccsc_code_iccv2017_amd import _lib as L
    rng = np.random.default_rng(7)
    b = rng.random(b_shape) if kind == "uniform" else rng.standard_normal(b_shape)
    var = getattr(L, "CCSC_" + variant)
    p = E.make_problem(var, b_shape, ks, 1.0, lam, steps + 1, 0.0, "none", seed=11)
    sm = 0.5 * rng.random(b_shape) if variant == "HS23" else None
    s = E.Session(ctx, p, b, smooth_init=sm)
    try:
        s.step(1)
        ts = []
        for _ in range(steps):
            t0 = time.perf_counter()
            s.step(1)
            ts.append(time.perf_counter() - t0)
        dt = float(np.median(ts))
        q = s.p
    finally:
        s.close()
    n = b_shape[-1]
    s8d, comp = config_bytes(q, b_shape, ks)
    return {
        "workload": label,
        "s_per_outer_iteration": dt,
        "timed_iterations": [round(t, 6) for t in ts],
        "patch_iters_per_s": n / dt,
        # SURVEY §8(d)'s staged byte model counts every stage's operands through HBM
        # (spectra the fused kernels keep in registers / LDS): not a physical fraction, it
        # can exceed 1; kept only for continuity with the survey
        "staged_model_bytes": s8d,
        "staged_model_frac_nonphysical": s8d / dt / 1e9 / HBM_PEAK_GBS if s8d else None,
        "compulsory_bytes": comp,
        "frac_compulsory": comp / dt / 1e9 / HBM_PEAK_GBS,
        "max_it_d": q.max_it_d, "max_it_z": q.max_it_z, "ni": q.ni,
        "dfactor": "woodbury" if q.dfactor == L.DFACTOR["woodbury"] else "cholesky",
    }


def copy_rate(local, gib=2.0, reps=10):
    """Measured device-to-device streaming rate on this GPU (the achievable
    rate beside the 8 TB/s spec): tools/copy_probe.hip, a hand-written 16-B-per-lane copy
    (4 or 8 loads in flight per lane, 8 or 16 256-thread workgroups per CU or one pass, plain
    and nontemporal policy: the best form) over two `gib` GiB buffers -- read + write bytes /
    time by HIP events, median of `reps`.  (torch's copy_ measured 4.7 TB/s, 25% under the
    guide's 6.29 TB/s float4 copy, which flattered frac_of_copy: VERDICT r05.)"""
    import ctypes as C
    import torch
    lib_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "libcopy_probe.so")
    if not os.path.exists(lib_path):
        log(f"WARNING: {lib_path} missing (python -m ccsc_code_iccv2017_amd.build): no copy rate")
        return None, None
    lib = C.CDLL(lib_path)
    lib.copy_probe.restype = C.c_int
    lib.copy_probe.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.POINTER(C.c_double),
                               C.POINTER(C.c_int)]
    n = int(gib * 2**30) // 8
    src = torch.empty(n, dtype=torch.float64, device=f"cuda:{local}").normal_()
    dst = torch.empty_like(src)
    torch.cuda.synchronize()
    gbs, form = C.c_double(0), C.c_int(0)
    rc = lib.copy_probe(C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()), n * 8, reps,
                        C.byref(gbs), C.byref(form))
    torch.cuda.synchronize()
    del src, dst
    torch.cuda.empty_cache()
    if rc != 0:
        log(f"WARNING: copy probe failed ({rc})")
        return None, None
    f = form.value
    return gbs.value, (f"{'nontemporal' if f & 1 else 'plain'} policy, {8 if f & 2 else 4} loads "
                       f"in flight per lane, " +
                       ("one pass" if f & 8 else f"{16 if f & 4 else 8} workgroups per CU"))


def shard_diag(local, K, steps=2):
    """Per-rank diagnostic, NOT a scaling result: the 8-GPU job's rank-0 shard (13 of the 100
    consensus blocks = 1,300 patches, ccsc_shard) timed alone on this one GPU with no
    exchanges -- its step time and per-kernel split, so the z-step's tail at 5.08 rounds of
    workgroups per CU (1,300 / 256) shows before an 8-GPU run."""
    from ccsc_code_iccv2017_amd import learners as E
    from ccsc_code_iccv2017_amd import synth
    import torch
    ni, psf = 100, 11
    p8 = E.resolve(E.make_problem(E.L.CCSC_DZPAR, (100, 100, 10000), [psf, psf, K], 1.0, 1.0, 20,
                                  0.0, "none", ni=ni, seed=2017 + 1))
    b0, nb = E.shard(p8, 0, 8)
    n = nb * ni
    p = E.make_problem(E.L.CCSC_DZPAR, (100, 100, n), [psf, psf, K], 1.0, 1.0, 1 + steps, 0.0,
                       "none", ni=ni, seed=2017 + 1)
    b = synth.images_2d(n, first=b0 * ni, chunk=ni, device=f"cuda:{local}", seed=2017 + 1)
    torch.cuda.synchronize()
    with E.Context(local) as ctx:
        s = E.Session(ctx, p, b)
        del b
        s.step(1)
        s.set_profiling(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            s.step(1)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        ks = {}
        for kid, name in enumerate(["zstep", "gram_chol", "dsolve", "dual_r2c", "c2r_dout"]):
            n_, ms_, _ = s.kernel_stats(kid)
            if n_:
                ks[name] = {"launches_per_step": n_ / steps, "avg_ms": ms_ / n_}
        s.close()
    return {"what": "8-GPU rank-0 shard timed alone on one GPU (no exchanges): a per-rank "
                    "diagnostic, not a scaling result",
            "blocks": nb, "patches": n, "ms_per_step": dt * 1e3, "per_kernel": ks,
            "zstep_rounds_per_cu": n / 256}


def configs_leg(local):
    """Every other BASELINE.json config on this GPU (rank 0, N = 1): seconds per outer
    iteration, patch-iters/s and the step-level byte fractions."""
    from ccsc_code_iccv2017_amd import learners as E
    out = {}
    with E.Context(local) as ctx:
        for key, label, variant, shape, ks, lam, kind in CONFIGS:
            t0 = time.perf_counter()
            out[key] = run_config(ctx, key, label, variant, shape, ks, lam, kind)
            log(f"config {key}: {out[key]['s_per_outer_iteration']:.4f} s per outer iteration "
                f"({time.perf_counter() - t0:.1f} s with setup)")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=10000, help="patches (C2: 10^4)")
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--tol", type=float, default=0.0,
                    help="inner/outer tol (the reference driver's 1e-3, learn_kernels_2D_large.m:24;"
                         " the metric is defined at tol = 0: fixed inner counts)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-shard-diag", action="store_true",
                    help="skip the one-GPU timing of the 8-GPU rank-0 shard (13 blocks)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the C1/C3/C4/C5 timings (one warm-up + three timed outer iterations each)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)

    from ccsc_code_iccv2017_amd import learners as E
    from ccsc_code_iccv2017_amd import synth

    copy_gbs, copy_form = copy_rate(local)   # before the plan fills HBM
    uid = None
    if world > 1:
        obj = [E.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]

    ni, K, psf = 100, args.K, 11
    p = E.make_problem(E.L.CCSC_DZPAR, (100, 100, args.n), [psf, psf, K], 1.0, 1.0,
                       args.warmup + args.steps, args.tol, "none", ni=ni, seed=2017 + 1)
    p = E.resolve(p)
    b0, nb = E.shard(p, rank, world)
    n_local = nb * ni
    plan = E.plan_bytes(p, rank, world)
    t_gen = time.perf_counter()
    b = synth.images_2d(n_local, first=b0 * ni, chunk=ni, device=f"cuda:{local}", seed=2017 + 1)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    log(f"[rank {rank}] blocks {b0}..{b0 + nb - 1} ({n_local} patches), data {time.perf_counter() - t_gen:.1f}s,"
        f" device plan {plan / 2**30:.1f} GiB")

    ctx = E.Context(local, rank, world, uid)
    sess = E.Session(ctx, p, b)
    del b
    obj_start = sess.objective()        # sanity: the learner must decrease it (outside timing)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        sess.step(1)
    sess.set_profiling(True)
    barrier()
    torch.cuda.synchronize()
    outer0 = len(sess.iterlog()["tim_vals"]) - 1
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sess.step(1)   # tol > 0: a converged learner stops early (the reference's break, dP:186-188)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    # outer iterations the engine ran (< steps only when a tol > 0 learner converged)
    done_steps = len(sess.iterlog()["tim_vals"]) - 1 - outer0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    comm_ranks, transport = ctx.comm_ranks()
    launches, zms, _ = sess.kernel_stats(0)
    kstats = {}
    for kid, name in enumerate(["zstep", "gram_chol", "dsolve", "dual_r2c", "c2r_dout"]):
        n_, ms_, by_ = sess.kernel_stats(kid)
        if n_:
            kstats[name] = {"launches": n_, "avg_ms": ms_ / n_,
                            "alg_GBps": by_ / (ms_ / n_ * 1e-3) / 1e9}
    it = sess.iterlog()
    obj = sess.objective()
    if rank == 0:
        log(f"per-kernel (rank 0): {json.dumps(kstats)}")
        if args.tol > 0:
            tr = it["trace"]
            log(f"tol {args.tol}: inner counts d {tr['n_d'].tolist()} z {tr['n_z'].tolist()}")
        log(f"objective {obj_start:.6e} at start, {obj:.6e} after {sess.outer} outer iterations; "
            f"tim_vals {it['tim_vals']}")

    if rank == 0 and not (np.isfinite(obj) and obj < obj_start):
        log(f"WARNING: objective did not decrease: {obj_start:.6e} -> {obj:.6e}")
    avg_ms = zms / max(launches, 1)
    t_launch = avg_ms * 1e-3
    traffic, traffic_src, traffic_kernel, traffic_stale, sq = pmc_traffic(n_local)
    if traffic_stale:
        log(f"WARNING: {traffic_src} predates the current kernel sources (traffic is stale)")
    r = psf // 2
    Pg, Fg = (100 + 2 * r) ** 2, (100 + 2 * r) * ((100 + 2 * r) // 2 + 1)
    # algorithmic bytes of the fused z-step per launch: every byte it must
    # move once -- the state a read + written (2 s P per (patch, filter) slice) and, per
    # patch, w read + written and B^ read (3 c F); the filter spectra (K c F) are shared
    compulsory = n_local * (K * 2 * 8 * Pg + 3 * 16 * Fg)
    achieved = compulsory / t_launch / 1e9 if launches else 0.0
    frac_dram = traffic / t_launch / 1e9 / HBM_PEAK_GBS if (traffic and launches) else None
    step_comp = step_compulsory_bytes(args.n, K, ni, Pg, Fg, p.max_it_d, p.max_it_z, False)
    step_s = dt / max(done_steps, 1)
    result = {
        "objective_start": obj_start,
        "objective_end": obj,
        "metric": "ADMM outer iters/sec x patches (whole node)",
        "value": args.n * done_steps / dt,
        "unit": "patch-iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / max(done_steps, 1) * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded local-CN 100x100 patches; device-RNG init d0/z0)",
        "config": {
            "workload": "C2: 2D dzParallel, K=100 filters 11x11, n=10000 patches 100x100 "
                        "(grid 110x110), ni=100 -> 100 consensus blocks, max_it_d=5, "
                        f"max_it_z=10, tol={args.tol:g}, objective excluded",
            "tol": args.tol,
            "n": args.n, "K": K, "psf": psf, "ni": ni, "blocks": args.n // ni,
            "parallelism": f"consensus blocks sharded over {world} rank(s); RCCL all-reduce "
                           f"per d-iteration, broadcast per outer iteration",
        },
        # the communicator the engine actually exchanged over (ccsc_comm_ranks:
        # ncclCommCount for RCCL) -- not WORLD_SIZE
        "comm": {"transport": transport, "ranks": comm_ranks},
        "rccl_ranks": comm_ranks if transport == "rccl" else None,
        "roofline": {
            "bound": limiter(frac_dram, sq),
            "kernel": "z-step (C2R of the w term + prox/dual + R2C + per-bin reduction, one WG/patch)",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            # measured streaming copy on this GPU (read + write) and the kernel against it
            "copy_GBps": copy_gbs,
            "copy_kernel": f"tools/copy_probe.hip, 16 B per lane, {copy_form}",
            "frac_of_copy": achieved / copy_gbs if copy_gbs else None,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "traffic_kernel": traffic_kernel,
            "traffic_stale": traffic_stale,
            "alg_bytes_per_launch": compulsory,
            "avg_launch_ms": avg_ms,
            "frac_dram": frac_dram,
            "sq": sq,
            # whole outer iteration: every kernel class's compulsory bytes (its inputs read
            # once, its outputs written once; step_compulsory_bytes) / step time / node peak
            "step_compulsory_bytes": step_comp,
            "step_frac": step_comp / step_s / 1e9 / (HBM_PEAK_GBS * world),
        },
    }
    result["configs"] = None
    result["cpu_baseline"] = None
    result["shard8_diag"] = None
    if rank == 0 and world == 1:
        sess.close()
        ctx.close()
        if not args.no_shard_diag and args.n == 10000:
            sd = shard_diag(local, K)
            # the shard against 1/8 of this run's full step: > 1 = the per-rank work costs
            # more than its share (tails, fixed per-launch costs)
            sd["vs_eighth_of_full_step"] = sd["ms_per_step"] / (result["ms_per_step"] / 8)
            result["shard8_diag"] = sd
            log(f"shard8 diag: {json.dumps(sd)}")
        if not args.no_configs:
            result["configs"] = configs_leg(local)
        if not args.no_cpu_baseline:
            cb = cpu_baseline(args)
            if result["configs"]:   # the GPU on the same config (C1) beside the CPU number
                g1 = result["configs"]["C1"]["patch_iters_per_s"]
                cb["gpu_same_config"] = {"config": "C1", "value": g1, "unit": "patch-iters/s",
                                         "gpu_over_cpu": g1 / cb["value"]}
            result["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(result), flush=True)
    sess.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
