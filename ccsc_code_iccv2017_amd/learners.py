"""Python mirror of the reference learners' interface over the libccsc C-ABI.

Same names, argument order, argument meaning and return tuples as the MATLAB
functions they replace (what a MEX wrapper would expose):

  d_res, z_res, DZ, iterations = admm_learn_conv2D_large_dParallel(
      b, kernel_size, lambda_residual, lambda_prior, max_it, tol, verbose, init)
                                   # 2D/admm_learn_conv2D_large_dParallel.m:1-4
  d_res, z_res, DZ, iterations = admm_learn_conv2D_large_dzParallel(...)
                                   # 2D/admm_learn_conv2D_large_dzParallel.m:1-4
  d_res, z_res, DZ, obj_val, iterations = admm_learn_conv3D_large(...)      # 3D/...:1-4
  d_res, z_res, DZ, obj_val, iterations = admm_learn_conv4D_lightfield(...) # 4D/...:1-4
  d_res, z_res, Dz, obj_val = admm_learn(b, kernel_size, lambda_residual, lambda_prior,
      max_it, tol, verbose, init, smooth_init)   # 2-3D/DictionaryLearning/admm_learn.m:1-4

Arrays carry the MATLAB shapes (b: [x, y, n]; kernel_size = [psf, psf, K];
d_res: [psf, psf, K]; z_res: [X, Y, K, n]; DZ: [X, Y, 1, n]) and are exchanged
column-major, so a Fortran-ordered NumPy array is bit-for-bit an mxArray.

``init`` (ignored by the reference, Q11) is honoured: ``{'d': [psf,psf,K],
'z': size_z}`` (dZ: ``size_z_crop`` = [X, Y, K, ni], replicated per block).
With ``init=None`` the engine draws d0/z0 on the device from ``seed``.

Errors are raised as ``CCSCError`` (the MATLAB reference raises on bad shapes
too; ``n % ni != 0`` is an error here rather than a silent floor, Q13).
"""
from __future__ import annotations

import ctypes as C
import os
import math

import numpy as np

from . import _lib as L


class Context:
    """One GPU (one rank).  ``uid`` (128 bytes from ``unique_id()`` on rank 0)
    is needed when ``nranks > 1``; the consensus then runs over RCCL.

    ``host_comm(op, array) -> None`` instead selects the host-staged transport
    (op 0: in-place sum all-reduce, op 1: in-place broadcast from rank 0), e.g.
    torch.distributed over gloo: used by the multi-rank GPU tests, which share
    one GPU between ranks."""

    def __init__(self, device: int = 0, rank: int = 0, nranks: int = 1, uid: bytes | None = None,
                 host_comm=None):
        self._lib = L.lib()
        eb = L.errbuf()
        if host_comm is not None:
            def _fn(user, op, buf, count):
                try:
                    arr = np.ctypeslib.as_array(buf, shape=(count,))
                    host_comm(op, arr)
                    return 0
                except Exception:  # noqa: BLE001 -- reported to the engine as a status
                    return 1
            self._cfn = L.COMM_FN(_fn)   # keep the trampoline alive
            self.ptr = self._lib.ccsc_create_hostcomm(device, rank, nranks, self._cfn, None, eb,
                                                      len(eb))
        else:
            self.ptr = self._lib.ccsc_create(device, rank, nranks, uid, eb, len(eb))
        if not self.ptr:
            raise L.CCSCError(L.CCSC_E_HIP, eb.value.decode(errors="replace"))
        self.device, self.rank, self.nranks = device, rank, nranks

    @classmethod
    def multi(cls, devices):
        """Single-process multi-device context (ccsc_create_multi): the learners then take
        the WHOLE problem and run rank i on devices[i] in its own host thread -- the
        drop-in path of one MATLAB call over a node's GPUs.  A repeated device ({0, 0})
        exchanges through host memory (one-GPU testing); distinct devices use RCCL."""
        self = cls.__new__(cls)
        self._lib = L.lib()
        eb = L.errbuf()
        devs = (C.c_int32 * len(devices))(*devices)
        self.ptr = self._lib.ccsc_create_multi(devs, len(devices), eb, len(eb))
        if not self.ptr:
            raise L.CCSCError(L.CCSC_E_HIP, eb.value.decode(errors="replace"))
        self.device, self.rank, self.nranks = devices[0], 0, 1
        self.devices = list(devices)
        # ccsc_create_multi builds a rank group for several devices, and for one under the
        # test hook CCSC_TEST_RCCL_SELF=1 (a 1-rank RCCL communicator); such a context
        # serves ccsc_learn only, not sessions
        selftest = os.environ.get("CCSC_TEST_RCCL_SELF", "0").strip()
        self._group = len(devices) > 1 or (selftest.isdigit() and int(selftest) != 0)
        return self

    @property
    def group(self):
        return getattr(self, "_group", False)

    def comm_ranks(self):
        """(ranks, transport) of the context's communicator (ccsc_comm_ranks): RCCL
        reports ncclCommCount, "host" the host-staged transport, "none" one rank."""
        eb = L.errbuf()
        n, t = C.c_int32(0), C.c_int32(0)
        L.check(self._lib.ccsc_comm_ranks(self.ptr, C.byref(n), C.byref(t), eb, len(eb)), eb)
        return n.value, L.TRANSPORT[t.value]

    def close(self):
        if self.ptr:
            self._lib.ccsc_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def unique_id() -> bytes:
    eb = L.errbuf()
    buf = C.create_string_buffer(128)
    L.check(L.lib().ccsc_get_unique_id(buf, eb, len(eb)), eb)
    return buf.raw


_VARIANT_FOR = {
    "dParallel": L.CCSC_DPAR,
    "dzParallel": L.CCSC_DZPAR,
}


def make_problem(variant, b_shape, kernel_size, lambda_residual, lambda_prior, max_it, tol,
                 verbose, *, ni=None, max_it_d=None, max_it_z=None, rho_d=None, rho_z=None,
                 theta_div=None, trace_objective=False, seed=0, precision="fp64",
                 dfactor="auto"):
    p = L.Problem()
    p.variant = variant
    p.ndim = 3 if variant == L.CCSC_L3D else 2
    p.sb[0], p.sb[1] = int(b_shape[0]), int(b_shape[1])
    if variant == L.CCSC_L3D:
        p.sb[2] = int(b_shape[2])
    p.views[0] = p.views[1] = 1
    if variant == L.CCSC_L4D and len(kernel_size) == 5:   # b: [x, y, U, V, n]; kernel [s, s, U, V, K]
        p.views[0], p.views[1] = int(kernel_size[2]), int(kernel_size[3])
    if variant == L.CCSC_HS23:                            # b: [x, y, W, n]; kernel [s, s, W, K]
        p.views[0] = int(kernel_size[2])
    p.n = int(b_shape[-1])
    p.K = int(kernel_size[-1])
    p.psf = int(kernel_size[0])
    p.lambda_residual = float(lambda_residual)
    p.lambda_prior = float(lambda_prior)
    p.max_it = int(max_it)
    p.tol = float(tol)
    if verbose not in L.VERBOSE:
        raise ValueError(f"verbose must be one of {sorted(L.VERBOSE)}")
    p.verbose = L.VERBOSE[verbose]
    p.ni = int(ni or 0)
    p.max_it_d = int(max_it_d or 0)
    p.max_it_z = int(max_it_z or 0)
    p.rho_d = float(rho_d or 0)
    p.rho_z = float(rho_z or 0)
    p.theta_div = float(theta_div or 0)
    if precision != "fp64":
        raise ValueError("precision must be 'fp64' (the reference computes in double)")
    p.precision = L.CCSC_FP64
    p.trace_objective = 1 if trace_objective else 0
    p.seed = int(seed)
    if dfactor not in L.DFACTOR:
        raise ValueError(f"dfactor must be one of {sorted(L.DFACTOR)}")
    p.dfactor = L.DFACTOR[dfactor]
    return p


def resolve(p: L.Problem) -> L.Problem:
    """Fill the variant defaults and validate; host only."""
    q = L.Problem.from_buffer_copy(p)
    eb = L.errbuf()
    L.check(L.lib().ccsc_resolve(C.byref(q), eb, len(eb)), eb)
    return q


def shard(p: L.Problem, rank: int, nranks: int):
    eb = L.errbuf()
    b0, nb = C.c_int64(), C.c_int64()
    L.check(L.lib().ccsc_shard(C.byref(p), rank, nranks, C.byref(b0), C.byref(nb), eb, len(eb)), eb)
    return b0.value, nb.value


def plan_bytes(p: L.Problem, rank: int = 0, nranks: int = 1) -> int:
    eb = L.errbuf()
    out = C.c_uint64()
    L.check(L.lib().ccsc_plan_bytes(C.byref(p), rank, nranks, C.byref(out), eb, len(eb)), eb)
    return out.value


def _f64(a):
    return None if a is None else np.asfortranarray(np.asarray(a, dtype=np.float64))


class Session:
    """Stateful learner (warm restart, bench): create -> step(k) -> results.
    The 2-3D learner (variant CCSC_HS23) also takes ``smooth_init``."""

    def __init__(self, ctx: Context, p: L.Problem, b, d0=None, z0=None, smooth_init=None):
        self.ctx = ctx
        self.p = resolve(p)
        eb = L.errbuf()
        L.check(L.lib().ccsc_supported(C.byref(self.p), eb, len(eb)), eb)   # CCSC_E_UNSUPPORTED
        self._b = _f64(b)
        self._d0 = _f64(d0)
        self._z0 = _f64(z0)
        eb = L.errbuf()
        if self.p.variant == L.CCSC_HS23:
            if smooth_init is None:
                raise ValueError("the 2-3D learner needs smooth_init (admm_learn.m:4)")
            self._sm = _f64(smooth_init)
            if self._sm.shape != self._b.shape:
                raise ValueError("smooth_init must have the shape of b")
            self.ptr = L.lib().ccsc_session_create_hs23(
                ctx.ptr, C.byref(self.p), L.dptr(self._b), L.dptr(self._sm), L.dptr(self._d0),
                L.dptr(self._z0), eb, len(eb))
        else:
            self.ptr = L.lib().ccsc_session_create(ctx.ptr, C.byref(self.p), L.dptr(self._b),
                                                   L.dptr(self._d0), L.dptr(self._z0), eb,
                                                   len(eb))
        if not self.ptr:
            raise L.CCSCError(L.CCSC_E_INVALID, eb.value.decode(errors="replace"))
        b0, nb = shard(self.p, ctx.rank, ctx.nranks)
        self.block_begin, self.nblocks = b0, nb
        # (the 2-3D learner's shards are runs of images: ccsc_shard counts images for it)
        self.n_local = nb if self.p.variant == L.CCSC_HS23 else nb * self.p.ni
        self.outer = 0

    def step(self, n_outer: int = 1) -> bool:
        eb = L.errbuf()
        done = C.c_int32(0)
        L.check(L.lib().ccsc_session_step(self.ptr, n_outer, C.byref(done), eb, len(eb)), eb)
        self.outer += n_outer
        return bool(done.value)

    def objective(self) -> float:
        eb = L.errbuf()
        v = C.c_double()
        L.check(L.lib().ccsc_session_objective(self.ptr, C.byref(v), eb, len(eb)), eb)
        return v.value

    def set_profiling(self, on: bool):
        L.check(L.lib().ccsc_session_set_profiling(self.ptr, 1 if on else 0), L.errbuf())

    def kernel_stats(self, kernel_id: int):
        eb = L.errbuf()
        n = C.c_int64()
        ms = C.c_double()
        by = C.c_double()
        L.check(L.lib().ccsc_session_kernel_stats(self.ptr, kernel_id, C.byref(n), C.byref(ms),
                                                  C.byref(by), eb, len(eb)), eb)
        return n.value, ms.value, by.value

    def grid(self):
        r = self.p.psf // 2
        g = (self.p.sb[0] + 2 * r, self.p.sb[1] + 2 * r)
        if self.p.variant == L.CCSC_L3D:
            g += (self.p.sb[2] + 2 * r,)
        return g

    def results(self, want_z=True, want_DZ=True, want_obj=False):
        p = self.p
        if p.variant == L.CCSC_L3D:
            X, Y, T = self.grid()
            d_res = np.zeros((p.psf, p.psf, p.psf, p.K), order="F")
            z_res = np.zeros((X, Y, T, p.K, self.n_local), order="F") if want_z else None
            DZ = np.zeros((X, Y, T, self.n_local), order="F") if want_DZ else None
            obj = np.zeros(1) if want_obj else None
            out = L.Outputs(L.dptr(d_res), L.dptr(z_res), L.dptr(DZ), L.dptr(obj))
            eb = L.errbuf()
            L.check(L.lib().ccsc_session_results(self.ptr, C.byref(out), eb, len(eb)), eb)
            return d_res, z_res, DZ, (float(obj[0]) if want_obj else None)
        X, Y = self.grid()
        if p.variant == L.CCSC_HS23:
            W = p.views[0]
            d_res = np.zeros((p.psf, p.psf, W, p.K), order="F")
            z_res = np.zeros((X, Y, p.K, self.n_local), order="F") if want_z else None
            DZ = np.zeros((X, Y, W, self.n_local), order="F") if want_DZ else None
        elif p.variant == L.CCSC_L4D:
            U, V = p.views[0], p.views[1]
            d_res = np.zeros((p.psf, p.psf, U, V, p.K), order="F")
            z_res = np.zeros((X, Y, 1, 1, p.K, self.n_local), order="F") if want_z else None
            DZ = (np.zeros((p.sb[0], p.sb[1], U, V, self.n_local), order="F")
                  if want_DZ else None)
        else:
            d_res = np.zeros((p.psf, p.psf, p.K), order="F")
            z_res = np.zeros((X, Y, p.K, self.n_local), order="F") if want_z else None
            DZ = np.zeros((X, Y, 1, self.n_local), order="F") if want_DZ else None
        obj = np.zeros(1) if want_obj else None
        out = L.Outputs(L.dptr(d_res), L.dptr(z_res), L.dptr(DZ), L.dptr(obj))
        eb = L.errbuf()
        L.check(L.lib().ccsc_session_results(self.ptr, C.byref(out), eb, len(eb)), eb)
        return d_res, z_res, DZ, (float(obj[0]) if want_obj else None)

    def iterlog(self, capacity=None):
        p = self.p
        cap = capacity or (self.outer + 1)
        a = {k: np.full(cap, np.nan) for k in ("obj_vals_d", "obj_vals_z", "tim_vals")}
        tr = {
            "obj_d": np.full(cap * p.max_it_d, np.nan),
            "obj_z": np.full(cap * p.max_it_z, np.nan),
            "d_diff": np.full(cap * p.max_it_d, np.nan),
            "z_diff": np.full(cap * p.max_it_z, np.nan),
        }
        nd = np.zeros(cap, dtype=np.int32)
        nz = np.zeros(cap, dtype=np.int32)
        fl = np.zeros(cap, dtype=np.int32)
        lg = L.IterLog(cap, 0, L.dptr(a["obj_vals_d"]), L.dptr(a["obj_vals_z"]),
                       L.dptr(a["tim_vals"]), L.dptr(tr["obj_d"]), L.dptr(tr["obj_z"]),
                       L.dptr(tr["d_diff"]), L.dptr(tr["z_diff"]), L.iptr(nd), L.iptr(nz),
                       L.iptr(fl))
        eb = L.errbuf()
        L.check(L.lib().ccsc_session_iterlog(self.ptr, C.byref(lg), eb, len(eb)), eb)
        cnt = lg.count
        it = {k: v[:cnt].copy() for k, v in a.items()}
        nout = max(cnt - 1, 0)
        it["trace"] = {
            "obj_d": tr["obj_d"][: nout * p.max_it_d].reshape(nout, p.max_it_d),
            "obj_z": tr["obj_z"][: nout * p.max_it_z].reshape(nout, p.max_it_z),
            "d_diff": tr["d_diff"][: nout * p.max_it_d].reshape(nout, p.max_it_d),
            "z_diff": tr["z_diff"][: nout * p.max_it_z].reshape(nout, p.max_it_z),
            "n_d": nd[:nout].copy(),
            "n_z": nz[:nout].copy(),
            "flags": fl[:nout].copy(),
        }
        return it

    def close(self):
        if self.ptr:
            L.lib().ccsc_session_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _learn_2d(variant, b, kernel_size, lambda_residual, lambda_prior, max_it, tol, verbose, init,
              ctx=None, device=0, want_z=True, want_DZ=True, **kw):
    b = np.asarray(b, dtype=np.float64)
    if b.ndim == 2:
        b = b[:, :, None]
    if b.ndim != 3:
        raise ValueError("b must be [x, y, n]")
    own = ctx is None
    if own:
        ctx = Context(device)
    try:
        p = make_problem(variant, b.shape, kernel_size, lambda_residual, lambda_prior, max_it, tol,
                         verbose, **kw)
        d0 = z0 = None
        if init is not None and len(init) > 0:
            d0 = init.get("d")
            z0 = init.get("z")
        if ctx.group:
            return learn_once(ctx, p, b, d0, z0, want_z=want_z, want_DZ=want_DZ)
        s = Session(ctx, p, b, d0, z0)
        try:
            done = False
            while s.outer < s.p.max_it and not done:
                done = s.step(1)
            d_res, z_res, DZ, _ = s.results(want_z=want_z, want_DZ=want_DZ)
            iterations = s.iterlog()
        finally:
            s.close()
    finally:
        if own:
            ctx.close()
    return d_res, z_res, DZ, iterations


def learn_once(ctx, p, b, d0=None, z0=None, want_z=True, want_DZ=True):
    """One ccsc_learn call over the whole problem (the MEX path): on a multi-device
    context the engine shards it over the devices.  2D learners; returns
    (d_res, z_res, DZ, iterations) like the session path."""
    p = resolve(p)
    psf, K = p.psf, p.K
    r = psf // 2
    X, Y = p.sb[0] + 2 * r, p.sb[1] + 2 * r
    b = np.asfortranarray(b, dtype=np.float64)
    d0 = None if d0 is None else np.asfortranarray(d0, dtype=np.float64)
    z0 = None if z0 is None else np.asfortranarray(z0, dtype=np.float64)
    d_res = np.zeros((psf, psf, K), order="F")
    z_res = np.zeros((X, Y, K, p.n), order="F") if want_z else None
    DZ = np.zeros((X, Y, 1, p.n), order="F") if want_DZ else None
    out = L.Outputs(L.dptr(d_res), L.dptr(z_res), L.dptr(DZ), L.dptr(None))
    cap = p.max_it + 1
    a = {k: np.full(cap, np.nan) for k in ("obj_vals_d", "obj_vals_z", "tim_vals")}
    tr = {"d_diff": np.full(cap * p.max_it_d, np.nan), "z_diff": np.full(cap * p.max_it_z, np.nan)}
    nd = np.zeros(cap, dtype=np.int32)
    nz = np.zeros(cap, dtype=np.int32)
    lg = L.IterLog(cap, 0, L.dptr(a["obj_vals_d"]), L.dptr(a["obj_vals_z"]),
                   L.dptr(a["tim_vals"]), L.dptr(None), L.dptr(None), L.dptr(tr["d_diff"]),
                   L.dptr(tr["z_diff"]), L.iptr(nd), L.iptr(nz), L.iptr(None))
    eb = L.errbuf()
    L.check(L.lib().ccsc_learn(ctx.ptr, C.byref(p), L.dptr(b), L.dptr(d0), L.dptr(z0),
                               C.byref(out), C.byref(lg), L.CB(), None, eb, len(eb)), eb)
    cnt = lg.count
    it = {k: v[:cnt].copy() for k, v in a.items()}
    nout = max(cnt - 1, 0)
    it["trace"] = {"d_diff": tr["d_diff"][: nout * p.max_it_d].reshape(nout, p.max_it_d),
                   "z_diff": tr["z_diff"][: nout * p.max_it_z].reshape(nout, p.max_it_z),
                   "n_d": nd[:nout].copy(), "n_z": nz[:nout].copy()}
    return d_res, z_res, DZ, it


def admm_learn_conv2D_large_dParallel(b, kernel_size, lambda_residual, lambda_prior, max_it, tol,
                                      verbose, init=None, **kw):
    """Drop-in for 2D/admm_learn_conv2D_large_dParallel.m:1-199."""
    return _learn_2d(L.CCSC_DPAR, b, kernel_size, lambda_residual, lambda_prior, max_it, tol,
                     verbose, init, **kw)


def admm_learn_conv2D_large_dzParallel(b, kernel_size, lambda_residual, lambda_prior, max_it, tol,
                                       verbose, init=None, **kw):
    """Drop-in for 2D/admm_learn_conv2D_large_dzParallel.m:1-206."""
    return _learn_2d(L.CCSC_DZPAR, b, kernel_size, lambda_residual, lambda_prior, max_it, tol,
                     verbose, init, **kw)


def admm_learn_conv4D_lightfield(b, kernel_size, lambda_residual, lambda_prior, max_it, tol,
                                 verbose, init=None, ctx=None, device=0, want_z=True,
                                 want_DZ=True, **kw):
    """Drop-in for 4D/admm_learn_conv4D_lightfield.m:1-212.

    b: [x, y, U, V, n] (single in the reference driver, Q15: widened to double);
    kernel_size = [psf, psf, U, V, K].  Returns (d_res [psf,psf,U,V,K],
    z_res [X,Y,1,1,K,n] complex (real part computed, Q8), DZ [x,y,U,V,n],
    obj_val, iterations) -- iterations carries empty fields like the reference
    (L4:64-72) plus the engine's 'trace'.
    """
    b = np.asarray(b, dtype=np.float64)
    if b.ndim == 4:
        b = b[..., None]
    if b.ndim != 5:
        raise ValueError("b must be [x, y, U, V, n]")
    own = ctx is None
    if own:
        ctx = Context(device)
    try:
        p = make_problem(L.CCSC_L4D, b.shape, kernel_size, lambda_residual, lambda_prior,
                         max_it, tol, verbose, **kw)
        d0 = z0 = None
        if init is not None and len(init) > 0:
            d0 = init.get("d")
            z0 = init.get("z")
            if z0 is not None:
                z0 = np.real(np.asarray(z0))
        s = Session(ctx, p, b, d0, z0)
        try:
            done = False
            while s.outer < s.p.max_it and not done:
                done = s.step(1)
            d_res, z_res, DZ, obj = s.results(want_z=want_z, want_DZ=want_DZ, want_obj=True)
            log = s.iterlog()
        finally:
            s.close()
    finally:
        if own:
            ctx.close()
    iterations = {"obj_vals_d": [], "obj_vals_z": [], "tim_vals": [], "it_vals": [],
                  "trace": log["trace"], "engine_tim_vals": log["tim_vals"]}
    if z_res is not None:
        z_res = z_res.astype(np.complex128)
    return d_res, z_res, DZ, obj, iterations


def admm_learn_conv3D_large(b, kernel_size, lambda_residual, lambda_prior, max_it, tol, verbose,
                            init=None, ctx=None, device=0, want_z=True, want_DZ=True, **kw):
    """Drop-in for 3D/admm_learn_conv3D_large.m:1-230 (function admm_learn_convND_large).

    b: [x, y, t, n]; kernel_size = [psf, psf, psf, K].  Returns (d_res [psf,psf,psf,K],
    z_res [X,Y,T,K,n], DZ [X,Y,T,n] (uncropped, L3:218-224), obj_val, iterations) --
    iterations carries the reference's empty fields (L3:72-75) plus the engine's 'trace'.
    """
    b = np.asarray(b, dtype=np.float64)
    if b.ndim == 3:
        b = b[..., None]
    if b.ndim != 4:
        raise ValueError("b must be [x, y, t, n]")
    own = ctx is None
    if own:
        ctx = Context(device)
    try:
        p = make_problem(L.CCSC_L3D, b.shape, kernel_size, lambda_residual, lambda_prior,
                         max_it, tol, verbose, **kw)
        d0 = z0 = None
        if init is not None and len(init) > 0:
            d0 = init.get("d")
            z0 = init.get("z")
        s = Session(ctx, p, b, d0, z0)
        try:
            done = False
            while s.outer < s.p.max_it and not done:
                done = s.step(1)
            d_res, z_res, DZ, obj = s.results(want_z=want_z, want_DZ=want_DZ, want_obj=True)
            log = s.iterlog()
        finally:
            s.close()
    finally:
        if own:
            ctx.close()
    iterations = {"obj_vals_d": [], "obj_vals_z": [], "tim_vals": [], "it_vals": [],
                  "trace": log["trace"], "engine_tim_vals": log["tim_vals"]}
    return d_res, z_res, DZ, obj, iterations


def admm_learn(b, kernel_size, lambda_residual, lambda_prior, max_it, tol, verbose, init=None,
               smooth_init=None, ctx=None, device=0, want_z=True, want_DZ=True, return_log=False,
               **kw):
    """Drop-in for 2-3D/DictionaryLearning/admm_learn.m:1-237 (hyperspectral learner).

    b, smooth_init: [x, y, W, n] (learn_hyperspectral.m:16-17 passes the 13x13 Gaussian
    low-pass of b); kernel_size = [psf, psf, W, K].  ``init = {'d': [psf,psf,K],
    'z': [X,Y,K,n]}`` (the reference's own draw: one filter replicated over W, L23:54-56;
    its init branch, L23:50-52, cannot run).  Returns (d_res [psf,psf,W,K], z_res [X,Y,K,n],
    Dz [X,Y,W,n] incl. smoothinit, obj_val) like the reference; ``return_log=True`` appends
    the engine's log (per-iteration objectives, 'rolled_back' for L23:204-213).
    """
    b = np.asarray(b, dtype=np.float64)
    if b.ndim == 3:
        b = b[..., None]
    if b.ndim != 4:
        raise ValueError("b must be [x, y, W, n]")
    if len(kernel_size) != 4 or int(kernel_size[2]) != b.shape[2]:
        raise ValueError("kernel_size must be [psf, psf, W, K] with W = size(b, 3)")
    if smooth_init is None:
        raise ValueError("smooth_init is required (admm_learn.m:4)")
    sm = np.asarray(smooth_init, dtype=np.float64).reshape(b.shape, order="F")
    own = ctx is None
    if own:
        ctx = Context(device)
    try:
        p = make_problem(L.CCSC_HS23, b.shape, kernel_size, lambda_residual, lambda_prior,
                         max_it, tol, verbose, **kw)
        d0 = z0 = None
        if init is not None and len(init) > 0:
            d0 = init.get("d")
            z0 = init.get("z")
        s = Session(ctx, p, b, d0, z0, smooth_init=sm)
        try:
            done = False
            while s.outer < s.p.max_it and not done:
                done = s.step(1)
            d_res, z_res, DZ, obj = s.results(want_z=want_z, want_DZ=want_DZ, want_obj=True)
            log = s.iterlog()
        finally:
            s.close()
    finally:
        if own:
            ctx.close()
    if not return_log:
        return d_res, z_res, DZ, obj
    log["rolled_back"] = bool(np.any(log["trace"]["flags"] & 1))
    log["outer"] = len(log["trace"]["flags"])
    return d_res, z_res, DZ, obj, log


def fft2d_test(ctx: Context, slices):
    """Kernel-level check: R2C half spectra + C2R round trip of [X, Y, count] slices."""
    a = np.asfortranarray(np.asarray(slices, dtype=np.float64))
    X, Y, cnt = a.shape
    Xh = X // 2 + 1
    hs = np.zeros(2 * Xh * Y * cnt)
    rt = np.zeros_like(a, order="F")
    eb = L.errbuf()
    L.check(L.lib().ccsc_test_fft2d(ctx.ptr, X, Y, cnt, L.dptr(a), L.dptr(hs), L.dptr(rt), eb,
                                    len(eb)), eb)
    h = hs.view(np.complex128).reshape(cnt, Y, Xh)          # [slice][y][x']
    return np.transpose(h, (2, 1, 0)), rt                     # [x', y, slice]
