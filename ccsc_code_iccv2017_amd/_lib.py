"""ctypes binding of libccsc.so (the C-ABI declared in include/ccsc.h).

The library is built in-tree by ``ccsc_code_iccv2017_amd.build``.  There is no
fallback: if the shared library is missing or lacks a symbol, loading fails
loudly (the GPU engine is the only implementation of the product path).
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "libccsc.so"

CCSC_OK = 0
CCSC_E_INVALID = -1
CCSC_E_HIP = -2
CCSC_E_RCCL = -3
CCSC_E_NOMEM = -4
CCSC_E_UNSUPPORTED = -5
CCSC_E_STATE = -6

CCSC_DPAR, CCSC_DZPAR, CCSC_L3D, CCSC_L4D, CCSC_HS23 = 0, 1, 2, 3, 4
ABI_VERSION = 7
VERBOSE = {"none": 0, "brief": 1, "all": 2}
CCSC_FP64 = 0
CCSC_FP32 = 1  # deprecated: CCSC_E_UNSUPPORTED
DFACTOR = {"auto": 0, "cholesky": 1, "woodbury": 2}
TRANSPORT = {0: "none", 1: "rccl", 2: "host"}


class Problem(C.Structure):
    _fields_ = [
        ("variant", C.c_int32),
        ("ndim", C.c_int32),
        ("sb", C.c_int64 * 3),
        ("views", C.c_int32 * 2),
        ("n", C.c_int64),
        ("K", C.c_int32),
        ("psf", C.c_int32),
        ("lambda_residual", C.c_double),
        ("lambda_prior", C.c_double),
        ("max_it", C.c_int32),
        ("tol", C.c_double),
        ("verbose", C.c_int32),
        ("ni", C.c_int32),
        ("max_it_d", C.c_int32),
        ("max_it_z", C.c_int32),
        ("rho_d", C.c_double),
        ("rho_z", C.c_double),
        ("theta_div", C.c_double),
        ("precision", C.c_int32),
        ("trace_objective", C.c_int32),
        ("seed", C.c_uint64),
        ("dfactor", C.c_int32),
    ]


_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class Outputs(C.Structure):
    _fields_ = [("d_res", _dp), ("z_res", _dp), ("DZ", _dp), ("obj_val", _dp)]


class IterLog(C.Structure):
    _fields_ = [
        ("capacity", C.c_int32),
        ("count", C.c_int32),
        ("obj_vals_d", _dp),
        ("obj_vals_z", _dp),
        ("tim_vals", _dp),
        ("trace_obj_d", _dp),
        ("trace_obj_z", _dp),
        ("trace_d_diff", _dp),
        ("trace_z_diff", _dp),
        ("n_d", _ip),
        ("n_z", _ip),
        ("flags", _ip),
    ]


# reconstruction solvers (ccsc_solve)
CCSC_SOLVE_INPAINT2D, CCSC_SOLVE_POISSON2D, CCSC_SOLVE_MULTICH, CCSC_SOLVE_VIDEO3D = 0, 1, 2, 3


class SolveProblem(C.Structure):
    _fields_ = [
        ("variant", C.c_int32),
        ("sb", C.c_int64 * 3),
        ("nch", C.c_int32),
        ("n", C.c_int64),
        ("K", C.c_int32),
        ("ksize", C.c_int32 * 3),
        ("psf_size", C.c_int32 * 3),
        ("lambda_residual", C.c_double),
        ("lambda_prior", C.c_double),
        ("max_it", C.c_int32),
        ("tol", C.c_double),
        ("verbose", C.c_int32),
    ]


class SolveInputs(C.Structure):
    _fields_ = [("b", _dp), ("kernels", _dp), ("mask", _dp), ("smooth_init", _dp), ("psf", _dp),
                ("x_orig", _dp)]


class SolveOutputs(C.Structure):
    _fields_ = [("z", _dp), ("res", _dp)]


class SolveLog(C.Structure):
    _fields_ = [("capacity", C.c_int32), ("iters", _ip), ("obj", _dp), ("psnr", _dp),
                ("diff", _dp), ("seconds", _dp)]


CB = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_double, C.c_double, C.c_double)
COMM_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.c_int64)

# name -> (restype, argtypes); mirrors include/ccsc.h exactly
SIGNATURES = {
    "ccsc_abi_version": (C.c_int32, []),
    "ccsc_resolve": (C.c_int32, [C.POINTER(Problem), C.c_char_p, C.c_size_t]),
    "ccsc_supported": (C.c_int32, [C.POINTER(Problem), C.c_char_p, C.c_size_t]),
    "ccsc_shard": (C.c_int32, [C.POINTER(Problem), C.c_int32, C.c_int32, C.POINTER(C.c_int64),
                               C.POINTER(C.c_int64), C.c_char_p, C.c_size_t]),
    "ccsc_plan_bytes": (C.c_int32, [C.POINTER(Problem), C.c_int32, C.c_int32,
                                    C.POINTER(C.c_uint64), C.c_char_p, C.c_size_t]),
    "ccsc_device_count": (C.c_int32, [C.POINTER(C.c_int32), C.c_char_p, C.c_size_t]),
    "ccsc_get_unique_id": (C.c_int32, [C.c_char_p, C.c_char_p, C.c_size_t]),
    "ccsc_create": (C.c_void_p, [C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_char_p,
                                 C.c_size_t]),
    "ccsc_create_hostcomm": (C.c_void_p, [C.c_int32, C.c_int32, C.c_int32, COMM_FN, C.c_void_p,
                                          C.c_char_p, C.c_size_t]),
    "ccsc_create_multi": (C.c_void_p, [C.POINTER(C.c_int32), C.c_int32, C.c_char_p, C.c_size_t]),
    "ccsc_destroy": (None, [C.c_void_p]),
    "ccsc_comm_ranks": (C.c_int32, [C.c_void_p, _ip, _ip, C.c_char_p, C.c_size_t]),
    "ccsc_learn": (C.c_int32, [C.c_void_p, C.POINTER(Problem), _dp, _dp, _dp,
                               C.POINTER(Outputs), C.POINTER(IterLog), CB, C.c_void_p,
                               C.c_char_p, C.c_size_t]),
    "ccsc_learn_hs23": (C.c_int32, [C.c_void_p, C.POINTER(Problem), _dp, _dp, _dp, _dp,
                                    C.POINTER(Outputs), C.POINTER(IterLog), CB, C.c_void_p,
                                    C.c_char_p, C.c_size_t]),
    "ccsc_session_create": (C.c_void_p, [C.c_void_p, C.POINTER(Problem), _dp, _dp, _dp,
                                         C.c_char_p, C.c_size_t]),
    "ccsc_session_create_hs23": (C.c_void_p, [C.c_void_p, C.POINTER(Problem), _dp, _dp, _dp, _dp,
                                              C.c_char_p, C.c_size_t]),
    "ccsc_session_step": (C.c_int32, [C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.c_char_p,
                                      C.c_size_t]),
    "ccsc_session_objective": (C.c_int32, [C.c_void_p, _dp, C.c_char_p, C.c_size_t]),
    "ccsc_session_results": (C.c_int32, [C.c_void_p, C.POINTER(Outputs), C.c_char_p,
                                         C.c_size_t]),
    "ccsc_session_iterlog": (C.c_int32, [C.c_void_p, C.POINTER(IterLog), C.c_char_p,
                                         C.c_size_t]),
    "ccsc_session_set_profiling": (C.c_int32, [C.c_void_p, C.c_int32]),
    "ccsc_session_kernel_stats": (C.c_int32, [C.c_void_p, C.c_int32, C.POINTER(C.c_int64),
                                              _dp, _dp, C.c_char_p, C.c_size_t]),
    "ccsc_session_destroy": (None, [C.c_void_p]),
    "ccsc_solve_supported": (C.c_int32, [C.POINTER(SolveProblem), C.c_char_p, C.c_size_t]),
    "ccsc_solve": (C.c_int32, [C.c_void_p, C.POINTER(SolveProblem), C.POINTER(SolveInputs),
                               C.POINTER(SolveOutputs), C.POINTER(SolveLog), C.c_char_p,
                               C.c_size_t]),
    "ccsc_local_cn": (C.c_int32, [C.c_void_p, _dp, _dp, C.c_int64, C.c_int32, C.c_int32,
                                  C.c_char_p, C.c_size_t]),
    "ccsc_local_cn_dev": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32,
                                      C.c_int32, C.c_char_p, C.c_size_t]),
    "ccsc_test_fft2d": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, _dp, _dp, _dp,
                                    C.c_char_p, C.c_size_t]),
}

_LIB = None


class CCSCError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libccsc error {code}: {msg}")
        self.code = code


def lib():
    """Load libccsc.so (no fallback)."""
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -m ccsc_code_iccv2017_amd.build` "
                "(the HIP engine has no CPU fallback)")
        # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7 (the soname of
        # /opt/rocm's).  With torch loaded first libccsc binds to that copy; loaded the
        # other way round the process maps both, and torch's then sees no GPU ("No HIP
        # GPUs are available") once libccsc has initialised the device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def errbuf():
    return C.create_string_buffer(1024)


def check(rc, eb):
    if rc != CCSC_OK:
        raise CCSCError(rc, eb.value.decode(errors="replace"))


def dptr(a):
    if a is None:
        return C.cast(None, _dp)
    return a.ctypes.data_as(_dp)


def iptr(a):
    if a is None:
        return C.cast(None, _ip)
    return a.ctypes.data_as(_ip)
