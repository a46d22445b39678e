"""ctypes binding of libabcgpu.so (the C ABI declared in include/abcgpu.h).

This is the ONLY route from the Python layer to the device kernels.  If the
library is missing or cannot be loaded, importing the GPU classes raises
immediately: there is no CPU fallback on the product path.
"""
import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ABCGPU_LIB", os.path.join(_HERE, "libabcgpu.so"))

P = C.c_void_p
I64 = C.c_int64
I32 = C.c_int
D = C.c_double
U64 = C.c_uint64
U32 = C.c_uint32
SZ = C.c_size_t

# name -> (restype, argtypes); mirrors include/abcgpu.h one to one
SIGNATURES = {
    "abc_last_error": (C.c_char_p, []),
    "abc_version": (I32, []),
    "abc_profile_begin": (I32, []),
    "abc_profile_end": (I32, [P, P]),
    "abc_profile_channel": (I32, [I32, P, P]),
    "abc_weighted_moments_workspace": (SZ, [I64, I32]),
    "abc_weighted_moments": (I32, [P, P, I64, I32, P, P, SZ, P]),
    "abc_scan_workspace": (SZ, [I64]),
    "abc_inclusive_scan_f64": (I32, [P, P, I64, P, SZ, P]),
    "abc_normalize_weights_workspace": (SZ, [I64]),
    "abc_normalize_weights": (I32, [P, I64, P, P, SZ, P]),
    "abc_mvn_packed_bytes": (SZ, [I64, I32, I32]),
    "abc_mvn_x3_layout": (I32, [I32, P, P]),
    "abc_mvn_pack_population": (I32, [P, P, I64, I32, P, P, I32, D, P, I32, P, P,
                                      P]),
    "abc_mvn_fit": (I32, [P, I32, D, I32, P, P, P, P, P, P, P]),
    "abc_mvn_logpdf_workspace": (SZ, [I64, I64, I32, I32]),
    "abc_mvn_logpdf": (I32, [P, I64, I32, P, P, P, I64, P, P, I32, I32, D, D,
                             P, P, P, SZ, P]),
    "abc_mvn_logpdf_direct": (I32, [P, I64, P, P, I64, I32, P, I32, P, I32,
                                    D, D, P, P]),
    "abc_cdf_guide": (I32, [P, I64, P, P]),
    "abc_ancestor_table_bytes": (I64, [I64, I32]),
    "abc_ancestor_table": (I32, [P, P, I64, I32, P, SZ, P]),
    "abc_propose": (I32, [P, P, P, I64, I32, P, P, P, U64, U32, I64, I64, I32,
                          P, P, P, P, P]),
    "abc_prior_logpdf": (I32, [P, I64, I32, P, P, P, P]),
    "abc_prior_uniforms": (I32, [P, P, I64, I32, U64, U32, I64, P]),
    "abc_simulate_linear_gaussian": (I32, [P, I64, I32, I32, P, P, P, U64,
                                           U32, I64, P, P]),
    "abc_pnorm": (I32, [P, I64, I32, P, P, D, P, P]),
    "abc_mask_gave_up": (I32, [P, P, I64, I32, D, P]),
    "abc_compact_workspace": (SZ, [I64]),
    "abc_accept_compact": (I32, [P, I64, D, P, P, P, SZ, P]),
    "abc_candidates_workspace": (SZ, [I64]),
    "abc_prior_support_box": (I32, [P, P, I32, P, P]),
    "abc_round_keep": (I32, [P, I32, I32, I64, P, P]),
    "abc_candidates_round": (I32, [P, I64, I64, D, P, D, I32, I64, P, P, P, P, SZ, P]),
    "abc_candidates_regen": (I32, [P, I64, P, I64, P, P, P, P, P, P, P]),
    "abc_pnorm_accept": (I32, [P, I64, I32, P, P, D, D, P, I32, I64, P, P, P, SZ, P]),
    "abc_candidates_propose_workspace": (SZ, []),
    "abc_candidates_propose": (I32, [P, I64, I64, P, P, P, P, P, SZ, P]),
    "abc_gather_rows": (I32, [P, P, I64, I32, P, P]),
    "abc_gather_rows_batch": (I32, [I32, P, P, P, P, P, I64, P]),
    "abc_importance_weights": (I32, [P, P, P, I64, D, P, P]),
    "abc_sort_pairs_workspace": (SZ, [I64]),
    "abc_sort_pairs_f64": (I32, [P, P, I64, P, P, P, SZ, P]),
    "abc_weighted_quantile_workspace": (SZ, [I64]),
    "abc_weighted_quantile": (I32, [P, P, I64, D, P, P, SZ, P]),
    "abc_weighted_quantile_sorted_workspace": (SZ, [I64]),
    "abc_weighted_quantile_sorted": (I32, [P, P, I64, D, P, P, SZ, P]),
    "abc_column_stats_workspace": (SZ, [I64, I32]),
    "abc_column_std": (I32, [P, I64, I32, P, P, SZ, P]),
    "abc_column_mad": (I32, [P, I64, I32, P, P, SZ, P]),
    "abc_local_fit_workspace": (SZ, [I64, I32]),
    "abc_local_fit": (I32, [P, P, I64, I32, I64, D, D, P, P, P, P, P, P, SZ,
                            P]),
    "abc_local_logpdf_workspace": (SZ, [I64, I64, I32]),
    "abc_local_logpdf": (I32, [P, I64, P, P, I64, I32, P, P, P, P, SZ, P]),
    "abc_local_propose": (I32, [P, P, P, I64, I32, P, P, P, U64, U32, I64,
                                I64, I32, P, P, P, P, P]),
    "abc_bootstrap_cv_workspace": (SZ, [I64]),
    "abc_bootstrap_cv": (I32, [P, I64, I64, P, D, P, P, P, SZ, P]),
    "abc_kernel_logpdf": (I32, [P, I64, I32, P, I32, P, I32, P, P, I32, D,
                                I32, P, P]),
    "abc_stochastic_accept": (I32, [P, I64, D, D, I32, I32, U64, U32, I64,
                                    P, P, P]),
    "abc_temper_workspace": (SZ, []),
    "abc_temper_sums": (I32, [P, P, P, I64, D, I32, I32, D, D, P, P, SZ, P]),
    "abc_comm_unique_id": (I32, [P]),
    "abc_comm_init": (I32, [P, I32, I32, P]),
    "abc_comm_destroy": (I32, [P]),
    "abc_comm_allgather": (I32, [P, P, P, SZ, P]),
    "abc_comm_allreduce": (I32, [P, P, P, SZ, I32, I32, P]),
    "abc_comm_broadcast": (I32, [P, P, SZ, I32, P]),
}



class CandidateSpec(C.Structure):
    """abc_candidate_spec (include/abcgpu.h), field for field."""
    _fields_ = [("d", C.c_int), ("S", C.c_int),
                ("X", P), ("cdf", P), ("guide", P), ("N", I64),
                ("L", P), ("per_particle_L", C.c_int),
                ("prior_kind", P), ("prior_params", P), ("max_attempts", C.c_int),
                ("src", P), ("a", P), ("sigma", P),
                ("x0", P), ("wf", P), ("p", D),
                ("seed", U64), ("generation", U32), ("anc_table", P),
                ("support_box", P)]


# C error codes (include/abcgpu.h)
ABC_OK = 0
ABC_ERR_INVALID = -1
ABC_ERR_HIP = -2
ABC_ERR_WORKSPACE = -3
ABC_ERR_NOT_ENOUGH_PARTICLES = -4
ABC_ERR_UNSUPPORTED = -5
ABC_ERR_COMM = -6
ABC_COMM_ID_BYTES = 128
ABC_COMM_F64, ABC_COMM_I64 = 0, 1
ABC_COMM_SUM, ABC_COMM_MAX, ABC_COMM_MIN = 0, 1, 2
ABC_PROF_DENSITY, ABC_PROF_CANDIDATES, ABC_PROF_REGEN, ABC_PROF_RESCUE = 0, 1, 2, 3
ABC_PREC_F64 = 0
ABC_PREC_F32 = 1
ABC_PREC_X3 = 2

PRIOR_KINDS = {"norm": 0, "uniform": 1, "expon": 2, "laplace": 3,
               "lognorm": 4, "gamma": 5, "beta": 6, "host": 7}


class NativeError(RuntimeError):
    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


_lib = None
_lock = threading.Lock()


def load():
    """Load libabcgpu.so once; raise if it is absent (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libabcgpu.so not found at {LIB_PATH}; build it with "
                "`python -m pyabc_amd.build` (hipcc, gfx950)")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def call(name, *args):
    """Invoke an entry point and raise on a non-zero return code."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != ABC_OK:
        msg = lib.abc_last_error().decode(errors="replace")
        if rc == ABC_ERR_INVALID:
            raise ValueError(f"{name}: {msg}")
        raise NativeError(name, rc, msg)
    return rc


def query(name, *args):
    """Invoke a size query (returns size_t)."""
    return int(getattr(load(), name)(*args))
