"""rocSPARSE SDDMM baseline over libbsmr_rocsparse.so (include/bsmr_rocsparse.h).

The counterpart of the reference's cuSPARSE baseline (include/cuSparseSDDMM.cuh:27-145,
baselines/cuSPARSE_SDDMM/src/cuSPARSE-main.cu): P = (A·B) ∘ spy(S) with alpha 1, beta 0, the
default algorithm, on the engine's own operand layouts. A measured comparison on the same box,
never a fallback for the engine (nothing in bsmr/__init__.py calls it).
"""
import ctypes as C
import os

from . import F32, PKG_ROOT, BsmrError

LIB_PATH = os.path.join(PKG_ROOT, "lib", "libbsmr_rocsparse.so")
EXPORTS = ["bsmr_rocsparse_create", "bsmr_rocsparse_sddmm", "bsmr_rocsparse_destroy",
           "bsmr_rocsparse_last_error"]
ALGS = {"default": 0, "dense": 1}

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  (share torch's HIP runtime and rocSPARSE, see bsmr.lib)
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise BsmrError(f"rocSPARSE baseline not built: {LIB_PATH} is missing "
                        "(run `make -C sddmm-gpu_amd`)")
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    L.bsmr_rocsparse_last_error.restype = C.c_char_p
    L.bsmr_rocsparse_create.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp,
                                        C.c_int, C.c_int, vp, C.POINTER(vp)]
    L.bsmr_rocsparse_sddmm.argtypes = [vp, vp, vp, vp]
    L.bsmr_rocsparse_destroy.argtypes = [vp]
    _lib = L
    return L


def _check(status, what):
    if status != 0:
        msg = lib().bsmr_rocsparse_last_error().decode(errors="replace")
        raise BsmrError(f"{what} failed with status {status}: {msg}")


class RocsparseSddmm:
    """rocsparse_sddmm on device CSR pointers (d_rowptr, d_colidx: int device addresses)."""

    def __init__(self, M, N, K, nnz, d_rowptr, d_colidx, dtype=F32, alg="default", stream=0):
        h = C.c_void_p()
        _check(lib().bsmr_rocsparse_create(M, N, K, nnz, d_rowptr, d_colidx, dtype, ALGS[alg],
                                           stream or None, C.byref(h)), "bsmr_rocsparse_create")
        self.h = h

    def __call__(self, dA, dB, dP):
        _check(lib().bsmr_rocsparse_sddmm(self.h, dA, dB, dP), "bsmr_rocsparse_sddmm")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.bsmr_rocsparse_destroy(self.h)
            self.h = None
