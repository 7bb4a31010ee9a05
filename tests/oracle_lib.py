"""ctypes binding of the CPU oracle (oracle/build/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product package.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "liboracle.so")

_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")


class Stats(C.Structure):
    _fields_ = [
        ("numRowPanels", C.c_int32),
        ("numClusters", C.c_int32),
        ("numDenseBlock", C.c_int32),
        ("averageDensity", C.c_float),
        ("originalNumDenseBlock", C.c_int32),
        ("originalAverageDensity", C.c_float),
        ("numDenseThreadBlocks", C.c_int32),
        ("numSparseThreadBlocks", C.c_int32),
        ("numDenseData", C.c_int32),
        ("numSparseData", C.c_int32),
        ("maxNumDenseColBlocksInRowPanel", C.c_uint32),
        ("numDenseBlocksTotal", C.c_uint32),
        ("rphmNumSparseThreadBlocks", C.c_uint32),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


ARRAYS = ["reorderedRows", "denseCols", "denseColOffsets", "sparseCols", "sparseColOffsets",
          "sparseValueOffsets", "blockOffsets", "blockValues", "sparseValues",
          "sparseRelativeRows", "sparseColIndices"]

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(LIB_PATH)
        for f in ("orc_load_mtx", "orc_load_smtx", "orc_load_snap", "orc_load"):
            getattr(L, f).restype = C.c_void_p
            getattr(L, f).argtypes = [C.c_char_p, C.c_int]
        L.orc_csr_from_arrays.restype = C.c_void_p
        L.orc_csr_from_arrays.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, _u32p, _u32p]
        L.orc_csr_info.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_uint32)]
        L.orc_csr_copy.argtypes = [C.c_void_p, _u32p, _u32p, _f32p]
        L.orc_csr_free.argtypes = [C.c_void_p]
        L.orc_make_data.argtypes = [C.c_uint64, _f32p]
        L.orc_block_size.restype = C.c_uint32
        L.orc_block_size.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
        L.orc_cluster_block_dim.restype = C.c_uint32
        L.orc_cluster_block_dim.argtypes = [C.c_uint32]
        L.orc_row_reorder.argtypes = [C.c_void_p, C.c_float, C.c_uint32, C.c_int, _u32p,
                                      C.POINTER(C.c_uint32), C.POINTER(C.c_int32),
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.orc_dispersion.argtypes = [C.c_void_p, C.c_uint32, _u32p]
        L.orc_plan_from_rows.restype = C.c_void_p
        L.orc_plan_from_rows.argtypes = [C.c_void_p, _u32p, C.c_uint32, C.c_int32, C.c_float]
        L.orc_plan_stats.argtypes = [C.c_void_p, C.POINTER(Stats)]
        L.orc_plan_array.restype = C.c_uint64
        L.orc_plan_array.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.orc_plan_free.argtypes = [C.c_void_p]
        L.orc_sddmm_cpu.argtypes = [C.c_void_p, C.c_uint32, _f32p, _f32p, _f32p, C.c_int]
        L.orc_sddmm_cpu_rows.argtypes = [C.c_void_p, C.c_uint32, _f32p, _f32p, _f32p,
                                         C.c_uint32, C.c_uint32, C.c_int]
        L.orc_sddmm_cpu_rows_bound.restype = C.c_int
        L.orc_sddmm_cpu_rows_bound.argtypes = [C.c_void_p, C.c_uint32, _f32p, _f32p, _f32p,
                                               C.c_uint32, C.c_uint32, C.c_int, C.c_void_p, C.c_int]
        L.orc_check_one.restype = C.c_int
        L.orc_check_one.argtypes = [C.c_float, C.c_float]
        L.orc_check_data.restype = C.c_uint64
        L.orc_check_data.argtypes = [C.c_uint64, _f32p, _f32p, C.c_int]
        _lib = L
    return _lib


class CSR:
    def __init__(self, handle):
        if not handle:
            raise ValueError("oracle loader rejected the matrix")
        self.h = handle
        M, N, nnz = C.c_uint32(), C.c_uint32(), C.c_uint32()
        lib().orc_csr_info(handle, C.byref(M), C.byref(N), C.byref(nnz))
        self.M, self.N, self.nnz = M.value, N.value, nnz.value

    @classmethod
    def load(cls, path, verbose=False):
        h = lib().orc_load(path.encode(), 1 if verbose else 0)  # suffix dispatch
        return cls(h) if h else None

    @classmethod
    def from_arrays(cls, M, N, rowptr, colidx):
        rowptr = np.ascontiguousarray(rowptr, dtype=np.uint32)
        colidx = np.ascontiguousarray(colidx, dtype=np.uint32)
        return cls(lib().orc_csr_from_arrays(M, N, len(colidx), rowptr, colidx))

    def arrays(self):
        rp = np.empty(self.M + 1, np.uint32)
        ci = np.empty(self.nnz, np.uint32)
        v = np.empty(self.nnz, np.float32)
        lib().orc_csr_copy(self.h, rp, ci, v)
        return rp, ci, v

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_csr_free(self.h)
            self.h = None


def make_data(n):
    out = np.empty(n, np.float32)
    lib().orc_make_data(n, out)
    return out


def block_size(M, N, free_mem):
    return lib().orc_block_size(M, N, free_mem)


def row_reorder(csr, alpha, bs, exact_all=False):
    out = np.empty(max(csr.M, 1), np.uint32)
    n = C.c_uint32()
    ncl = C.c_int32()
    ne, nt = C.c_uint64(), C.c_uint64()
    lib().orc_row_reorder(csr.h, alpha, bs, 1 if exact_all else 0, out, C.byref(n), C.byref(ncl),
                          C.byref(ne), C.byref(nt))
    return out[: n.value].copy(), ncl.value, (ne.value, nt.value)


def dispersion(csr, bs):
    out = np.empty(csr.M, np.uint32)
    lib().orc_dispersion(csr.h, bs, out)
    return out


class Plan:
    def __init__(self, csr, rows, num_clusters, delta):
        rows = np.ascontiguousarray(rows, dtype=np.uint32)
        self.csr = csr
        self.h = lib().orc_plan_from_rows(csr.h, rows, len(rows), num_clusters, delta)

    def stats(self):
        s = Stats()
        lib().orc_plan_stats(self.h, C.byref(s))
        return s.as_dict()

    def array(self, name):
        which = ARRAYS.index(name)
        n = lib().orc_plan_array(self.h, which, None)
        out = np.empty(n, np.uint32)
        if n:
            lib().orc_plan_array(self.h, which, out.ctypes.data)
        return out

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_plan_free(self.h)
            self.h = None


def sddmm_cpu(csr, K, A, B, threads=0):
    P = np.empty(csr.nnz, np.float32)
    lib().orc_sddmm_cpu(csr.h, K, np.ascontiguousarray(A, np.float32),
                        np.ascontiguousarray(B, np.float32), P, threads)
    return P


def check_data(a, b, verbose=False):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    assert a.shape == b.shape
    return int(lib().orc_check_data(a.size, a, b, 1 if verbose else 0))
