"""Python host mirror of the reference BSMR-SDDMM interface, over libbsmr_amd.so (include/bsmr.h).

Reference interface mirrored (paths relative to the reference root):
  * sparseMatrix::CSR<float>::initializeFromMatrixFile -> load_mtx        (src/Matrix.cpp:279-480)
  * Matrix<float>::makeData                            -> make_data       (src/Matrix.cpp:117-138)
  * BSMR(alpha, delta, S) + RPHM(S, bsmr)              -> Plan            (src/BSMR.cpp:16-265)
  * sddmm_gpu(M, N, K, dA, dB, rphm, dP, logger)       -> Plan.sddmm      (src/sddmmKernel.cu:2540)
  * evaluationReordering                               -> Plan.evaluate   (src/BSMR.cpp:826-994)

Every call goes through the HIP library; there is no CPU fallback. If the shared library is
missing the import fails loudly (build it with `make -C sddmm-gpu_amd` or
`python -c "import __graft_entry__ as g; g.build()"`).
"""
import ctypes as C
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# BSMR_LIB_PATH: another build of the same library (A/B timing of kernel variants only)
LIB_PATH = os.environ.get("BSMR_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libbsmr_amd.so")

F32, F16, BF16 = 0, 1, 2
CHECK_FAILED = 7  # BSMR_ERR_CHECK

ARRAYS = {
    "reorderedRows": 0, "denseCols": 1, "denseColOffsets": 2, "sparseCols": 3,
    "sparseColOffsets": 4, "sparseValueOffsets": 5, "blockOffsets": 6, "blockValues": 7,
    "sparseValues": 8, "sparseRelativeRows": 9, "sparseColIndices": 10, "dispersion": 11,
    "ascending": 12,
}

_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")


class BsmrError(RuntimeError):
    pass


class Tuning(C.Structure):
    """bsmr_tuning: launch-layout knobs (include/bsmr.h). "auto" = -1 (diag 0)."""
    _fields_ = [("diag", C.c_uint32), ("tile_min_f32", C.c_int32),
                ("tile_min_half", C.c_int32), ("piece_max", C.c_int32),
                ("piece_weight", C.c_float), ("shard_piece_weight", C.c_float),
                ("dense_min", C.c_float), ("orig_rows", C.c_int32), ("orig_contig", C.c_int32),
                ("dense_ks", C.c_int32), ("dense_ns", C.c_int32), ("out_staged", C.c_int32),
                ("l2_range_kb", C.c_int32), ("stage_nt", C.c_int32),
                ("rb_rows", C.c_int32), ("late_b", C.c_int32), ("item_cap", C.c_float),
                ("item_sched", C.c_int32), ("out_packed", C.c_int32),
                ("cluster_filter", C.c_int32), ("pair_min_items", C.c_int32),
                ("batches", C.c_int32), ("ptile", C.c_int32), ("ptile_tpi", C.c_int32),
                ("piece_balance", C.c_int32), ("col_blocks", C.c_int32)]


# tuning field <- its debug environment variable (bsmr_tuning_from_env)
TUNING_ENV = {f: "BSMR_" + f.upper() for f, _ in Tuning._fields_}


class PlanOptions(C.Structure):
    _fields_ = [("alpha", C.c_float), ("delta", C.c_float), ("free_mem_bytes", C.c_uint64),
                ("device", C.c_int), ("cluster_batch", C.c_uint32),
                ("exact_similarity", C.c_int), ("layout", C.c_int),
                ("lds_budget_kb", C.c_uint32), ("tuning", C.POINTER(Tuning))]


LAYOUTS = {"auto": 0, "rowblock": 1, "colmajor": 2}


class PlanStats(C.Structure):
    _fields_ = [("M", C.c_uint32), ("N", C.c_uint32), ("nnz", C.c_uint32),
                ("block_size", C.c_uint32), ("num_blocks_per_row", C.c_uint32),
                ("cluster_block_dim", C.c_uint32), ("num_clusters", C.c_int32),
                ("num_row_panels", C.c_uint32), ("num_reordered_rows", C.c_uint32),
                ("num_dense_tiles", C.c_uint32), ("max_dense_tiles_per_panel", C.c_uint32),
                ("num_residual", C.c_uint32), ("num_dense_thread_blocks", C.c_uint32),
                ("num_sparse_thread_blocks", C.c_uint32),
                ("exact_similarity_evals", C.c_uint64), ("total_similarity_evals", C.c_uint64),
                ("row_reorder_ms", C.c_float), ("col_reorder_ms", C.c_float),
                ("dense_items", C.c_uint32), ("residual_items", C.c_uint32),
                ("rb_rows", C.c_uint32 * 5), ("rb_items", C.c_uint32 * 5),
                ("rb_pieces", C.c_uint32 * 5), ("rb_entries", C.c_uint32 * 5),
                ("rb_tiles", C.c_uint32 * 5), ("rb_work_items", C.c_uint32 * 5),
                ("dense_sampled_tiles", C.c_uint32), ("rb_orig_rows", C.c_uint32),
                ("ptile_items", C.c_uint32), ("cluster_filter_used", C.c_uint32),
                ("cluster_filter_ms", C.c_float), ("rb_pairs", C.c_uint32),
                ("rb_batches", C.c_uint32), ("rb_col_blocks", C.c_uint32)]

    def as_dict(self):
        d = {}
        for k, _ in self._fields_:
            v = getattr(self, k)
            d[k] = list(v) if hasattr(v, "__len__") else v
        return d


class EvalStats(C.Structure):
    _fields_ = [("num_dense_block", C.c_int32), ("average_density", C.c_float),
                ("original_num_dense_block", C.c_int32), ("original_average_density", C.c_float),
                ("num_dense_data", C.c_int32), ("num_sparse_data", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class RowStage(C.Structure):
    """bsmr_row_stage: the clustering result a multi-GPU run computes once and broadcasts."""
    _fields_ = [("M", C.c_uint32), ("N", C.c_uint32), ("nnz", C.c_uint32),
                ("block_size", C.c_uint32), ("num_blocks_per_row", C.c_uint32),
                ("cluster_block_dim", C.c_uint32), ("num_zero_rows", C.c_uint32),
                ("num_reordered_rows", C.c_uint32), ("num_clusters", C.c_int32),
                ("alpha", C.c_float), ("row_reorder_ms", C.c_float),
                ("exact_similarity_evals", C.c_uint64), ("total_similarity_evals", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}

    def to_array(self):
        """The header as bytes in a uint8 array (to ship it in a broadcast)."""
        return np.frombuffer(bytes(self), dtype=np.uint8).copy()

    @classmethod
    def from_array(cls, a):
        return cls.from_buffer_copy(np.ascontiguousarray(a, np.uint8).tobytes())


ABI_VERSION = 13  # include/bsmr.h BSMR_ABI_VERSION

# every symbol include/bsmr.h declares (tests check the library exports all of them)
EXPORTS = [
    "bsmr_last_error", "bsmr_abi_version", "bsmr_csr_load_mtx", "bsmr_csr_load_smtx",
    "bsmr_csr_load_snap", "bsmr_csr_load", "bsmr_csr_create",
    "bsmr_csr_info", "bsmr_csr_rowptr", "bsmr_csr_colidx", "bsmr_csr_values", "bsmr_csr_free",
    "bsmr_make_data", "bsmr_tuning_default", "bsmr_tuning_from_env",
    "bsmr_plan_options_default", "bsmr_plan_create", "bsmr_plan_recolumn",
    "bsmr_plan_destroy", "bsmr_plan_get_stats", "bsmr_plan_get_array", "bsmr_plan_evaluate",
    "bsmr_sddmm", "bsmr_sddmm_batch", "bsmr_plan_shard", "bsmr_plan_shard_dtype",
    "bsmr_shard_cuts", "bsmr_plan_shard_rebalance", "bsmr_sddmm_panels",
    "bsmr_sddmm_panels_local",
    "bsmr_plan_export_rows", "bsmr_plan_import_rows",
    "bsmr_sddmm_profile", "bsmr_sddmm_cpu", "bsmr_check_one", "bsmr_check_data",
    "bsmr_plan_check", "bsmr_check_rphm_arrays", "bsmr_cost_cuts",
]

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    try:
        # Share torch's HIP runtime when torch is present: torch/lib/libamdhip64.so and
        # /opt/rocm's carry the same SONAME but torch asks for the unversioned name, so loading
        # ours first would put two HIP runtimes in the process.
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise BsmrError(f"HIP extension not built: {LIB_PATH} is missing "
                        "(run `make -C sddmm-gpu_amd`)")
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    L.bsmr_last_error.restype = C.c_char_p
    L.bsmr_abi_version.restype = C.c_int
    if L.bsmr_abi_version() != ABI_VERSION:  # the structs below mirror include/bsmr.h
        raise BsmrError(f"{LIB_PATH}: ABI {L.bsmr_abi_version()}, binding expects {ABI_VERSION} "
                        "(rebuild with `make -C sddmm-gpu_amd`)")
    for f in ("bsmr_csr_load_mtx", "bsmr_csr_load_smtx", "bsmr_csr_load_snap", "bsmr_csr_load"):
        getattr(L, f).argtypes = [C.c_char_p, C.c_int, C.POINTER(vp)]
    L.bsmr_csr_create.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, _u32p, _u32p, C.POINTER(vp)]
    L.bsmr_csr_info.argtypes = [vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                C.POINTER(C.c_uint32)]
    L.bsmr_csr_rowptr.restype = C.POINTER(C.c_uint32)
    L.bsmr_csr_rowptr.argtypes = [vp]
    L.bsmr_csr_colidx.restype = C.POINTER(C.c_uint32)
    L.bsmr_csr_colidx.argtypes = [vp]
    L.bsmr_csr_values.restype = C.POINTER(C.c_float)
    L.bsmr_csr_values.argtypes = [vp]
    L.bsmr_csr_free.argtypes = [vp]
    L.bsmr_make_data.argtypes = [C.c_uint64, _f32p]
    L.bsmr_plan_options_default.argtypes = [C.POINTER(PlanOptions)]
    L.bsmr_tuning_default.argtypes = [C.POINTER(Tuning)]
    L.bsmr_tuning_from_env.argtypes = [C.POINTER(Tuning)]
    L.bsmr_tuning_from_env.restype = C.c_int
    L.bsmr_plan_create.argtypes = [_u32p, _u32p, C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.POINTER(PlanOptions), C.POINTER(vp)]
    L.bsmr_plan_recolumn.argtypes = [vp, C.c_float]
    L.bsmr_plan_destroy.argtypes = [vp]
    L.bsmr_plan_get_stats.argtypes = [vp, C.POINTER(PlanStats)]
    L.bsmr_plan_get_array.argtypes = [vp, C.c_int, vp, C.POINTER(C.c_uint64)]
    L.bsmr_plan_evaluate.argtypes = [vp, C.POINTER(EvalStats)]
    L.bsmr_sddmm.argtypes = [vp, vp, vp, C.c_uint32, C.c_int, vp, vp]
    L.bsmr_sddmm_batch.argtypes = [vp, C.c_uint32, vp, vp, C.c_uint32, C.c_int, vp, vp]
    L.bsmr_plan_shard.argtypes = [vp, C.c_uint32, C.c_int, C.c_int, C.POINTER(C.c_uint32),
                                  C.POINTER(C.c_uint32)]
    L.bsmr_plan_shard_dtype.argtypes = [vp, C.c_uint32, C.c_int, C.c_int, C.c_int,
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.bsmr_shard_cuts.argtypes = [_u32p, _u32p, C.c_uint32, C.c_uint32, C.c_int, _u32p]
    L.bsmr_plan_shard_rebalance.argtypes = [vp, C.c_uint32, C.c_int, C.c_int, _u32p, _f32p, _u32p]
    L.bsmr_cost_cuts.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, vp, vp, _u32p]
    L.bsmr_sddmm_panels.argtypes = [vp, vp, vp, C.c_uint32, C.c_int, vp, C.c_uint32,
                                    C.c_uint32, vp]
    L.bsmr_sddmm_panels_local.argtypes = [vp, vp, vp, C.c_uint32, C.c_int, vp, C.c_uint32,
                                          C.c_uint32, vp]
    L.bsmr_plan_export_rows.argtypes = [vp, C.POINTER(RowStage), vp]
    L.bsmr_plan_import_rows.argtypes = [_u32p, _u32p, C.POINTER(RowStage), vp,
                                        C.POINTER(PlanOptions), C.POINTER(vp)]
    L.bsmr_sddmm_cpu.argtypes = [_u32p, _u32p, C.c_uint32, C.c_uint32, C.c_uint32, _f32p, _f32p,
                                 _f32p, C.c_int]
    L.bsmr_check_one.restype = C.c_int
    L.bsmr_check_one.argtypes = [C.c_float, C.c_float]
    L.bsmr_check_data.restype = C.c_uint64
    L.bsmr_check_data.argtypes = [C.c_uint64, _f32p, _f32p, C.c_int]
    L.bsmr_sddmm_profile.argtypes = [vp, vp, vp, C.c_uint32, C.c_int, vp, C.c_int, vp,
                                     C.POINTER(C.c_float), C.POINTER(C.c_float),
                                     C.POINTER(C.c_float)]
    L.bsmr_plan_check.argtypes = [vp, C.c_uint32, C.c_int, C.c_int]
    L.bsmr_plan_check.restype = C.c_int
    L.bsmr_check_rphm_arrays.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32] + [_u32p] * 2 + \
        [C.c_uint32] + [_u32p] * 11 + [C.c_float, C.c_int]
    L.bsmr_check_rphm_arrays.restype = C.c_int
    _lib = L
    return L


def _check(status, what):
    if status != 0:
        msg = lib().bsmr_last_error().decode(errors="replace")
        raise BsmrError(f"{what} failed with status {status}: {msg}")


_default_tuning = {}


def tuning_from_env(env=None):
    """The tuning knobs given as BSMR_<FIELD> variables, as a {field: value} dict for Plan(tuning=).
    env: a mapping (e.g. a test's parameters); None reads this process's environment through the
    library's own parser (bsmr_tuning_from_env). The library never reads them by itself."""
    t = Tuning()
    lib().bsmr_tuning_default(C.byref(t))
    base = {f: getattr(t, f) for f, _ in Tuning._fields_}
    if env is None:
        lib().bsmr_tuning_from_env(C.byref(t))
        return {f: getattr(t, f) for f, _ in Tuning._fields_ if getattr(t, f) != base[f]}
    out = {}
    for f, _ in Tuning._fields_:
        v = env.get(TUNING_ENV[f])
        if v is None:
            continue
        if f in ("orig_rows", "out_staged", "stage_nt", "item_sched", "out_packed", "cluster_filter",
                 "batches", "ptile", "piece_balance"):  # tri-state: "0" never, "1" always, else auto
            out[f] = 0 if v.startswith("0") else 1 if v.startswith("1") else -1
        elif f in ("piece_weight", "shard_piece_weight", "dense_min", "item_cap"):
            out[f] = float(v)
        else:
            out[f] = int(v)
    return out


def set_default_tuning(tuning):
    """Tuning applied to every later Plan built without an explicit `tuning` (tools and bench
    call this with tuning_from_env() so their A/B runs can be steered from the environment)."""
    global _default_tuning
    _default_tuning = dict(tuning or {})


def _tuning_struct(tuning):
    t = Tuning()
    lib().bsmr_tuning_default(C.byref(t))
    for k, v in (tuning or {}).items():
        if k not in TUNING_ENV:
            raise BsmrError(f"unknown tuning field {k!r}")
        setattr(t, k, v)
    return t


def make_data(n):
    """Matrix<float>::makeData stream: default-seeded mt19937, uniform [0, 2)."""
    out = np.empty(int(n), np.float32)
    lib().bsmr_make_data(out.size, out)
    return out


class Csr:
    """Host CSR (uint32 rowptr/colidx), as sparseMatrix::CSR<float>."""

    def __init__(self, handle):
        self.h = handle
        M, N, nnz = C.c_uint32(), C.c_uint32(), C.c_uint32()
        lib().bsmr_csr_info(handle, C.byref(M), C.byref(N), C.byref(nnz))
        self.M, self.N, self.nnz = M.value, N.value, nnz.value

    @classmethod
    def load_mtx(cls, path, verbose=False):
        return cls._load("bsmr_csr_load_mtx", path, verbose)

    @classmethod
    def load(cls, path, verbose=False):
        """Any supported file (.mtx/.mmio, .smtx, SNAP .txt) by suffix; None if rejected."""
        return cls._load("bsmr_csr_load", path, verbose)

    @classmethod
    def _load(cls, fn, path, verbose):
        h = C.c_void_p()
        st = getattr(lib(), fn)(path.encode(), 1 if verbose else 0, C.byref(h))
        if st != 0:
            return None
        return cls(h)

    @classmethod
    def from_arrays(cls, M, N, rowptr, colidx):
        rowptr = np.ascontiguousarray(rowptr, np.uint32)
        colidx = np.ascontiguousarray(colidx, np.uint32)
        h = C.c_void_p()
        _check(lib().bsmr_csr_create(M, N, len(colidx), rowptr, colidx, C.byref(h)),
               "bsmr_csr_create")
        return cls(h)

    @property
    def rowptr(self):
        return np.ctypeslib.as_array(lib().bsmr_csr_rowptr(self.h), shape=(self.M + 1,)).copy()

    @property
    def colidx(self):
        return np.ctypeslib.as_array(lib().bsmr_csr_colidx(self.h), shape=(self.nnz,)).copy()

    @property
    def values(self):
        return np.ctypeslib.as_array(lib().bsmr_csr_values(self.h), shape=(self.nnz,)).copy()

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.bsmr_csr_free(self.h)
            self.h = None


def load_mtx(path, verbose=False):
    return Csr.load_mtx(path, verbose)


def load(path, verbose=False):
    return Csr.load(path, verbose)


class Plan:
    """Device-resident BSMR plan (reordered rows, dense 16x16 tiles, residual lists)."""

    def __init__(self, M, N, rowptr, colidx, alpha=0.3, delta=0.3, free_mem_bytes=0, device=0,
                 cluster_batch=0, exact_similarity=False, layout="auto", lds_budget_kb=0,
                 tuning=None, _row_stage=None):
        """tuning: {bsmr_tuning field: value} (None = the process default, normally empty)."""
        rowptr = np.ascontiguousarray(rowptr, np.uint32)
        colidx = np.ascontiguousarray(colidx, np.uint32)
        o = PlanOptions()
        lib().bsmr_plan_options_default(C.byref(o))
        o.alpha = float(np.float32(alpha))
        o.delta = float(np.float32(delta))
        o.free_mem_bytes = int(free_mem_bytes)
        o.device = int(device)
        o.cluster_batch = int(cluster_batch)
        o.exact_similarity = 1 if exact_similarity else 0
        o.layout = LAYOUTS[layout]
        o.lds_budget_kb = int(lds_budget_kb)
        self._tuning = _tuning_struct(_default_tuning if tuning is None else tuning)
        o.tuning = C.pointer(self._tuning)
        self.M, self.N, self.nnz = int(M), int(N), int(len(colidx))
        h = C.c_void_p()
        if _row_stage is None:
            _check(lib().bsmr_plan_create(rowptr, colidx, M, N, len(colidx), C.byref(o),
                                          C.byref(h)), "bsmr_plan_create")
        else:
            hdr, rows_ptr = _row_stage
            _check(lib().bsmr_plan_import_rows(rowptr, colidx, C.byref(hdr), rows_ptr,
                                               C.byref(o), C.byref(h)), "bsmr_plan_import_rows")
        self.h = h

    @classmethod
    def from_row_stage(cls, rowptr, colidx, hdr, rows, delta=0.3, device=0, layout="auto",
                       lds_budget_kb=0, tuning=None):
        """bsmr_plan_import_rows: the plan of an exported row stage (no clustering). rows: a
        uint32 numpy array, or an int device pointer (e.g. a broadcast tensor's data_ptr())."""
        if isinstance(rows, np.ndarray):
            rows = np.ascontiguousarray(rows, np.uint32)
            ptr = rows.ctypes.data
        else:
            ptr = int(rows)
        return cls(hdr.M, hdr.N, rowptr, colidx, alpha=hdr.alpha, delta=delta, device=device,
                   layout=layout, lds_budget_kb=lds_budget_kb, tuning=tuning,
                   _row_stage=(hdr, ptr))

    def export_rows(self, rows_out=None):
        """bsmr_plan_export_rows: (header, rows). rows_out: None (a numpy array is returned) or
        an int pointer (host or device) receiving num_reordered_rows uint32."""
        hdr = RowStage()
        _check(lib().bsmr_plan_export_rows(self.h, C.byref(hdr), None), "bsmr_plan_export_rows")
        if rows_out is None:
            rows = np.empty(max(hdr.num_reordered_rows, 1), np.uint32)
            _check(lib().bsmr_plan_export_rows(self.h, C.byref(hdr), rows.ctypes.data),
                   "bsmr_plan_export_rows")
            return hdr, rows[:hdr.num_reordered_rows]
        _check(lib().bsmr_plan_export_rows(self.h, C.byref(hdr), int(rows_out)),
               "bsmr_plan_export_rows")
        return hdr, None

    def recolumn(self, delta):
        _check(lib().bsmr_plan_recolumn(self.h, float(np.float32(delta))), "bsmr_plan_recolumn")

    def stats(self):
        s = PlanStats()
        _check(lib().bsmr_plan_get_stats(self.h, C.byref(s)), "bsmr_plan_get_stats")
        return s.as_dict()

    def array(self, name):
        which = ARRAYS[name]
        n = C.c_uint64()
        _check(lib().bsmr_plan_get_array(self.h, which, None, C.byref(n)), "bsmr_plan_get_array")
        out = np.empty(n.value, np.uint32)
        if n.value:
            _check(lib().bsmr_plan_get_array(self.h, which, out.ctypes.data, C.byref(n)),
                   "bsmr_plan_get_array")
        return out

    def evaluate(self):
        e = EvalStats()
        _check(lib().bsmr_plan_evaluate(self.h, C.byref(e)), "bsmr_plan_evaluate")
        return e.as_dict()

    def check(self, K=0, dtype=F32, verbose=True):
        """bsmr_plan_check (the reference's check_rphm, BSMR.cpp:932-953): (True, "") when the plan
        and, for K > 0, the launch layout of (K, dtype) pass; (False, first error) otherwise."""
        st = lib().bsmr_plan_check(self.h, K, dtype, 1 if verbose else 0)
        if st == 0:
            return True, ""
        msg = lib().bsmr_last_error().decode(errors="replace")
        if st != CHECK_FAILED:
            raise BsmrError(f"bsmr_plan_check failed with status {st}: {msg}")
        return False, msg

    def sddmm(self, dA, dB, K, dP, stream=0, dtype=F32):
        """dA, dB, dP: device pointers (int) — e.g. torch tensor .data_ptr()."""
        _check(lib().bsmr_sddmm(self.h, dA, dB, K, dtype, dP, stream or None), "bsmr_sddmm")

    def sddmm_batch(self, num_batch, dA, dB, K, dP, stream=0, dtype=F32):
        """num_batch (A, B) pairs: batch b at dA + b*M*K, dB + b*N*K elements, dP + b*nnz."""
        _check(lib().bsmr_sddmm_batch(self.h, num_batch, dA, dB, K, dtype, dP, stream or None),
               "bsmr_sddmm_batch")

    def sddmm_panels(self, dA, dB, K, dP, p0, p1, stream=0, dtype=F32):
        _check(lib().bsmr_sddmm_panels(self.h, dA, dB, K, dtype, dP, p0, p1, stream or None),
               "bsmr_sddmm_panels")

    def sddmm_panels_local(self, dA_local, dB, K, dP, p0, p1, stream=0, dtype=F32):
        """Shard launch with a shard-local A: rows of reordered positions [16 p0, 16 p1)."""
        _check(lib().bsmr_sddmm_panels_local(self.h, dA_local, dB, K, dtype, dP, p0, p1,
                                             stream or None), "bsmr_sddmm_panels_local")

    def shard(self, K, rank, world, dtype=F32):
        """Panel range [p0, p1) of `rank` (bsmr_plan_shard_dtype)."""
        p0, p1 = C.c_uint32(), C.c_uint32()
        _check(lib().bsmr_plan_shard_dtype(self.h, K, dtype, rank, world, C.byref(p0),
                                           C.byref(p1)), "bsmr_plan_shard_dtype")
        return p0.value, p1.value

    def shard_rebalance(self, K, world, prev_cuts, shard_ms, dtype=F32):
        """Cuts [0 = c_0 <= ... <= c_world = P] re-balanced by measured shard times
        (bsmr_plan_shard_rebalance); prev_cuts: the cuts those times were measured on."""
        prev = np.ascontiguousarray(prev_cuts, np.uint32)
        ms = np.ascontiguousarray(shard_ms, np.float32)
        if len(prev) != world + 1 or len(ms) != world:
            raise ValueError("shard_rebalance: prev_cuts needs world + 1 entries, shard_ms world")
        cuts = np.zeros(world + 1, np.uint32)
        _check(lib().bsmr_plan_shard_rebalance(self.h, K, dtype, world, prev, ms, cuts),
               "bsmr_plan_shard_rebalance")
        return [int(c) for c in cuts]

    def profile(self, dA, dB, K, dP, iters=10, stream=0, dtype=F32):
        d, r, t = C.c_float(), C.c_float(), C.c_float()
        _check(lib().bsmr_sddmm_profile(self.h, dA, dB, K, dtype, dP, iters, stream or None,
                                        C.byref(d), C.byref(r), C.byref(t)),
               "bsmr_sddmm_profile")
        return {"dense_ms": d.value, "residual_ms": r.value, "total_ms": t.value}

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.bsmr_plan_destroy(self.h)
            self.h = None


def shard_cuts(block_offsets, sparse_value_offsets, K, world):
    """Panel cut points [0 = c_0 <= ... <= c_world = P] of the row-panel sharding cost model."""
    bo = np.ascontiguousarray(block_offsets, np.uint32)
    so = np.ascontiguousarray(sparse_value_offsets, np.uint32)
    P = len(bo) - 1
    cuts = np.zeros(world + 1, np.uint32)
    _check(lib().bsmr_shard_cuts(bo, so, P, K, world, cuts), "bsmr_shard_cuts")
    return cuts


def cost_cuts(block_cost, panels_per_block, P, world, prev_cuts=None, shard_ms=None):
    """bsmr_cost_cuts: row-block cuts of P panels by block costs (host only), optionally re-balanced
    by the times shard_ms[r] measured on prev_cuts (bsmr_plan_shard_rebalance's rule)."""
    bc = np.ascontiguousarray(block_cost, np.float64)
    cuts = np.zeros(world + 1, np.uint32)
    pc = None if prev_cuts is None else np.ascontiguousarray(prev_cuts, np.uint32)
    ms = None if shard_ms is None else np.ascontiguousarray(shard_ms, np.float32)
    if (pc is None) != (ms is None) or (pc is not None and (len(pc) != world + 1 or len(ms) != world)):
        raise ValueError("cost_cuts: prev_cuts (world + 1) and shard_ms (world) go together")
    ptr = (lambda a: None if a is None else a.ctypes.data)
    _check(lib().bsmr_cost_cuts(ptr(bc), len(bc), panels_per_block, P, world, ptr(pc), ptr(ms),
                                cuts), "bsmr_cost_cuts")
    return [int(c) for c in cuts]


def sddmm_cpu(M, N, rowptr, colidx, K, A, B, threads=0):
    """bsmr_sddmm_cpu: the reference's host SDDMM (host.cpp:45-76) as product code."""
    rowptr = np.ascontiguousarray(rowptr, np.uint32)
    colidx = np.ascontiguousarray(colidx, np.uint32)
    P = np.empty(len(colidx), np.float32)
    _check(lib().bsmr_sddmm_cpu(rowptr, colidx, M, N, K, np.ascontiguousarray(A, np.float32),
                                np.ascontiguousarray(B, np.float32), P, threads), "bsmr_sddmm_cpu")
    return P


def check_rphm_arrays(M, N, rowptr, colidx, arrays, delta, verbose=True):
    """bsmr_check_rphm_arrays: the reference's check_rphm (BSMR.cpp:932-953) over host arrays.
    `arrays` maps the plan array names (ARRAYS keys) to uint32 arrays. Returns (ok, first error)."""
    a = {k: np.ascontiguousarray(v, dtype=np.uint32) for k, v in arrays.items()}
    rp = np.ascontiguousarray(rowptr, dtype=np.uint32)
    ci = np.ascontiguousarray(colidx, dtype=np.uint32)
    order = ["denseColOffsets", "denseCols", "sparseColOffsets", "sparseCols",
             "sparseValueOffsets", "blockOffsets", "blockValues", "sparseValues",
             "sparseRelativeRows", "sparseColIndices"]
    rows = a["reorderedRows"]
    st = lib().bsmr_check_rphm_arrays(M, N, len(ci), rp, ci, len(rows), rows,
                                      *[a[k] for k in order], float(delta), 1 if verbose else 0)
    if st == 0:
        return True, ""
    msg = lib().bsmr_last_error().decode(errors="replace")
    if st != CHECK_FAILED:
        raise BsmrError(f"bsmr_check_rphm_arrays failed with status {st}: {msg}")
    return False, msg


def check_data(data1, data2, verbose=False):
    """bsmr_check_data (checkData.hpp:44-79): number of mismatches; verbose prints the report."""
    a = np.ascontiguousarray(data1, np.float32)
    b = np.ascontiguousarray(data2, np.float32)
    if a.shape != b.shape:
        raise ValueError("check_data: sizes differ")
    return int(lib().bsmr_check_data(a.size, a, b, 1 if verbose else 0))
