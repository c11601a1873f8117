"""ctypes binding of libgcnk.so (the C-ABI declared in include/gcnk.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C <package>/csrc``).  There is no fallback: if the library is missing
or fails to load, every op raises ``RuntimeError`` — the hot path never
silently runs anywhere but the HIP kernels.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB = os.path.join(_HERE, "libgcnk.so")
VARIANT_DIR = os.path.join(os.path.dirname(_HERE), "_variants")


def _resolve_lib():
    """The in-tree library, unless GCNK_LIB names an experiment variant built by
    `make -C <pkg>/csrc variant` (it must live in <repo>/_variants/; anything
    else is refused, so a stale export cannot swap in a foreign binary).  A
    variant is announced on stderr; tests/conftest.py refuses to run on one."""
    want = os.environ.get("GCNK_LIB")
    if not want:
        return PRODUCT_LIB
    path = os.path.realpath(want)
    if os.path.dirname(path) != os.path.realpath(VARIANT_DIR):
        raise RuntimeError(f"GCNK_LIB={want}: only experiment variants in {VARIANT_DIR} may replace {PRODUCT_LIB}")
    import sys
    print(f"[gcnk] loading experiment variant {path} (not the product library)", file=sys.stderr)
    return path


LIB_PATH = _resolve_lib()
ABI_VERSION = 12

# C-ABI return codes (gcnk.h)
OK, EARG, EUNSUP, EHIP = 0, -1, -2, -3

# SpMM epilogues (gcnk.h GCNK_EPI_*)
EPI_NONE, EPI_BIAS, EPI_BIAS_RELU, EPI_BIAS_RELU_DROP, EPI_BIAS_RELU_HASH = 0, 1, 2, 3, 4
# GEMM epilogues (gcnk.h GCNK_GEMM_EPI_*)
GEMM_EPI_NONE, GEMM_EPI_BIAS, GEMM_EPI_BIAS_RELU, GEMM_EPI_MASK_POS = 0, 1, 2, 5

_vp, _i32, _i64, _u64, _f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float

# name -> (restype, argtypes); every symbol include/gcnk.h declares
SIGNATURES = {
    "gcnk_abi_version": (ctypes.c_int, []),
    "gcnk_debug_set_stamps": (ctypes.c_int, [_vp]),
    "gcnk_last_error": (ctypes.c_char_p, []),
    "gcnk_spmm_groups": (_i32, [_i32, _i32]),
    "gcnk_spmm_default_ipc": (_i32, [_i32, _i64, _i32, _i32]),
    # rowptr, colind, M, K, nnz, ipc, groups, dense_threshold, stream
    "gcnk_spmm_plan_bytes": (_i64, [_vp, _vp, _i32, _i32, _i64, _i32, _i32, _f32, _vp]),
    # rowptr, colind, val, M, K, nnz, ipc, groups, dense_threshold, plan, plan_bytes, stream
    "gcnk_spmm_plan_build": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _i64, _i32, _i32, _f32, _vp, _i64, _vp]),
    "gcnk_spmm_plan_bytes_host": (_i64, [_vp, _vp, _i32, _i32, _i64, _i32, _i32, _f32]),
    "gcnk_spmm_plan_build_host": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _i64, _i32, _i32, _f32, _vp, _i64]),
    "gcnk_spmm_plan_query": (ctypes.c_int, [_vp, _vp, _vp]),
    "gcnk_spmm_workspace_bytes": (_i64, [_vp, _i32]),
    "gcnk_spmm_counter_bytes": (_i64, [_vp]),
    "gcnk_spmm_csr_f32": (ctypes.c_int, [
        _vp, _vp,                 # plan (device), plan header (host, 16 words)
        _vp, _i64, _i32,          # B, ldb, F
        _vp, _i64,                # C, ldc
        _vp, _i32,                # bias, epilogue
        _vp, _i64, _f32,          # drop_mask, ldm, drop_scale
        _f32, _u64, _u64, _vp,    # keep_prob, seed, offset, rng_base
        _vp, _i64,                # workspace, workspace_bytes
        _vp, _i64,                # counters, counter_bytes
        _i32, _vp,                # lanes_hint, stream
    ]),
    "gcnk_spmm_csr_f32_part": (ctypes.c_int, [
        _vp, _vp,                 # plan (device), plan header (host, 16 words)
        _vp, _i64, _i32,          # B, ldb, F
        _vp, _i64,                # C, ldc
        _vp, _i32,                # bias, epilogue
        _vp, _i64, _f32,          # drop_mask, ldm, drop_scale
        _f32, _u64, _u64, _vp,    # keep_prob, seed, offset, rng_base
        _vp, _i64,                # workspace, workspace_bytes
        _vp, _i64,                # counters, counter_bytes
        _i32, _i32, _vp,          # lanes_hint, part, stream
    ]),
    "gcnk_spmm_proj_f32": (ctypes.c_int, [
        _vp, _vp,                 # plan, plan header
        _vp, _i64, _i32,          # B, ldb, F
        _vp, _i64,                # C (nullable), ldc
        _vp, _i32,                # bias, epilogue
        _vp, _i64, _f32,          # drop_mask, ldm, drop_scale
        _f32, _u64, _u64, _vp,    # keep_prob, seed, offset, rng_base
        _vp, _i64, _i32, _vp, _i64,  # W, ldw, P, C2, ldc2
        _vp, _i64,                # workspace, workspace_bytes
        _vp, _i64,                # counters, counter_bytes
        _i32, _vp,                # lanes_hint, stream
    ]),
    "gcnk_gemm_workspace_bytes": (_i64, [_i32, _i32, _i32, _i32]),
    "gcnk_gemm_f32": (ctypes.c_int, [
        _i32, _i32, _i32, _i32, _i32,   # transA, transB, M, N, K
        _vp, _i64, _vp, _i64,           # A, lda, B, ldb
        _vp, _i64,                      # C, ldc
        _vp, _i32, _vp, _i64, _f32,     # bias, epilogue, R, ldr, scale
        _i32, _vp, _i64, _vp,           # split_k, workspace, workspace_bytes, stream
    ]),
    "gcnk_colsum_workspace_bytes": (_i64, [_i32, _i32]),
    "gcnk_colsum_f32": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _i64, _vp]),
    "gcnk_gcn_bwd2_workspace_bytes": (_i64, [_i32, _i32, _i32]),
    "gcnk_gcn_bwd2_f32": (ctypes.c_int, [
        _vp, _i64, _vp, _i64, _vp, _i64,   # H, ldh, gS, ldgs, W, ldw
        _vp, _i64, _i32, _i32, _i32, _f32,  # G, ldg, M, N, P, scale
        _vp, _i64, _vp, _vp, _vp,          # gZ1, ldz, gW, gb1, gb2
        _vp, _i64, _vp]),                  # workspace, bytes, stream
    "gcnk_stream_copy_f32": (ctypes.c_int, [_vp, _vp, _i64, _vp]),
    "gcnk_debug_poison_lds": (ctypes.c_int, [ctypes.c_uint32, _vp]),
    "gcnk_hubfactor_lds_bytes": (_i64, [_i32, _i32, _i32, _i32, _i32]),
    "gcnk_hubfactor_gc1_f32": (ctypes.c_int, [
        _i32, _i32, _i32, _i32, _i32,     # M, F, Kc, nhub, P
        _vp, _i64, _vp, _i64, _i32,       # U, ldu, W, ldw, k0
        _vp, _i64, _vp, _i32,             # S, lds, rec, rec_words
        _vp, _i32,                        # bias, epilogue
        _vp, _i64, _f32,                  # drop_mask, ldm, drop_scale
        _f32, _u64, _u64, _vp,            # keep_prob, seed, offset, rng_base
        _vp, _i64, _vp, _i64, _vp, _i64,  # W2, ldw2, H, ldh, C2, ldc2
        _vp]),                            # stream
    "gcnk_dense_gc1_f32": (ctypes.c_int, [
        _i32, _i32, _i32, _i32,           # M, K, F, P
        _vp, _i64, _vp, _i64,             # AX, ldax, W1, ldw1
        _vp, _i32,                        # bias, epilogue
        _vp, _i64, _f32,                  # drop_mask, ldm, drop_scale
        _f32, _u64, _u64, _vp,            # keep_prob, seed, offset, rng_base
        _vp, _i64, _vp, _i64, _vp, _i64,  # W2, ldw2, H, ldh, C2, ldc2
        _vp]),                            # stream
    "gcnk_aggregate_f32": (ctypes.c_int, [_vp, _vp, _vp, _i32, _vp, _i64, _i32, _vp, _i64, _i32, _vp]),
    # record (host struct gcnk_gcn_fwd), W1, b1, W2, b2, out, ldo, H1, ldh, epilogue, mask, ldm, scale,
    # keep_prob, seed, offset, rng_base, stream
    "gcnk_gcn_forward_f32": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _i32, _vp, _i64, _f32,
                                            _f32, _u64, _u64, _vp, _vp]),
    "gcnk_gcn_fwd_layout": (_i32, [_vp, _i32]),
    "gcnk_factor_u_f32": (ctypes.c_int, [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _i32, _vp]),
    "gcnk_factor_records": (ctypes.c_int, [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _i32, _vp, _vp]),
    "gcnk_factor_analyze_workspace_bytes": (_i64, [_i32, _i32]),
    # rowptr, colind, M, hmin, x_rowptr, x_colind, x_val, x_dense, ldx, K, max_hubs, info, hubs, cnt (host),
    # workspace, bytes, stream
    "gcnk_factor_analyze": (ctypes.c_int, [_vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp,
                                           _vp, _i64, _vp]),
    "gcnk_factor_xl_f32": (ctypes.c_int, [_vp, _vp, _vp, _i32, _vp, _i32, _i32, _vp, _i64, _i32, _vp]),
    "gcnk_csr_gather_rows": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "gcnk_dense_gather_rows_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _i64, _vp]),
    "gcnk_gcn_backward_f32": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _f32, _vp, _vp, _vp, _vp, _vp]),
    "gcnk_class_stats": (ctypes.c_int, [_vp, _i64, _vp, _vp, _i64, _i32, _vp, _vp]),
    "gcnk_edgelist_size": (ctypes.c_int, [ctypes.c_char_p, _vp, _vp]),
    "gcnk_edgelist_csr": (ctypes.c_int, [ctypes.c_char_p, _i64, _i64, _vp, _vp, _vp]),
    "gcnk_csr_to_dense": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _vp, _i64, _vp]),
    "gcnk_bernoulli_mt19937": (ctypes.c_int, [_vp, _vp, _vp, _i64, ctypes.c_double, _vp, _i32]),
    "gcnk_bernoulli_mt19937_start": (ctypes.c_int, [_vp, _vp, _vp, _i64, ctypes.c_double, _vp, _vp]),
    "gcnk_bernoulli_mt19937_wait": (ctypes.c_int, [_vp]),
    "gcnk_sym_normalize_workspace_bytes": (_i64, [_i32, _i64]),
    "gcnk_sym_normalize": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "gcnk_csr_transpose_workspace_bytes": (_i64, [_i32, _i32, _i64]),
    "gcnk_coo_to_csr_workspace_bytes": (_i64, [_i64, _i32, _i32]),
    "gcnk_coo_to_csr": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _vp]),
    "gcnk_csr_transpose": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
}

_lock = threading.Lock()
_lib = None


class GcnkError(RuntimeError):
    """Raised when a libgcnk entry point returns a non-zero code."""


def load():
    """Load libgcnk.so once and bind every declared symbol; raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libgcnk.so not found at {LIB_PATH}: build it with __graft_entry__.build() "
                "or `make -C <package>/csrc` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.gcnk_abi_version()
        if v != ABI_VERSION:
            raise RuntimeError(f"libgcnk ABI version {v} != expected {ABI_VERSION}")
        _lib = lib
        return lib


def check(rc, what):
    if rc != OK:
        msg = load().gcnk_last_error().decode(errors="replace")
        kind = {EARG: "bad argument", EUNSUP: "unsupported", EHIP: "HIP error"}.get(rc, "error")
        raise GcnkError(f"{what} failed ({kind}, rc={rc}): {msg} [{LIB_PATH}]")
