"""Functional ops on the HIP kernels and the autograd Functions of the GCN path.

Each op replaces an arithmetic site of the reference (cited per function);
tensors cross the C-ABI as raw device pointers plus torch's current stream,
so every op is asynchronous and hipGraph-capturable.
"""
import ctypes
import os

import torch

from . import _lib, factor
from .sparse import CSR, DENSE_THRESHOLD, as_csr, require_device

_NULL = ctypes.c_void_p(0)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else _NULL


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _dense_f32(t, what):
    require_device(t, what)
    if t.dtype != torch.float32:
        raise RuntimeError(f"{what} must be float32 (the reference computes in fp32), got {t.dtype}")
    if t.dim() != 2:
        raise RuntimeError(f"{what} must be 2-D, got shape {tuple(t.shape)}")
    if t.stride(1) != 1:
        t = t.contiguous()
    return t


def default_ipc(a, F, lanes=0):
    return int(_lib.load().gcnk_spmm_default_ipc(a.shape[0], a.nnz, F, int(lanes)))


def spmm(a, B, bias=None, epilogue=_lib.EPI_NONE, mask=None, scale=1.0, keep_prob=1.0, seed=0, offset=0,
         out=None, ipc=None, lanes=0, dense=None, rng_base=None):
    """C = epi(A @ B) with A a CSR (or torch sparse) and B dense [K, F].

    Replaces ``th.spmm(adj, support)`` (reference layer.py:106) and
    ``th.spmm(X, W)`` with sparse X (layer.py:102); the epilogue fuses
    ``+ bias`` (layer.py:110), ``th.relu`` (layer.py:182) and the dropout
    multiply (layer.py:185).  ``rng_base``: optional one-element int64 device
    tensor added to ``offset`` by the kernel (hash dropout in captured graphs,
    include/gcnk.h GCNK_EPI_BIAS_RELU_HASH)."""
    a = as_csr(a)
    B = _dense_f32(B, "dense operand")
    _check_rng_base(rng_base, B.device)
    M, K = a.shape
    if B.shape[0] != K:
        raise RuntimeError(f"spmm shape mismatch: sparse {tuple(a.shape)} @ dense {tuple(B.shape)}")
    if B.device != a.device:
        raise RuntimeError(f"spmm device mismatch: {a.device} vs {B.device}")
    F = B.shape[1]
    if out is None:
        out = torch.empty((M, F), dtype=torch.float32, device=B.device)
    if bias is not None:
        bias = bias.contiguous()
    if mask is not None:
        mask = mask.contiguous()
    lib = _lib.load()
    if ipc is None:
        ipc = default_ipc(a, F, lanes)
    groups = int(lib.gcnk_spmm_groups(F, int(lanes)))
    plan = a.plan(ipc, groups, DENSE_THRESHOLD if dense is None else dense)
    wsb = plan.workspace_bytes(F)
    ws = torch.empty((wsb + 3) // 4, dtype=torch.float32, device=B.device) if wsb > 0 else None
    cnt = plan.counters(B.device)
    args = (_ptr(plan.buf), ctypes.cast(plan.hdr, ctypes.c_void_p),
            _ptr(B), B.stride(0), F,
            _ptr(out), out.stride(0),
            _ptr(bias), epilogue,
            _ptr(mask), mask.stride(0) if mask is not None else 0, float(scale),
            float(keep_prob), int(seed) & (2**64 - 1), int(offset) & (2**64 - 1), _ptr(rng_base),
            _ptr(ws), wsb, _ptr(cnt), 4 * cnt.numel() if cnt is not None else 0, int(lanes))
    hdr = plan.hdr
    nsingle, ntile, nunits = int(hdr[15]), int(hdr[8]), int(hdr[5])
    with torch.cuda.device(B.device):
        if OVERLAP_TILE_PARTS and nsingle > 0 and (ntile > nsingle or nunits > 0):
            # the single-chunk tile blocks on a side stream, the rest (multi-chunk
            # blocks, their reduce launch, the row kernel) on the caller's stream;
            # they write disjoint rows of `out` and the caller's stream joins the
            # side stream before anything reads it (captured into hipGraphs as a
            # fork/join)
            main = torch.cuda.current_stream(B.device)
            side = _side_stream(B.device)
            side.wait_stream(main)
            rc = lib.gcnk_spmm_csr_f32_part(*args, 1, ctypes.c_void_p(side.cuda_stream))
            _lib.check(rc, "gcnk_spmm_csr_f32_part")
            rc = lib.gcnk_spmm_csr_f32_part(*args, 2, _stream(B.device))
            main.wait_stream(side)
        else:
            rc = lib.gcnk_spmm_csr_f32(*args, _stream(B.device))
    _lib.check(rc, "gcnk_spmm_csr_f32")
    return out


def _check_rng_base(t, device):
    if t is not None and (t.dtype != torch.int64 or t.numel() < 1 or t.device != device):
        raise RuntimeError("rng_base must be an int64 tensor of >= 1 element on the operand's device")


# Overlap the two independent parts of a hybrid plan (gcnk_spmm_csr_f32_part)
# on two streams: R8's X W1 would run its document blocks beside the dense
# topic rows and their reduce launch.  Off: replayed from a hipGraph the
# fork/join measured 26.2 us for X W1 against 14.2 us on one stream
# (profiles/r01_variants.log).
OVERLAP_TILE_PARTS = False
_SIDE_STREAMS = {}


def _side_stream(device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _SIDE_STREAMS.get(idx)
    if st is None:
        st = _SIDE_STREAMS[idx] = torch.cuda.Stream(device=idx)
    return st


# Fuse gc2's H1 W2 into the gc1 aggregation epilogue (gcnk_spmm_proj_f32):
# one launch fewer, and the eval forward never writes or re-reads H1.  R8
# (profiles/r02_forward_schedules.log): fused A S1 + H1 W2 11.2 us against
# 10.1 + 3.4 us for the SpMM + skinny-GEMM pair, forward 36.2 vs 39.1 us.
# (Round 1's version, W in registers at 4 waves per SIMD, took 20.8 us.)
# GCNK_FUSE_PROJECTION=0 turns it off (experiments).  Only for gc2 widths up
# to FUSE_MAX_P: the 20ng-shaped graph's 20 classes take the 32-channel kernel,
# whose per-row projection costs more than the launch it saves (forward 106 us
# fused vs 58 us unfused, profiles/r02_variants.log).
FUSE_PROJECTION = os.environ.get("GCNK_FUSE_PROJECTION", "1") != "0"
FUSE_MAX_P = int(os.environ.get("GCNK_FUSE_MAX_P", "8"))
# gc2's backward + gc1's ReLU/dropout backward in one pass over H1 (gcn_bwd2)
FUSE_BACKWARD = os.environ.get("GCNK_FUSE_BACKWARD", "1") != "0"


def spmm_proj(a, B, W, bias=None, epilogue=_lib.EPI_NONE, mask=None, scale=1.0, keep_prob=1.0, seed=0, offset=0,
              store_main=True, ipc=None, lanes=0, rng_base=None):
    """(H, C2) with H = epi(A @ B) and C2 = H @ W, the projection fused into
    the SpMM epilogue (gcnk_spmm_proj_f32): gc1's aggregation + bias + ReLU +
    dropout (reference layer.py:106,110,182,185) followed by gc2's support
    ``th.spmm(H1, W2)`` (layer.py:102) while H1's elements are in registers.
    With ``store_main=False`` H is never written (returned as None).  Where the
    fused kernel does not apply (library returns unsupported) the same result
    comes from gcnk_spmm_csr_f32 + gcnk_gemm_f32."""
    a = as_csr(a)
    B = _dense_f32(B, "dense operand")
    W = _dense_f32(W, "projection")
    _check_rng_base(rng_base, B.device)
    M, K = a.shape
    F = B.shape[1]
    if B.shape[0] != K or W.shape[0] != F:
        raise RuntimeError(f"spmm_proj shape mismatch: {tuple(a.shape)} @ {tuple(B.shape)} @ {tuple(W.shape)}")
    P = W.shape[1]
    lib = _lib.load()
    if not lanes:
        lanes = 64   # the projection needs a whole row in one lane group (one column tile)
    if ipc is None:
        ipc = default_ipc(a, F, lanes)
    groups = int(lib.gcnk_spmm_groups(F, int(lanes)))
    plan = a.plan(ipc, groups, DENSE_THRESHOLD)
    H = torch.empty((M, F), dtype=torch.float32, device=B.device) if store_main else None
    if bias is not None:
        bias = bias.contiguous()
    if mask is not None:
        mask = mask.contiguous()
    wsb = plan.workspace_bytes(F)
    ws = torch.empty((wsb + 3) // 4, dtype=torch.float32, device=B.device) if wsb > 0 else None
    cnt = plan.counters(B.device)
    C2 = torch.empty((M, P), dtype=torch.float32, device=B.device)
    with torch.cuda.device(B.device):
        rc = lib.gcnk_spmm_proj_f32(
            _ptr(plan.buf), ctypes.cast(plan.hdr, ctypes.c_void_p),
            _ptr(B), B.stride(0), F,
            _ptr(H), F,
            _ptr(bias), epilogue,
            _ptr(mask), mask.stride(0) if mask is not None else 0, float(scale),
            float(keep_prob), int(seed) & (2**64 - 1), int(offset) & (2**64 - 1), _ptr(rng_base),
            _ptr(W), W.stride(0), P, _ptr(C2), C2.stride(0),
            _ptr(ws), wsb, _ptr(cnt), 4 * cnt.numel() if cnt is not None else 0, int(lanes), _stream(B.device))
    if rc == _lib.EUNSUP:
        H = spmm(a, B, bias=bias, epilogue=epilogue, mask=mask, scale=scale, keep_prob=keep_prob, seed=seed,
                 offset=offset, ipc=ipc, lanes=lanes, rng_base=rng_base)
        return (H if store_main else None), gemm(H, W)
    _lib.check(rc, "gcnk_spmm_proj_f32")
    return H, C2


# gc1 through the hub factorisation (factor.py, csrc/factor.hip) when the
# (A-hat, X) pair has the doc-topic structure and the factored launch is the
# faster one (factor.pays); GCNK_FACTOR_GC1=1 takes it whenever the operands
# factor, =0 never (experiments, A/B timing).
_FACTOR_ENV = os.environ.get("GCNK_FACTOR_GC1", "auto")
FACTOR_GC1 = "auto" if _FACTOR_ENV == "auto" else _FACTOR_ENV != "0"


def factor_for(adj, xop):
    """The HubFactor gc1 runs through for (adj, X), or None (the SpMM path)."""
    if not FACTOR_GC1:
        return None
    f = factor.get(adj, xop)
    if f is not None and FACTOR_GC1 == "auto" and not factor.pays(f, adj.device):
        return None
    return f


def hubfactor_gc1(f, W1, b1, W2, epilogue=_lib.EPI_BIAS_RELU, mask=None, scale=1.0, keep_prob=1.0, seed=0,
                  offset=0, rng_base=None, store_h1=True, S=None):
    """(H1, S2) of gc1 + gc2's support through the hub factorisation ``f``
    (factor.HubFactor): S_T = X[hubs] W1 (layer.py:102), then one launch of
    gcnk_hubfactor_gc1_f32 -- H1 = drop(relu(A-hat X W1 + b1))
    (layer.py:106,110,182,185) and S2 = H1 W2 (layer.py:102, gc2).  Returns
    None when the shapes are outside the kernel's range (the caller takes the
    SpMM path).  ``S``: S_T already computed (timing probes)."""
    W1 = _dense_f32(W1, "gc1 weight")
    W2 = _dense_f32(W2, "gc2 weight")
    _check_rng_base(rng_base, W1.device)
    M, F, P = f.M, W1.shape[1], W2.shape[1]
    if W1.stride(0) != F:
        W1 = W1.contiguous()   # the kernel stages W1[k0:k0+Kc], S_T and W2 as flat copies
    if W2.stride(0) != P:
        W2 = W2.contiguous()
    if W2.shape[0] != F or P > 32 or F % 4 or F > 256:
        return None
    lib = _lib.load()
    if int(lib.gcnk_hubfactor_lds_bytes(F, f.Kc, f.H, f.rec_words, P)) > 160 * 1024:
        return None
    if S is None:
        S = f.hub_times(W1, train=store_h1).contiguous()
    H1 = torch.empty((M, F), dtype=torch.float32, device=W1.device) if store_h1 else None
    S2 = torch.empty((M, P), dtype=torch.float32, device=W1.device)
    if b1 is not None:
        b1 = b1.contiguous()
    if mask is not None:
        mask = mask.contiguous()
    with torch.cuda.device(W1.device):
        rc = lib.gcnk_hubfactor_gc1_f32(
            M, F, f.Kc, f.H, P, _ptr(f.U), f.U.stride(0), _ptr(W1), W1.stride(0), f.k0, _ptr(S), S.stride(0),
            _ptr(f.rec), f.rec_words, _ptr(b1), epilogue,
            _ptr(mask), mask.stride(0) if mask is not None else 0, float(scale),
            float(keep_prob), int(seed) & (2**64 - 1), int(offset) & (2**64 - 1), _ptr(rng_base),
            _ptr(W2), W2.stride(0), _ptr(H1), F, _ptr(S2), P, _stream(W1.device))
    if rc == _lib.EUNSUP:
        return None
    _lib.check(rc, "gcnk_hubfactor_gc1_f32")
    return H1, S2


# gc1 from a cached A-hat X (csrc/dense_gc1.hip) for a dense, narrow X (at most
# DENSE_AX_MAX_K features: the gensim-shaped topic features of README.md:77,95):
# one launch (A-hat X) W1 + b1, ReLU, dropout and gc2's H1 W2 instead of the
# X W1 GEMM, the F-wide SpMM and the projection.  GCNK_DENSE_AX=0 turns it off
# (A/B timing), =1 / auto (default) takes it wherever it applies.
DENSE_AX = os.environ.get("GCNK_DENSE_AX", "auto") != "0"
DENSE_AX_MAX_K = 128


class DenseAX:
    """A-hat X [M x K] (fp32, rows padded to a multiple of 4 floats), built once
    per (A-hat, X) pair: float64 row sums in CSR order rounded once
    (gcnk_aggregate_f32, the factored path's U kernel with every row light)."""

    __slots__ = ("AX", "K", "_src")


def dense_ax_for(adj, xop, F=None, P=None):
    """The cached DenseAX of (adj, X) when the narrow-feature gc1 applies, else None."""
    if not DENSE_AX or xop.dense is None:
        return None
    M, K = xop.shape
    if adj.shape[0] != adj.shape[1] or adj.shape[1] != M or K > DENSE_AX_MAX_K or K == 0:
        return None
    if (F is not None and (F > 256 or F % 4)) or (P is not None and P > 32):   # (csrc/dense_gc1.hip's range)
        return None
    src = xop.dense
    key = (id(src), src.data_ptr(), src._version, adj.val.data_ptr(), adj.val._version)
    cache = getattr(adj, "_dense_ax", None)
    if cache is None:
        cache = adj._dense_ax = {}
    hit = cache.get(key)
    if hit is not None:
        return hit
    if src.stride(1) != 1:
        src = src.contiguous()
    Kp = (K + 3) // 4 * 4
    AX = torch.empty((adj.shape[0], Kp), dtype=torch.float32, device=adj.device)
    with torch.cuda.device(adj.device):
        _lib.check(_lib.load().gcnk_aggregate_f32(_ptr(adj.rowptr), _ptr(adj.colind), _ptr(adj.val), adj.shape[0],
                                                  _ptr(src), src.stride(0), K, _ptr(AX), Kp, Kp,
                                                  _stream(adj.device)), "gcnk_aggregate_f32")
    d = DenseAX()
    d.AX, d.K, d._src = AX, K, xop.dense   # (holds the operand: its id cannot be recycled while cached)
    while len(cache) >= 4:
        cache.pop(next(iter(cache)))
    cache[key] = d
    return d


def dense_gc1(d, W1, b1, W2, epilogue=_lib.EPI_BIAS_RELU, mask=None, scale=1.0, keep_prob=1.0, seed=0, offset=0,
              rng_base=None, store_h1=True):
    """(H1, S2) of gc1 + gc2's support from A-hat X (DenseAX ``d``): one launch of
    gcnk_dense_gc1_f32 -- H1 = drop(relu((A-hat X) W1 + b1)) (reference
    layer.py:102,106,110,182,185) and S2 = H1 W2 (layer.py:102, gc2).  None
    where the kernel refuses the operands (GCNK_EUNSUP: rows of W1 / b1 / H1
    that are not 16-B aligned, or row strides that put W1, W2 or a 16-row tile
    of A-hat X past its 32-bit buffer offsets -- not reachable with the
    module's contiguous operands): the caller then takes the SpMM path."""
    W1 = _dense_f32(W1, "gc1 weight")
    W2 = _dense_f32(W2, "gc2 weight")
    _check_rng_base(rng_base, W1.device)
    M, F, P = d.AX.shape[0], W1.shape[1], W2.shape[1]
    if W1.shape[0] != d.K or W2.shape[0] != F:
        raise RuntimeError(f"dense_gc1 shape mismatch: A-hat X [{M} x {d.K}], W1 {tuple(W1.shape)}, "
                           f"W2 {tuple(W2.shape)}")
    H1 = torch.empty((M, F), dtype=torch.float32, device=W1.device) if store_h1 else None
    S2 = torch.empty((M, P), dtype=torch.float32, device=W1.device)
    if b1 is not None:
        b1 = b1.contiguous()
    if mask is not None:
        mask = mask.contiguous()
    with torch.cuda.device(W1.device):
        rc = _lib.load().gcnk_dense_gc1_f32(
            M, d.K, F, P, _ptr(d.AX), d.AX.stride(0), _ptr(W1), W1.stride(0), _ptr(b1), epilogue,
            _ptr(mask), mask.stride(0) if mask is not None else 0, float(scale),
            float(keep_prob), int(seed) & (2**64 - 1), int(offset) & (2**64 - 1), _ptr(rng_base),
            _ptr(W2), W2.stride(0), _ptr(H1), F, _ptr(S2), P, _stream(W1.device))
    if rc == _lib.EUNSUP:
        return None
    _lib.check(rc, "gcnk_dense_gc1_f32")
    return H1, S2


def default_split_k(M, N, K, trans=False):
    """K-slabs for a GEMM: only long reductions with a small output (H^T g,
    K = nodes) are split; short ones (H1 W2, K = 200) stay whole so the skinny
    kernel takes them.  ``trans``: an operand is transposed (the small-M
    kernel, which takes one 64-deep chunk per slab, is NN only)."""
    if M <= 64 and K >= 512 and N % 4 == 0 and not trans:
        # the small-M split-K kernel (csrc/gemm.hip): 64-deep k chunks
        return (K + 63) // 64
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    split_k = 1
    while K >= 1024 and split_k < 128 and tiles * split_k < 512 and K // (split_k * 2) >= 64:
        split_k *= 2
    return split_k


def gemm(A, B, transA=False, transB=False, bias=None, epilogue=_lib.GEMM_EPI_NONE, R=None, scale=1.0,
         split_k=None, out=None):
    """C = epi(op(A) @ op(B)) on fp32 MFMA.

    Replaces the dense ``th.spmm(H1, W2)`` of gc2 (reference layer.py:102,
    lowered to mm by ATen) and the dense autograd products."""
    A = _dense_f32(A, "A")
    B = _dense_f32(B, "B")
    M, K = (A.shape[1], A.shape[0]) if transA else (A.shape[0], A.shape[1])
    Kb, N = (B.shape[1], B.shape[0]) if transB else (B.shape[0], B.shape[1])
    if K != Kb:
        raise RuntimeError(f"gemm shape mismatch: op(A) {M}x{K} @ op(B) {Kb}x{N}")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=A.device)
    if split_k is None:
        split_k = default_split_k(M, N, K, trans=transA or transB)
    lib = _lib.load()
    wsb = lib.gcnk_gemm_workspace_bytes(M, N, K, split_k)
    ws = torch.empty((wsb + 3) // 4, dtype=torch.float32, device=A.device) if wsb > 0 else None
    if R is not None:
        R = _dense_f32(R, "R")
    with torch.cuda.device(A.device):
        rc = lib.gcnk_gemm_f32(int(transA), int(transB), M, N, K, _ptr(A), A.stride(0), _ptr(B), B.stride(0),
                               _ptr(out), out.stride(0), _ptr(bias.contiguous() if bias is not None else None),
                               epilogue, _ptr(R), R.stride(0) if R is not None else 0, float(scale), int(split_k),
                               _ptr(ws), wsb, _stream(A.device))
    _lib.check(rc, "gcnk_gemm_f32")
    return out


def colsum(X):
    """out[n] = sum_m X[m, n] — the bias gradient (autograd of layer.py:110)."""
    X = _dense_f32(X, "X")
    M, N = X.shape
    lib = _lib.load()
    wsb = lib.gcnk_colsum_workspace_bytes(M, N)
    ws = torch.empty(max((wsb + 3) // 4, 1), dtype=torch.float32, device=X.device)
    out = torch.empty(N, dtype=torch.float32, device=X.device)
    with torch.cuda.device(X.device):
        rc = lib.gcnk_colsum_f32(_ptr(X), X.stride(0), M, N, _ptr(out), _ptr(ws), wsb, _stream(X.device))
    _lib.check(rc, "gcnk_colsum_f32")
    return out


_BWD2_WS = {}


def _bwd2_workspace(M, N, P, dev):
    """gcnk_gcn_bwd2_f32's workspace for torch's current stream, allocated once
    and reused by every call of that shape on that stream (no allocation on
    the eager backward's path)."""
    key = (M, N, P, dev.index, torch.cuda.current_stream(dev).cuda_stream)
    hit = _BWD2_WS.get(key)
    if hit is None:
        wsb = int(_lib.load().gcnk_gcn_bwd2_workspace_bytes(M, N, P))
        if len(_BWD2_WS) >= 32:
            # (a workspace a captured graph launched with is never freed: the
            # graph replays into it)
            victim = next((k for k, v in _BWD2_WS.items() if not v[2]), None)
            if victim is not None:
                _BWD2_WS.pop(victim)
        hit = _BWD2_WS[key] = [wsb, torch.zeros((wsb + 3) // 4, dtype=torch.float32, device=dev), False]
    if torch.cuda.is_current_stream_capturing():
        hit[2] = True
    return hit[0], hit[1]


def gcn_bwd2(H1, gS2, W2, G=None, scale=1.0, want_gw=True, want_gb1=True):
    """The fused backward of gc2 and of gc1's ReLU + dropout (gcnk_gcn_bwd2_f32):
    returns (gZ1, gW2, gb1, gb2) with

        gZ1 = (H1 > 0) ? scale * (gS2 @ W2^T) : 0      (mm + dropout noise + threshold_backward)
        gW2 = H1^T @ gS2,  gb1 = colsum(gZ1),  gb2 = colsum(G) (None without G)

    (autograd of reference layer.py:182-188 through layer.py:102-110).  None
    when the shape is outside the fused kernel (more than 32 classes): the
    caller takes the gemm + colsum route."""
    H1 = _dense_f32(H1, "H1")
    gS2 = _dense_f32(gS2, "gS2")
    W2 = _dense_f32(W2, "W2")
    M, N = H1.shape
    P = W2.shape[1]
    if P > 32 or M == 0 or N == 0 or P == 0:
        return None
    if gS2.shape != (M, P) or W2.shape[0] != N:
        raise RuntimeError(f"gcn_bwd2 shape mismatch: H1 {tuple(H1.shape)}, gS2 {tuple(gS2.shape)}, "
                           f"W2 {tuple(W2.shape)}")
    if G is not None:
        G = _dense_f32(G, "G")
        if G.shape != (M, P):
            raise RuntimeError(f"gcn_bwd2 shape mismatch: G {tuple(G.shape)} vs {(M, P)}")
    dev = H1.device
    gZ1 = torch.empty((M, N), dtype=torch.float32, device=dev)
    gW2 = torch.empty((N, P), dtype=torch.float32, device=dev) if want_gw else None
    gb1 = torch.empty(N, dtype=torch.float32, device=dev) if want_gb1 else None
    gb2 = torch.empty(P, dtype=torch.float32, device=dev) if G is not None else None
    lib = _lib.load()
    wsb, ws = _bwd2_workspace(M, N, P, dev)
    with torch.cuda.device(dev):
        rc = lib.gcnk_gcn_bwd2_f32(_ptr(H1), H1.stride(0), _ptr(gS2), gS2.stride(0), _ptr(W2), W2.stride(0),
                                   _ptr(G), G.stride(0) if G is not None else 0, M, N, P, float(scale),
                                   _ptr(gZ1), gZ1.stride(0), _ptr(gW2), _ptr(gb1), _ptr(gb2), _ptr(ws), wsb,
                                   _stream(dev))
    _lib.check(rc, "gcnk_gcn_bwd2_f32")
    return gZ1, gW2, gb1, gb2


# ----------------------------------------------------------------------------------------
# Operand for the first product of a layer: sparse (CSR) or dense infeatn.

# A sparse infeatn at least this full (nnz / (rows x cols)) is multiplied as a
# dense matrix on the MFMA GEMM: a gensim-style 100-d X (50-70 % fill) would
# otherwise leave every 64-row block of the tile path split over two 64-column
# chunks and a slab reduce (20ng-shaped X W1: 71 us sparse, 19.7 us dense).
DENSE_OPERAND_FILL = 0.2
DENSE_OPERAND_MAX_BYTES = 1 << 30


def dense_copy(a):
    """The dense [M, K] fp32 copy of CSR ``a`` (gcnk_csr_to_dense), cached on it."""
    d = getattr(a, "_dense", None)
    if d is None:
        M, K = a.shape
        d = torch.empty((M, K), dtype=torch.float32, device=a.device)
        with torch.cuda.device(a.device):
            _lib.check(_lib.load().gcnk_csr_to_dense(_ptr(a.rowptr), _ptr(a.colind), _ptr(a.val), M, K, _ptr(d),
                                                     d.stride(0), _stream(a.device)), "gcnk_csr_to_dense")
        a._dense = d
    return d


class Operand:
    """``infeatn`` of GraphConvolution.forward: sparse -> CSR (or, when at least
    DENSE_OPERAND_FILL full, its cached dense copy), dense -> tensor."""

    __slots__ = ("csr", "dense")

    def __init__(self, x):
        if isinstance(x, CSR):
            self.csr, self.dense = x, None
        elif isinstance(x, torch.Tensor) and (x.is_sparse or x.layout == torch.sparse_csr):
            self.csr, self.dense = as_csr(x), None
        else:
            self.csr, self.dense = None, _dense_f32(x, "infeatn")
        if self.csr is not None:
            M, K = self.csr.shape
            if M * K > 0 and self.csr.nnz >= DENSE_OPERAND_FILL * M * K and 4 * M * K <= DENSE_OPERAND_MAX_BYTES:
                self.csr, self.dense = None, dense_copy(self.csr)

    @property
    def shape(self):
        return self.csr.shape if self.csr is not None else tuple(self.dense.shape)

    def times(self, W):
        """infeatn @ W  (layer.py:102)."""
        if self.csr is not None:
            return spmm(self.csr, W)
        return gemm(self.dense, W)

    def t_times(self, G):
        """infeatn^T @ G  (autograd of layer.py:102 w.r.t. W)."""
        if self.csr is not None:
            return spmm(self.csr.t(), G)
        return gemm(self.dense, G, transA=True)


class GraphConvFn(torch.autograd.Function):
    """out = A (X W) + b — one GraphConvolution (reference layer.py:84-112)."""

    @staticmethod
    def forward(ctx, W, b, x, xop, adj):
        support = xop.times(W)                                   # layer.py:102
        out = spmm(adj, support, bias=b,                         # layer.py:106,110
                   epilogue=_lib.EPI_BIAS if b is not None else _lib.EPI_NONE)
        ctx.xop, ctx.adj = xop, adj
        ctx.has_bias = b is not None
        ctx.save_for_backward(W)
        return out

    @staticmethod
    def backward(ctx, g):
        (W,) = ctx.saved_tensors
        g = g.contiguous()
        gW = gb = gx = None
        gS = spmm(ctx.adj.t(), g)                                # d/d support of A @ support
        if ctx.needs_input_grad[0]:
            gW = ctx.xop.t_times(gS)
        if ctx.has_bias and ctx.needs_input_grad[1]:
            gb = colsum(g)
        if ctx.xop.dense is not None and ctx.needs_input_grad[2]:
            gx = gemm(gS, W, transB=True)
        return gW, gb, gx, None, None


# (ABI 11 also had the factored forward's gW1 through the factor -- A_H^T gZ1,
# X_hubs^T on the short-K GEMM, U^T gZ1 on a one-pass small-M GEMM: 30.2 us in
# R8's replayed step against 22.8 for A-hat^T gZ1 + X^T gS1,
# profiles/r05_train_trace.json -- removed in ABI 12.)


# The whole forward from one C call (record.py, gcnk_gcn_forward_f32) wherever
# a record applies; GCNK_FORWARD_RECORD=0 issues it op by op (A/B timing).
USE_RECORD = os.environ.get("GCNK_FORWARD_RECORD", "1") != "0"


def record_forward(W1, b1, W2, b2, xop, adj, epi, mask, scale, keep, seed, offset, keep_h1, rng_base):
    """(out, H1) of GCN.forward (reference layer.py:164-190) through the
    cached launch record of (adj, X) -- or None where the forward is issued op
    by op (no record applies, or records are off)."""
    if not USE_RECORD:
        return None
    from . import record
    dev = W1.device
    F, P = W1.shape[1], W2.shape[1]
    if W2.shape[0] != F or W1.shape[0] != xop.shape[1] or adj.shape[1] != xop.shape[0] or adj.device != dev:
        raise RuntimeError(f"GCN forward shape mismatch: X {tuple(xop.shape)}, adj {tuple(adj.shape)}, "
                           f"W1 {tuple(W1.shape)}, W2 {tuple(W2.shape)}")
    if W1.dtype != torch.float32 or W2.dtype != torch.float32:
        raise RuntimeError("GCN weights must be float32 (the reference computes in fp32)")
    if not W1.is_contiguous():
        W1 = W1.contiguous()
    if not W2.is_contiguous():
        W2 = W2.contiguous()
    if b1 is not None and not b1.is_contiguous():
        b1 = b1.contiguous()
    if b2 is not None and not b2.is_contiguous():
        b2 = b2.contiguous()
    if mask is not None and not mask.is_contiguous():
        mask = mask.contiguous()
    if dev.index != torch.cuda.current_device():
        with torch.cuda.device(dev):
            return record_forward(W1, b1, W2, b2, xop, adj, epi, mask, scale, keep, seed, offset, keep_h1, rng_base)
    rec, stream = record.get(adj, xop, F, P, dev, train=bool(keep_h1))
    if rec is None:
        return None
    if rec.kind == record.DENSE_AX and not all(t is None or t.data_ptr() % 16 == 0 for t in (W1, b1)):
        return None   # (gcnk_dense_gc1_f32 takes 16-B aligned W1 / b1 rows: the per-op path falls back)
    return rec.run(W1, b1, W2, b2, epi, mask, float(scale), float(keep), int(seed), int(offset), rng_base,
                   keep_h1, stream)


def record_backward(ctx, g, W2, H1, need):
    """(gW1, gb1, gW2, gb2) of GCNFn.backward through the cached backward
    record of (adj, X) -- or None where it is issued op by op (records or the
    fused gcn_bwd2 off, more than 32 classes, or only gc2's grads wanted)."""
    P = W2.shape[1]
    if not (USE_RECORD and FUSE_BACKWARD) or P > 32 or not (need[0] or need[1]) or \
            g.dtype != torch.float32 or H1.stride(1) != 1 or not W2.is_contiguous() or g.shape != (H1.shape[0], P):
        return None
    from . import record
    dev = g.device
    if dev.index != torch.cuda.current_device():
        with torch.cuda.device(dev):
            return record_backward(ctx, g, W2, H1, need)
    rec, stream = record.get_backward(ctx.adj, ctx.xop, H1.shape[1], P, dev)
    return rec.run(g, H1, W2, ctx.scale, need[0], ctx.has_b1 and need[1], need[2], ctx.has_b2 and need[3], stream)


class GCNFn(torch.autograd.Function):
    """The two-layer forward of reference layer.py:164-190 as one fused graph:

        S1 = X W1                   spmm (sparse X) / gemm (dense X)      layer.py:102
        H1 = drop(relu(A S1 + b1))  spmm + fused epilogue                 layer.py:106,110,182,185
        S2 = H1 W2                  skinny MFMA gemm, or fused into that   layer.py:102 (gc2)
                                    epilogue (FUSE_PROJECTION; H1 then kept
                                    only when a backward needs it)
        Z  = A S2 + b2              spmm + bias                            layer.py:106,110 (gc2)

    Backward (trainer.py:361):
        gS2 = A^T g;
        gZ1 = (H1 > 0) ? (gS2 W2^T) * scale : 0   (== ATen's mul-by-noise then
              threshold_backward because H1 > 0 <=> kept and Z1 > 0),
        gW2 = H1^T gS2,  gb1 = colsum(gZ1),  gb2 = colsum(g)
              -- all four in one pass over H1 (gcn_bwd2; P > 32 classes: gemm
              with the MASK_POS epilogue, split-K gemm, colsum);
        gS1 = A^T gZ1;  gW1 = X^T gS1.
    """

    @staticmethod
    def forward(ctx, W1, b1, W2, b2, xop, adj, epi, mask, scale, keep, seed, offset, keep_h1=True, rng_base=None):
        res = record_forward(W1, b1, W2, b2, xop, adj, epi, mask, scale, keep, seed, offset, keep_h1, rng_base)
        if res is not None:
            out, H1 = res
            ctx.xop, ctx.adj, ctx.scale = xop, adj, float(scale)
            ctx.dax = ctx.fac = None
            ctx.has_b1, ctx.has_b2 = b1 is not None, b2 is not None
            ctx.save_for_backward(W2, H1)
            return out
        dax = dense_ax_for(adj, xop, W1.shape[1], W2.shape[1])
        fac = factor_for(adj, xop) if dax is None else None
        res = None
        if dax is not None:
            res = dense_gc1(dax, W1, b1, W2, epilogue=epi, mask=mask, scale=scale, keep_prob=keep, seed=seed,
                            offset=offset, rng_base=rng_base, store_h1=keep_h1)
        elif fac is not None:
            res = hubfactor_gc1(fac, W1, b1, W2, epilogue=epi, mask=mask, scale=scale, keep_prob=keep, seed=seed,
                                offset=offset, rng_base=rng_base, store_h1=keep_h1)
        out = None
        if res is not None:
            H1, S2 = res
        elif FUSE_PROJECTION and W2.shape[1] <= FUSE_MAX_P:
            S1 = xop.times(W1)
            H1, S2 = spmm_proj(adj, S1, W2, bias=b1, epilogue=epi, mask=mask, scale=scale, keep_prob=keep,
                               seed=seed, offset=offset, store_main=keep_h1, rng_base=rng_base)
        else:
            S1 = xop.times(W1)
            H1 = spmm(adj, S1, bias=b1, epilogue=epi, mask=mask, scale=scale, keep_prob=keep, seed=seed,
                      offset=offset, rng_base=rng_base)
            S2 = gemm(H1, W2)
        if out is None:
            out = spmm(adj, S2, bias=b2, epilogue=_lib.EPI_BIAS if b2 is not None else _lib.EPI_NONE)
        ctx.xop, ctx.adj, ctx.scale = xop, adj, float(scale)
        ctx.dax = dax
        ctx.fac = fac if (dax is None and res is not None) else None
        ctx.has_b1, ctx.has_b2 = b1 is not None, b2 is not None
        ctx.save_for_backward(W2, H1)
        return out

    @staticmethod
    def backward(ctx, g):
        W2, H1 = ctx.saved_tensors
        g = g.contiguous()
        need = ctx.needs_input_grad
        res = record_backward(ctx, g, W2, H1, need)
        if res is not None:
            return res + (None,) * 10
        gW1 = gb1 = gW2 = gb2 = None
        adjT = ctx.adj.t()
        gS2 = spmm(adjT, g)
        fused = gcn_bwd2(H1, gS2, W2, G=g if ctx.has_b2 and need[3] else None, scale=ctx.scale,
                         want_gw=need[2], want_gb1=ctx.has_b1 and need[1]) \
            if FUSE_BACKWARD and (need[0] or need[1]) else None
        if fused is not None:
            gZ1, gW2, gb1, gb2 = fused
        else:
            if ctx.has_b2 and need[3]:
                gb2 = colsum(g)
            if need[2]:
                gW2 = gemm(H1, gS2, transA=True)
            gZ1 = None
            if need[0] or need[1]:
                gZ1 = gemm(gS2, W2, transB=True, epilogue=_lib.GEMM_EPI_MASK_POS, R=H1, scale=ctx.scale)
                if ctx.has_b1 and need[1]:
                    gb1 = colsum(gZ1)
        if need[0]:
            if ctx.dax is not None:   # Z1 = (A-hat X) W1  =>  gW1 = (A-hat X)^T gZ1
                gW1 = gemm(ctx.dax.AX[:, :ctx.dax.K], gZ1, transA=True)
            else:
                gS1 = spmm(adjT, gZ1)
                gW1 = ctx.xop.t_times(gS1)
        return gW1, gb1, gW2, gb2, None, None, None, None, None, None, None, None, None, None
