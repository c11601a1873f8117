"""Device CSR operands for the SpMM kernels, built once per graph and cached.

The reference hands ``th.spmm`` torch sparse COO tensors every call:
  * A-hat from ``utils.sparse_mx_to_torch_sparse_tensor`` (utils.py:196-203):
    fp32 values, int64 indices, column-major order, uncoalesced;
  * X from ``trainer.py:226-238``: row-major COO.
ATen re-coalesces such tensors on every call.  Here the first forward
converts them once to an int32 CSR resident in HBM (plus, lazily, the
transposed CSR the autograd products need and the SpMM plan per column-width
class) and later calls hit the cache.

HBM layout of one CSR operand (M rows, K cols, nnz nonzeros):
  rowptr int32[M+1] | colind int32[nnz] | val fp32[nnz]
  plan   int32[...]  row units + dense tile blocks (include/gcnk.h),
                     one per (ipc, groups, dense threshold)
"""
import collections
import ctypes
import threading

import torch

from . import _lib

_INT32_MAX = 2**31 - 1


def _stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(t, what):
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        dev = getattr(t, "device", type(t))
        raise RuntimeError(
            f"{what} must be a tensor on a ROCm GPU (got {dev}); this framework runs the GCN hot path "
            "only through its HIP kernels — move the model and inputs with .to('cuda').")


DENSE_THRESHOLD = 0.25  # row blocks at least this dense (condensed) run on the MFMA tile path

class Plan:
    """A built SpMM plan: device buffer + the 16-word host header (gcnk.h).

    Plans with arrival counters (heavy rows of several segments, combined
    inside the launch) need a COUNTER REGION (gcnk_spmm_counter_bytes):
    zeroed once, then used by one stream's calls in order -- the kernels leave
    it zero for the next call, so it is never cleared again.  One region per stream for eager calls; calls
    captured into a hipGraph take one region per capturing stream (every
    graph captured there shares it: their replays must not run concurrently
    on two streams), handed out from SPARE_REGIONS regions zeroed when the
    plan is built, so a captured graph holds no memset node."""

    __slots__ = ("buf", "hdr", "_counters", "_spares", "_captured", "_lock")
    SPARE_REGIONS = 16   # pre-zeroed regions handed to capturing streams

    def __init__(self, buf, hdr):
        self.buf, self.hdr = buf, hdr
        self._counters = {}
        self._spares = None
        self._captured = {}
        self._lock = threading.Lock()

    @property
    def header(self):
        return list(self.hdr)

    def workspace_bytes(self, F):
        return int(_lib.load().gcnk_spmm_workspace_bytes(ctypes.cast(self.hdr, ctypes.c_void_p), int(F)))

    def counter_bytes(self):
        return int(_lib.load().gcnk_spmm_counter_bytes(ctypes.cast(self.hdr, ctypes.c_void_p)))

    def prime(self, device):
        """Zero SPARE_REGIONS counter regions now (eagerly, outside any capture)."""
        n = self.counter_bytes()
        if n <= 0 or self._spares is not None:
            return
        words = (n + 7) // 8 * 2   # whole uint64 words
        block = torch.zeros(self.SPARE_REGIONS * words, dtype=torch.int32, device=device)
        self._spares = list(block.split(words))

    def counters(self, device):
        """The counter region for a call on torch's current stream (None when the
        plan needs none); see the class docstring."""
        n = self.counter_bytes()
        if n <= 0:
            return None
        words = (n + 7) // 8 * 2
        key = torch.cuda.current_stream(device).cuda_stream
        if torch.cuda.is_current_stream_capturing():
            c = self._captured.get(key)
            if c is None:
                with self._lock:
                    c = self._captured.get(key)
                    if c is None:
                        if not self._spares:
                            raise RuntimeError(
                                f"SpMM plan: hipGraph captures on more than {self.SPARE_REGIONS} streams; "
                                "each capturing stream needs a pre-zeroed counter region (Plan.SPARE_REGIONS)")
                        c = self._captured[key] = self._spares.pop()
            return c
        c = self._counters.get(key)
        if c is None:
            with self._lock:
                c = self._counters.get(key)
                if c is None:
                    c = self._counters[key] = torch.zeros(words, dtype=torch.int32, device=device)
        return c


class CSR:
    """A sparse matrix in int32 CSR on one device, with cached schedules."""

    def __init__(self, rowptr, colind, val, shape):
        self.rowptr = rowptr.contiguous()
        self.colind = colind.contiguous()
        self.val = val.contiguous()
        self.shape = (int(shape[0]), int(shape[1]))
        self.nnz = int(self.colind.numel())
        self.device = self.rowptr.device
        self._plans = {}
        self._t = None
        self._lock = threading.Lock()

    def __repr__(self):
        return f"CSR(shape={self.shape}, nnz={self.nnz}, device={self.device})"

    # -- hybrid plan (gcnk_spmm_plan_build), one per (ipc, groups, dense threshold) -------
    def plan(self, ipc, groups, dense_threshold=DENSE_THRESHOLD):
        """Returns a Plan (device buffer + host header); built once per key (setup sync)."""
        key = (ipc, groups, float(dense_threshold))
        p = self._plans.get(key)
        if p is not None:
            return p
        with self._lock:
            p = self._plans.get(key)
            if p is not None:
                return p
            lib = _lib.load()
            M, K = self.shape
            with torch.cuda.device(self.device):
                s = _stream_ptr(self.device)
                nbytes = lib.gcnk_spmm_plan_bytes(self.rowptr.data_ptr(), self.colind.data_ptr(), M, K, self.nnz,
                                                  ipc, groups, float(dense_threshold), s)
                if nbytes < 0:
                    _lib.check(int(nbytes), "gcnk_spmm_plan_bytes")
                buf = torch.empty((nbytes + 3) // 4, dtype=torch.int32, device=self.device)
                _lib.check(lib.gcnk_spmm_plan_build(self.rowptr.data_ptr(), self.colind.data_ptr(),
                                                    self.val.data_ptr(), M, K, self.nnz, ipc, groups,
                                                    float(dense_threshold), buf.data_ptr(), nbytes, s),
                           "gcnk_spmm_plan_build")
                hdr = (ctypes.c_int32 * 16)()
                _lib.check(lib.gcnk_spmm_plan_query(buf.data_ptr(), ctypes.cast(hdr, ctypes.c_void_p), s),
                           "gcnk_spmm_plan_query")
                p = Plan(buf, hdr)
                p.prime(self.device)
            self._plans[key] = p
            return p

    # -- transpose (gcnk_csr_transpose), cached ---------------------------------------
    def t(self):
        if self._t is not None:
            return self._t
        with self._lock:
            if self._t is None:
                self._t = transpose(self)
                self._t._t = self
            return self._t


def transpose(a):
    lib = _lib.load()
    M, K = a.shape
    dev = a.device
    rp_t = torch.empty(K + 1, dtype=torch.int32, device=dev)
    ci_t = torch.empty(a.nnz, dtype=torch.int32, device=dev)
    v_t = torch.empty(a.nnz, dtype=torch.float32, device=dev)
    wsb = lib.gcnk_csr_transpose_workspace_bytes(M, K, a.nnz)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        _lib.check(lib.gcnk_csr_transpose(a.rowptr.data_ptr(), a.colind.data_ptr(), a.val.data_ptr(), M, K, a.nnz,
                                          rp_t.data_ptr(), ci_t.data_ptr(), v_t.data_ptr(), ws.data_ptr(), wsb,
                                          _stream_ptr(dev)), "gcnk_csr_transpose")
    return CSR(rp_t, ci_t, v_t, (K, M))


def _check_int32(M, K, nnz):
    if M > _INT32_MAX or K > _INT32_MAX or nnz > _INT32_MAX or M + nnz >= _INT32_MAX:
        raise RuntimeError(f"sparse operand too large for int32 CSR (M={M}, K={K}, nnz={nnz})")


def from_torch(t):
    """Torch sparse tensor (COO in any order / uncoalesced, or CSR) on a GPU -> CSR.

    Duplicates in an uncoalesced COO are summed (what th.spmm computes)."""
    require_device(t, "sparse operand")
    if t.dim() != 2:
        raise RuntimeError(f"sparse operand must be 2-D, got {t.dim()}-D")
    M, K = t.shape
    if t.layout == torch.sparse_csr:
        rowptr = t.crow_indices().to(torch.int32)
        colind = t.col_indices().to(torch.int32)
        val = t.values().to(torch.float32)
        _check_int32(M, K, colind.numel())
        return CSR(rowptr, colind, val, (M, K))
    if t.layout != torch.sparse_coo:
        raise RuntimeError(f"unsupported sparse layout {t.layout}")
    # gcnk_coo_to_csr: stable sort of (row, col), duplicates summed in input
    # order (ATen's coalesce arithmetic), row pointers -- one pass on the device
    idx = t._indices()
    vals = t._values()
    if vals.dtype != torch.float32:
        vals = vals.to(torch.float32)
    nnz_in = vals.numel()
    _check_int32(M, K, nnz_in)
    rows, cols, vals = idx[0].contiguous(), idx[1].contiguous(), vals.contiguous()
    dev = t.device
    rowptr = torch.empty(M + 1, dtype=torch.int32, device=dev)
    colind = torch.empty(max(nnz_in, 1), dtype=torch.int32, device=dev)
    val = torch.empty(max(nnz_in, 1), dtype=torch.float32, device=dev)
    lib = _lib.load()
    wsb = int(lib.gcnk_coo_to_csr_workspace_bytes(nnz_in, M, K))
    if wsb < 0:
        _lib.check(wsb, "gcnk_coo_to_csr_workspace_bytes")
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        _lib.check(lib.gcnk_coo_to_csr(rows.data_ptr(), cols.data_ptr(), vals.data_ptr(), nnz_in, M, K,
                                       rowptr.data_ptr(), colind.data_ptr(), val.data_ptr(), ws.data_ptr(), wsb,
                                       _stream_ptr(dev)), "gcnk_coo_to_csr")
    nnz = int(rowptr[M])   # one-time setup sync
    if nnz < 0:
        raise RuntimeError(f"sparse COO operand has an index outside its shape {tuple(t.shape)}")
    return CSR(rowptr, colind[:nnz], val[:nnz], (M, K))


def from_arrays(rowptr, colind, val, shape, device):
    """Build a CSR from host/numpy arrays (already sorted CSR)."""
    rp = torch.as_tensor(rowptr).to(device=device, dtype=torch.int32)
    ci = torch.as_tensor(colind).to(device=device, dtype=torch.int32)
    v = torch.as_tensor(val).to(device=device, dtype=torch.float32)
    _check_int32(shape[0], shape[1], ci.numel())
    return CSR(rp, ci, v, shape)


def preprocess_adj(adj):
    """Â = D^-1/2 (A + I) D^-1/2 on the device (gcnk_sym_normalize): the
    reference's ``utils.preprocess_adj(adj, is_sparse=True)`` (utils.py:185-213)
    for an adjacency that is already a GPU tensor, with the reference's
    float64 arithmetic and one rounding to fp32, so the values are bit-for-bit
    what the host path produces.  ``adj``: symmetric A as a torch sparse
    tensor (any COO order, duplicates summed) or a CSR on the GPU.  Returns the
    CSR of Â (usable directly as ``adj`` of GCN.forward).

    The kernel needs sorted, duplicate-free columns per row and a symmetric A
    (the reference evaluates (A D)^T D, which is D A D only when A = A^T; its
    trainer builds max(A, A^T), trainer.py:148).  Both are checked here (one
    setup-time sync) and violations raise instead of giving wrong values."""
    a = adj if isinstance(adj, CSR) else from_torch(adj)
    n, k = a.shape
    if n != k:
        raise RuntimeError(f"preprocess_adj: adjacency must be square, got {a.shape}")
    _check_sorted_symmetric(a)
    lib = _lib.load()
    dev = a.device
    rp = torch.empty(n + 1, dtype=torch.int32, device=dev)
    ci = torch.empty(a.nnz + n, dtype=torch.int32, device=dev)
    v = torch.empty(a.nnz + n, dtype=torch.float32, device=dev)
    wsb = int(lib.gcnk_sym_normalize_workspace_bytes(n, a.nnz))
    if wsb < 0:
        _lib.check(wsb, "gcnk_sym_normalize_workspace_bytes")
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        _lib.check(lib.gcnk_sym_normalize(a.rowptr.data_ptr(), a.colind.data_ptr(), a.val.data_ptr(), n, a.nnz,
                                          rp.data_ptr(), ci.data_ptr(), v.data_ptr(), ws.data_ptr(), wsb,
                                          _stream_ptr(dev)), "gcnk_sym_normalize")
    nnz = int(rp[n])   # one-time setup sync
    return CSR(rp, ci[:nnz], v[:nnz], (n, n))


def _check_sorted_symmetric(a):
    n = a.shape[0]
    if a.nnz == 0:
        return
    rows = torch.repeat_interleave(torch.arange(n, device=a.device, dtype=torch.int32), a.rowptr.diff())
    unsorted = bool(((a.colind[1:] <= a.colind[:-1]) & (rows[1:] == rows[:-1])).any())
    if unsorted:
        raise RuntimeError("preprocess_adj: CSR columns must be sorted and duplicate-free within each row "
                           "(build it with from_torch, which coalesces)")
    t = transpose(a)
    if not (torch.equal(t.rowptr, a.rowptr) and torch.equal(t.colind, a.colind) and torch.equal(t.val, a.val)):
        raise RuntimeError("preprocess_adj: the adjacency is not symmetric; the reference's (A D)^T D "
                           "(utils.py:212) is D^-1/2 A D^-1/2 only for A = A^T -- symmetrise it first "
                           "(max(A, A^T) as trainer.py:148 does)")


class _Cache:
    """LRU of torch sparse tensor -> CSR, keyed by storage identity + version.

    The entry keeps a reference to the source tensor so its storage cannot be
    recycled (which would make a stale key collide)."""

    def __init__(self, capacity=16):
        self.capacity = capacity
        self._d = collections.OrderedDict()
        self._lock = threading.Lock()

    @staticmethod
    def key(t):
        if t.layout == torch.sparse_csr:
            parts = (t.crow_indices(), t.col_indices(), t.values())
        else:
            parts = (t._indices(), t._values())
        return (t.layout, tuple(t.shape), t.device.index,
                tuple(p.data_ptr() for p in parts), tuple(p._version for p in parts))

    def get(self, t):
        k = self.key(t)
        with self._lock:
            hit = self._d.get(k)
            if hit is not None:
                self._d.move_to_end(k)
                return hit[1]
        csr = from_torch(t)
        with self._lock:
            self._d[k] = (t, csr)
            self._d.move_to_end(k)
            while len(self._d) > self.capacity:
                self._d.popitem(last=False)
        return csr

    def clear(self):
        with self._lock:
            self._d.clear()


CACHE = _Cache()


def as_csr(t):
    """CSR view of a torch sparse tensor (cached) or pass-through of a CSR."""
    if isinstance(t, CSR):
        return t
    if not isinstance(t, torch.Tensor) or not t.is_sparse and t.layout != torch.sparse_csr:
        raise RuntimeError("expected a torch sparse tensor or a CSR")
    return CACHE.get(t)
