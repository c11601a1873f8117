"""Drop-in ``GraphConvolution`` / ``GCN`` modules running on the gfx950 kernels.

Mirrors the reference's module interface (layer.py:25-190): constructor
arguments, Parameter shapes (weight stored [in, out], not nn.Linear's
[out, in]), ``state_dict`` keys (gc1.weight, gc1.bias, gc2.weight, gc2.bias),
initialisation RNG order and ``__repr__`` — so ``trainer.py`` can pass
``model = GCN`` (trainer.py:432) and instantiate it with
``nfeat/nhid/nclass/dropout`` kwargs (trainer.py:300-303) unchanged.

Differences by design:
  * ``forward`` runs only on ROCm tensors (no CPU fallback).  Inputs may be
    torch sparse COO (any order, uncoalesced — as utils.py:196-203 and
    trainer.py:226-238 produce them), torch sparse CSR, or dense.
  * The sparse operands are converted once to device CSR and cached.
  * ``GCN.forward`` runs the two layers as one fused autograd graph
    (ops.GCNFn): bias, ReLU and dropout live in the SpMM epilogue.
  * Dropout masks: ``dropout_rng="cpu"`` (default) draws them exactly as the
    reference's CPU ``th.dropout`` does — ``bernoulli_(1-p)`` on a float32
    CPU tensor from torch's default generator — so a seeded run consumes the
    same random stream as the reference and trains on identical masks;
    ``dropout_rng="device"`` generates them inside the kernel (counter-based
    hash), with no host work and no mask traffic.  The hash offset lives on
    the device (``_rng_base``, advanced by the forward itself), so a training
    step captured in a hipGraph draws a fresh mask on every replay.
"""
import ctypes
import math
import os
import threading

import numpy as np
import torch
from torch.nn import Module, Parameter

from . import _lib
from . import ops
from .ops import GCNFn, GraphConvFn, Operand
from .sparse import as_csr


_MT_STATE_BYTES = 5056   # torch's CPU generator state tensor (CPUGeneratorImplState)
_mt_checked = None


def _mt_fields(b):
    """Views of the MT19937 fields in torch's CPU generator state bytes:
    left (int32 @ 8), next (uint64 @ 16), state words (624 x uint64 @ 24)."""
    return b[8:12].view(np.int32), b[16:24].view(np.int64), b[24:24 + 624 * 8].view(np.uint64)


def _mt_draw(b, n, p, out):
    left, nxt, words = _mt_fields(b)
    st32 = np.ascontiguousarray(words, dtype=np.uint32)
    lf = np.ascontiguousarray(left.copy())
    nx = np.ascontiguousarray(nxt.copy())
    rc = _lib.load().gcnk_bernoulli_mt19937(st32.ctypes.data, lf.ctypes.data, nx.ctypes.data, int(n), float(p),
                                            out.ctypes.data, int(min(16, os.cpu_count() or 1)))
    _lib.check(rc, "gcnk_bernoulli_mt19937")
    words[:] = st32
    left[:] = lf
    nxt[:] = nx


def _mt_self_check():
    """The native draw must equal torch's own bernoulli_ (masks and the state
    it leaves) on this torch build; checked once on a private generator."""
    g = torch.Generator().manual_seed(20260501)
    g.set_state(g.get_state())
    st = g.get_state()
    if st.numel() != _MT_STATE_BYTES:
        return False
    for n, p in ((1000, 0.5), (1300, 0.37)):
        st = g.get_state()
        ref = torch.empty(n, dtype=torch.float32).bernoulli_(p, generator=g).numpy().astype(np.uint8)
        want = g.get_state().numpy()
        b = st.numpy().copy()
        got = np.empty(n, np.uint8)
        _mt_draw(b, n, p, got)
        if not (np.array_equal(got, ref) and np.array_equal(b, want)):
            return False
    return True


class _Speculation:
    """The next mask of the same shape, drawn on a native worker thread
    (gcnk_bernoulli_mt19937_start) from the generator state the current draw
    leaves, while the GPU runs the step.  Owns the buffers the worker writes
    until wait() has joined it."""

    __slots__ = ("key", "before", "after", "out", "_st32", "_lf", "_nx", "_job")

    def __init__(self, key, before, out):
        self.key, self.before, self.out = key, before, out
        self.after = before.copy()
        left, nxt, words = _mt_fields(self.after)
        self._st32 = np.ascontiguousarray(words, dtype=np.uint32)
        self._lf = left.copy()
        self._nx = nxt.copy()
        job = ctypes.c_void_p()
        _lib.check(_lib.load().gcnk_bernoulli_mt19937_start(
            self._st32.ctypes.data, self._lf.ctypes.data, self._nx.ctypes.data, int(out.numel()), float(key[1]),
            out.data_ptr(), ctypes.byref(job)), "gcnk_bernoulli_mt19937_start")
        self._job = job

    def wait(self):
        if self._job is None:
            return
        _lib.check(_lib.load().gcnk_bernoulli_mt19937_wait(self._job), "gcnk_bernoulli_mt19937_wait")
        self._job = None
        left, nxt, words = _mt_fields(self.after)
        words[:] = self._st32
        left[:] = self._lf
        nxt[:] = self._nx

    def __del__(self):
        try:
            self.wait()
        except Exception:
            pass


_spec = None
_spec_lock = threading.Lock()
_draw_lock = threading.RLock()
SPECULATE_MASKS = True


def host_keep_mask(shape, p):
    """uint8 keep-mask (1 = kept) of ``torch.empty(shape).bernoulli_(p)`` drawn
    from torch's default CPU generator -- the draw of the reference's CPU
    th.dropout (layer.py:185), bit for bit, with the generator left where that
    call leaves it -- through the native MT19937 restatement
    (gcnk_bernoulli_mt19937, ~10x faster than torch's serial loop).

    A training loop draws one mask per step and nothing else from the CPU
    generator in between, so after each draw the next one (same shape and p)
    is drawn speculatively on a worker thread from the state this draw leaves;
    the next call uses it only if the generator is still exactly in that state
    (anything else that drew, or a reseed, discards it), so the stream is
    unchanged either way.  Falls back to torch's own bernoulli_ if this torch
    build's generator state does not match the layout the restatement was
    checked against."""
    global _mt_checked
    if _mt_checked is None:
        _mt_checked = _mt_self_check()
    n = 1
    for d in shape:
        n *= int(d)
    pinned = torch.cuda.is_available()
    if not _mt_checked:
        out = torch.empty(shape, dtype=torch.uint8, pin_memory=pinned)
        out.copy_(torch.empty(shape, dtype=torch.float32).bernoulli_(p))
        return out
    # get_state -> draw -> set_state as one step: two threads drawing masks (or
    # a thread drawing from the CPU generator meanwhile, through this module)
    # must not both start from one state and lose an advance
    with _draw_lock:
        return _host_keep_mask_locked(shape, p, n, pinned)


def _host_keep_mask_locked(shape, p, n, pinned):
    global _spec
    g = torch.default_generator
    b = g.get_state().numpy().copy()
    key = (tuple(int(d) for d in shape), float(p))
    with _spec_lock:
        spec, _spec = _spec, None
    out = None
    if spec is not None:
        spec.wait()
        if spec.key == key and np.array_equal(spec.before, b):
            out, b = spec.out, spec.after
    if out is None:
        out = torch.empty(shape, dtype=torch.uint8, pin_memory=pinned)
        _mt_draw(b, n, p, out.numpy().reshape(-1))
    g.set_state(torch.from_numpy(b))
    if SPECULATE_MASKS:
        nxt = _Speculation(key, b.copy(), torch.empty(shape, dtype=torch.uint8, pin_memory=pinned))
        with _spec_lock:
            _spec = nxt
    return out


def _aliases(t):
    """The tensors whose version counters track in-place changes of t's data."""
    if isinstance(t, torch.Tensor):
        if t.layout == torch.sparse_coo:
            return (t._indices(), t._values())
        if t.layout == torch.sparse_csr:
            return (t.crow_indices(), t.col_indices(), t.values())
        return (t,)
    return ()


def _vkey(t, aliases):
    return (getattr(t, "_version", None),) + tuple(p._version for p in aliases)


class GraphConvolution(Module):
    """out = adj @ (infeatn @ weight) + bias   (reference layer.py:25-123)."""

    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = Parameter(torch.empty(in_features, out_features, dtype=torch.float32))
        if bias:
            self.bias = Parameter(torch.empty(out_features, dtype=torch.float32))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        # U(-1/sqrt(out), 1/sqrt(out)); weight first, then bias (layer.py:75-82) —
        # the same draws from the same generator as the reference.
        bound = 1.0 / math.sqrt(self.weight.size(1))
        with torch.no_grad():
            self.weight.uniform_(-bound, bound)
            if self.bias is not None:
                self.bias.uniform_(-bound, bound)

    def forward(self, infeatn, adj):
        xop = Operand(infeatn)
        a = as_csr(adj)
        x_dense = xop.dense if xop.dense is not None else None
        return GraphConvFn.apply(self.weight, self.bias, x_dense, xop, a)

    def __repr__(self):
        return f"{type(self).__name__} ({self.in_features} -> {self.out_features})"


class GCN(Module):
    """Two-layer GCN: gc2(dropout(relu(gc1(x, adj))), adj)  (reference layer.py:126-190)."""

    def __init__(self, nfeat, nhid, nclass, dropout, dropout_rng="cpu"):
        super().__init__()
        self.gc1 = GraphConvolution(nfeat, nhid)
        self.gc2 = GraphConvolution(nhid, nclass)
        self.dropout = dropout
        if dropout_rng not in ("cpu", "device"):
            raise ValueError("dropout_rng must be 'cpu' or 'device'")
        self.dropout_rng = dropout_rng
        # hash-dropout stream position, read and advanced on the device (not in state_dict)
        self.register_buffer("_rng_base", torch.zeros(1, dtype=torch.int64), persistent=False)
        self._memo = None   # (x, adj, version keys, Operand, CSR) of the last call

    def _dropout_args(self, nrows, device):
        """Epilogue code and mask/scale for layer.py:185 (ATen dropout semantics)."""
        p = float(self.dropout)
        if not self.training or p == 0.0:   # ATen returns the input untouched (no RNG draw)
            return _lib.EPI_BIAS_RELU, None, 1.0, 1.0, 0, 0
        nhid = self.gc1.out_features
        if p >= 1.0:                         # ATen: input * 0
            return _lib.EPI_BIAS_RELU_DROP, torch.zeros((nrows, nhid), dtype=torch.uint8, device=device), \
                0.0, 0.0, 0, 0
        # noise = bernoulli(1-p) / (1-p) with the division done in float32 (ATen)
        scale = float(torch.ones((), dtype=torch.float32).div_(1.0 - p))
        if self.dropout_rng == "cpu":
            mask = host_keep_mask((nrows, nhid), 1.0 - p).to(device, non_blocking=True)
            return _lib.EPI_BIAS_RELU_DROP, mask, scale, 1.0 - p, 0, 0
        seed = int(torch.initial_seed()) & (2**64 - 1)
        return _lib.EPI_BIAS_RELU_HASH, None, scale, 1.0 - p, seed, 0

    def _operands(self, x, adj):
        """(Operand of x, CSR of adj), memoised for the inputs of the previous
        call: the trainer passes the same two tensors every epoch
        (trainer.py:357,382), and re-deriving the cache keys cost ~10 us."""
        m = self._memo
        if m is not None and m[0] is x and m[1] is adj and m[2] == _vkey(x, m[5]) and m[3] == _vkey(adj, m[6]):
            return m[4], m[7]
        a = as_csr(adj)
        xop = Operand(x)
        xa, aa = _aliases(x), _aliases(adj)
        self._memo = (x, adj, _vkey(x, xa), _vkey(adj, aa), xop, xa, aa, a)
        return xop, a

    def forward(self, x, adj):
        xop, a = self._operands(x, adj)
        epi, mask, scale, keep, seed, offset = self._dropout_args(a.shape[0], a.device)
        W1, b1, W2, b2 = self.gc1.weight, self.gc1.bias, self.gc2.weight, self.gc2.bias
        # H1 is needed only by a backward pass; inference never writes it to HBM
        keep_h1 = torch.is_grad_enabled() and (W1.requires_grad or W2.requires_grad or
                                               (b1 is not None and b1.requires_grad) or
                                               (b2 is not None and b2.requires_grad))
        hashed = epi == _lib.EPI_BIAS_RELU_HASH
        if hashed and self._rng_base.device != a.device:
            raise RuntimeError(f"GCN buffers are on {self._rng_base.device}, operands on {a.device}: call .to()")
        rng = self._rng_base if hashed else None
        out = None
        if not keep_h1:   # inference (trainer.py:382 under no_grad): no autograd node, one C call
            res = ops.record_forward(W1, b1, W2, b2, xop, a, epi, mask, scale, keep, seed, offset, False, rng)
            out = res[0] if res is not None else None
        if out is None:
            out = GCNFn.apply(W1, b1, W2, b2, xop, a, epi, mask, scale, keep, seed, offset, keep_h1, rng)
        if hashed:   # the next call (or graph replay) draws the next rows*nhid hash positions
            self._rng_base.add_(a.shape[0] * self.gc1.out_features)
        return out
