"""Hub factorisation of the first GCN layer (csrc/factor.hip).

The reference's gc1 computes ``th.spmm(adj, th.spmm(X, W1)) + b1``
(layer.py:102,106,110).  On its doc-topic graph (trainer.py:98-148,
utils.py:185-213) A-hat's rows split into a few hub rows (the topics) and
light rows (the documents) whose nonzeros are hub columns plus their own
diagonal, and X's document rows are supported on a small column range (the
topic-weight columns, trainer.py:226-238).  Then

    A X W1 = U W1[k0:k0+Kc] + A_H (X_hubs W1)

with U [M x Kc] dense (rows in the block order ``perm``) -- row d (light): A_dd X[d, Kc]; row t (hub):
sum over light d of A_td X[d, Kc] -- and A_H = A-hat restricted to hub columns.
U and A_H depend only on (A-hat, X), so they are built here ONCE per operand
pair (host, float64, rounded to fp32 once) and cached on the adjacency; every
forward then runs X_hubs W1 (the tile GEMM over X's dense hub rows) and one
launch of gcnk_hubfactor_gc1_f32 (U W1[Kc] on MFMA + A_H S_T + bias + ReLU +
dropout + the gc2 projection H1 W2), and the hub rows' 600-term gather sums
of the SpMM never run.  The association differs from A (X W1) only in fp32
rounding (checked against the reference's goldens to 1e-4, tests/).
"""
import os
import threading

import numpy as np
import torch

from .sparse import from_arrays

MAX_HUBS = 128    # hub rows staged in LDS (S_T [hubs x F]; the kernel checks the LDS budget)
# X[hubs] W1 through the SpMM tile plan on their CSR ("spmm", default) or the
# split-K MFMA GEMM on a dense copy ("gemm": R8 9.5 + 4.9 us against the tile
# plan's 7.1 + 4.9, profiles/r03_factor.md)
XHUB = os.environ.get("GCNK_FACTOR_XHUB", "spmm")
MAX_KC = 128      # X's light-row column range (U's width)
ROWS_PER_BLOCK = 32   # csrc/factor.hip kRB
# record words before the items: 33 row offsets | 3 pad | 32 row ids (-1 past
# M) -- csrc/factor.hip kRecHead.  A block's rows are a slice of the row order
# `perm` (hub rows spread evenly between the light rows, so no block carries
# more than one or two hub rows' long item lists: the item loop is LDS-bound per
# workgroup, and R8's contiguous topic rows made three blocks the kernel's tail).
REC_HEAD = 68
REC_ROW = 36

_lock = threading.Lock()


class HubFactor:
    """The (A-hat, X)-fixed operands of the factored gc1, resident on the device."""

    __slots__ = ("M", "H", "hubs", "k0", "Kc", "U", "perm", "rec", "rec_words", "nblk", "x_hub", "x_hub_dense",
                 "_src")

    def hub_times(self, W):
        """S_T = X[hubs] @ W  (the hub rows of reference layer.py:102)."""
        from .ops import gemm, spmm
        if self.x_hub is not None and (XHUB != "gemm" or self.x_hub_dense is None):
            return spmm(self.x_hub, W)
        return gemm(self.x_hub_dense, W)


def _hub_rows(rp, ci, M):
    """Hub rows of A-hat (degree >= max(64, 8 x mean), at most MAX_HUBS) and
    whether every other row references only hub columns and itself."""
    deg = np.diff(rp)
    nnz = int(rp[-1])
    hmin = max(64, 8 * ((nnz + M - 1) // M))
    hubs = np.flatnonzero(deg >= hmin)
    if len(hubs) == 0 or len(hubs) > MAX_HUBS or len(hubs) >= M:
        return None
    is_hub = np.zeros(M, bool)
    is_hub[hubs] = True
    rows = np.repeat(np.arange(M), deg)
    bad = ~is_hub[rows] & ~is_hub[ci] & (ci != rows)
    if bad.any():
        return None
    return hubs, is_hub, rows


def build(adj, xop):
    """HubFactor for (adj, X) or None when the operands lack the structure."""
    import scipy.sparse as sp
    M, K = adj.shape
    if M != K or xop.shape[0] != M:
        return None
    rp = adj.rowptr.cpu().numpy().astype(np.int64)
    ci = adj.colind.cpu().numpy().astype(np.int64)
    v = adj.val.cpu().numpy().astype(np.float64)
    hr = _hub_rows(rp, ci, M)
    if hr is None:
        return None
    hubs, is_hub, rows = hr
    H = len(hubs)
    light = ~is_hub
    # X restricted to the light rows: its column range [k0, k0 + Kc)
    if xop.csr is not None:
        x = xop.csr
        xrp = x.rowptr.cpu().numpy().astype(np.int64)
        xci = x.colind.cpu().numpy().astype(np.int64)
        xv = x.val.cpu().numpy().astype(np.float64)
        X = sp.csr_matrix((xv, xci, xrp), shape=x.shape)
    else:
        X = sp.csr_matrix(xop.dense.cpu().numpy().astype(np.float64))
    XL = sp.diags(light.astype(np.float64)) @ X       # hub rows zeroed
    XL.eliminate_zeros()
    if XL.nnz:
        k0, k1 = int(XL.indices.min()), int(XL.indices.max()) + 1
    else:
        k0, k1 = 0, 1
    Kc = k1 - k0
    if Kc > MAX_KC:
        return None
    Kcp = (Kc + 3) // 4 * 4
    Xr = XL[:, k0:k1]
    A = sp.csr_matrix((v, ci, rp), shape=(M, M))
    diag = A.diagonal()
    Uo = np.zeros((M, Kcp), np.float64)
    Uo[light, :Kc] = (sp.diags(diag[light]) @ Xr[light]).toarray()
    Uo[hubs, :Kc] = (A[hubs] @ Xr).toarray()          # Xr's hub rows are zero: light columns only
    # row order: light rows in order, hub j placed at position ~ (j + 1/2) M / H
    lights = np.flatnonzero(light)
    pos = ((np.arange(H) + 0.5) * M / H).astype(np.int64)
    perm = np.insert(lights, np.minimum(pos - np.arange(H), len(lights)), hubs)
    assert len(perm) == M and np.array_equal(np.sort(perm), np.arange(M))
    U = Uo[perm]
    # A_H: every row's hub-column nonzeros, as per-32-row-block records (row order perm)
    hub_index = np.full(M, -1, np.int64)
    hub_index[hubs] = np.arange(H)
    mh = is_hub[ci]
    counts = np.bincount(rows[mh], minlength=M)                     # hub items per original row
    hstart = np.concatenate([[0], np.cumsum(counts)])
    hcols, hvals = hub_index[ci[mh]], v[mh].astype(np.float32)      # CSR order within a row
    nblk = (M + ROWS_PER_BLOCK - 1) // ROWS_PER_BLOCK
    pcounts = counts[perm]
    pstart = np.concatenate([[0], np.cumsum(pcounts)])
    rec_words = 0
    for b in range(nblk):
        r0, r1 = b * ROWS_PER_BLOCK, min(M, (b + 1) * ROWS_PER_BLOCK)
        rec_words = max(rec_words, REC_HEAD + 2 * int(pstart[r1] - pstart[r0]))
    rec_words = (rec_words + 3) // 4 * 4
    rec = np.zeros((nblk, rec_words), np.int32)
    for b in range(nblk):
        r0, r1 = b * ROWS_PER_BLOCK, min(M, (b + 1) * ROWS_PER_BLOCK)
        off = pstart[r0:r1 + 1] - pstart[r0]
        rec[b, :len(off)] = off
        rec[b, len(off):ROWS_PER_BLOCK + 1] = off[-1]
        rec[b, REC_ROW:REC_ROW + ROWS_PER_BLOCK] = -1
        rec[b, REC_ROW:REC_ROW + (r1 - r0)] = perm[r0:r1]
        items = np.concatenate([np.arange(hstart[r], hstart[r + 1]) for r in perm[r0:r1]]).astype(np.int64)
        rec[b, REC_HEAD:REC_HEAD + 2 * len(items):2] = hcols[items]
        rec[b, REC_HEAD + 1:REC_HEAD + 2 * len(items):2] = hvals[items].view(np.int32)
    dev = adj.device
    f = HubFactor()
    f.nblk = nblk
    f.M, f.H, f.k0, f.Kc = M, H, k0, Kc
    f.hubs = torch.from_numpy(hubs.astype(np.int64)).to(dev)
    f.perm = torch.from_numpy(perm.astype(np.int64))            # host: tests and tools
    f.U = torch.from_numpy(U.astype(np.float32)).to(dev)
    f.rec = torch.from_numpy(rec).to(dev)
    f.rec_words = rec_words
    Xh = X[hubs].tocsr()
    Xh.sort_indices()
    if xop.csr is not None:
        f.x_hub = from_arrays(Xh.indptr.astype(np.int32), Xh.indices.astype(np.int32), Xh.data.astype(np.float32),
                              (H, X.shape[1]), dev)
        f.x_hub_dense = torch.from_numpy(Xh.toarray().astype(np.float32)).to(dev) \
            if XHUB == "gemm" and H * X.shape[1] * 4 <= 64 << 20 else None
    else:
        f.x_hub = None
        f.x_hub_dense = xop.dense.index_select(0, f.hubs).contiguous()
    return f


def get(adj, xop):
    """The cached HubFactor of (adj, X), built on first use; None when the
    operands do not factor (the caller runs the generic SpMM path)."""
    src = xop.csr if xop.csr is not None else xop.dense
    key = (id(src), src.data_ptr() if isinstance(src, torch.Tensor) else src.rowptr.data_ptr(),
           src._version if isinstance(src, torch.Tensor) else src.val._version)
    cache = getattr(adj, "_factors", None)
    if cache is None:
        with _lock:
            cache = getattr(adj, "_factors", None)
            if cache is None:
                cache = adj._factors = {}
    hit = cache.get(key)
    if hit is not None:
        return hit[1]
    with _lock:
        hit = cache.get(key)
        if hit is not None:
            return hit[1]
        f = build(adj, xop)
        if f is not None:
            f._src = src
        while len(cache) >= 4:
            cache.pop(next(iter(cache)))
        cache[key] = (src, f)   # the entry holds the operand: its id cannot be recycled while cached
        return f
