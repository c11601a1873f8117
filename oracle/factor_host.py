"""ORACLE (test infrastructure only): host float64 restatement of the hub
factorisation of gc1 that factor.py builds on the device (csrc/factor_build.hip).

The reference's gc1 is ``th.spmm(adj, th.spmm(X, W1)) + b1`` (layer.py:102,
106,110) on the doc-topic graph of trainer.py:98-148 / utils.py:185-213.  With
hubs = A-hat's long rows (the topics) and light rows touching only hub columns
and themselves,

    A-hat X W1 = U W1[k0:k0+Kc] + A_H (X_hubs W1)

U [M x Kc] = (A-hat restricted to light columns) X[:, k0:k0+Kc] in float64 by
scipy's sparse product (per output element: A's row items in CSR order),
rounded to fp32 once; A_H as per-32-row-block records of the row order perm.
tests/test_factor.py checks these operands reproduce A-hat X W1 of the
reference, and tests/test_gpu_parity.py pins the device build to them bit for
bit.  No product code imports this module.
"""
import dataclasses

import numpy as np

MAX_HUBS = 128
MAX_KC = 128
ROWS_PER_BLOCK = 32
REC_HEAD = 68
REC_ROW = 36


@dataclasses.dataclass
class HostFactor:
    M: int
    H: int
    k0: int
    Kc: int
    nblk: int
    rec_words: int
    hubs: np.ndarray
    perm: np.ndarray
    U: np.ndarray
    rec: np.ndarray
    x_hub_rowptr: np.ndarray
    x_hub_colind: np.ndarray
    x_hub_val: np.ndarray


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
    """HostFactor for (adj, X) or None when the operands lack the structure.
    adj: an object with rowptr / colind / val / shape (torch tensors, any
    device); xop: .csr (same) or .dense, and .shape."""
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
    Xh = X[hubs].tocsr()
    Xh.sort_indices()
    return HostFactor(M=M, H=H, k0=k0, Kc=Kc, nblk=nblk, rec_words=rec_words, hubs=hubs.astype(np.int64),
                      perm=perm.astype(np.int64), U=U.astype(np.float32), rec=rec,
                      x_hub_rowptr=Xh.indptr.astype(np.int32), x_hub_colind=Xh.indices.astype(np.int32),
                      x_hub_val=Xh.data.astype(np.float32))
