"""Inputs for the hot path: the R8 fixture and seeded synthetic graphs.

All loaders return tensors laid out exactly as the reference hands them to
``th.spmm`` (host memory; callers move them to the GPU):
  * ``adj``: torch sparse COO fp32, int64 indices, uncoalesced, in the order
    utils.sparse_mx_to_torch_sparse_tensor produces (utils.py:196-203);
  * ``features``: torch sparse COO fp32 in row-major nonzero order
    (trainer.py:226-238).

Synthetic generators (own code, seeded; BASELINE.json configs 3-5, SURVEY.md
§8(d)) stand in for corpora that are absent here.
"""
import numpy as np
import torch


def _coo(rows, cols, vals, shape):
    idx = torch.from_numpy(np.vstack((np.asarray(rows, np.int64), np.asarray(cols, np.int64))))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(np.asarray(vals, np.float32)), shape)


def dense_to_coo(x):
    """Row-major COO of the nonzeros of a dense matrix (sp.csr_matrix(.).tocoo())."""
    r, c = np.nonzero(x)
    return _coo(r, c, x[r, c], x.shape)


def sym_normalize(rows, cols, vals, n):
    """Â = D^-1/2 (A+I) D^-1/2 as utils.py:185-213 computes it (float64, one
    rounding to fp32), returned in the COO order ``normalize_adj(...).tocoo()``
    yields for a symmetric A: sorted by (row, col), but not flagged coalesced.
    Input: symmetric A (both directions)."""
    rows = np.asarray(rows, np.int64)
    cols = np.asarray(cols, np.int64)
    v = np.asarray(vals, np.float32).astype(np.float64)
    # A + I, duplicates summed, row-major
    r = np.concatenate([rows, np.arange(n)])
    c = np.concatenate([cols, np.arange(n)])
    w = np.concatenate([v, np.ones(n)])
    key = r * n + c
    order = np.argsort(key, kind="stable")
    key, w = key[order], w[order]
    uniq, start = np.unique(key, return_index=True)
    w = np.add.reduceat(w, start)
    rr, cc = uniq // n, uniq % n
    rowsum = np.bincount(rr, weights=w, minlength=n)
    with np.errstate(divide="ignore"):
        d = np.power(rowsum, -0.5)
    d[np.isinf(d)] = 0.0
    out = ((d[rr] * w) * d[cc]).astype(np.float32)
    return rr, cc, out


def load_r8_fixture(path):
    """R8 as the reference prepared it (tests/golden/r8_graph.npz, written by
    tests/golden/make_golden.py from the reference's own PrepareData)."""
    z = np.load(path, allow_pickle=False)
    N, nfeat, ndoc, ntopic, nclass = (int(v) for v in z["shape"])
    adj = _coo(z["adj_row"], z["adj_col"], z["adj_val"], (N, N))
    dense = np.zeros((N, nfeat), np.float32)
    dense[:ndoc, :ntopic] = z["x_doc"]
    dense[ndoc:, :] = z["x_topic"]
    return {
        "adj": adj,
        "features": dense_to_coo(dense),
        "features_dense": dense,
        "a_rows": z["a_row"], "a_cols": z["a_col"], "a_vals": z["a_val"],
        "target": z["target"], "train_lst": z["train_lst"], "test_lst": z["test_lst"],
        "nfeat": nfeat, "nclass": nclass, "nodes": N, "ndoc": ndoc, "ntopic": ntopic,
        "label_names": [str(s) for s in z["label_names"]],
    }


def doc_topic_graph(ndoc, ntopic, nclass, seed=0, theta_threshold=0.015, tt_prob=None, emb_dim=100):
    """Synthetic doc-topic graph with the reference builder's structure
    (build_graph.py:99-133): doc-topic edges weighted by θ ≥ threshold with
    θ ~ Dirichlet(1/K) (sklearn LDA's default prior), topic-topic edges with
    cosine-like weights U(0.35, 0.76).  Features are the gensim-shaped
    [θ | 0] / L2-normalised embedding rows (trainer.py:197-221)."""
    rng = np.random.default_rng(seed)
    theta = rng.dirichlet(np.full(ntopic, 1.0 / ntopic), size=ndoc)
    d, t = np.nonzero(theta >= theta_threshold)
    w = theta[d, t]
    rows = [d, ndoc + t]
    cols = [ndoc + t, d]
    vals = [w, w]
    p = 237 / 1225 if tt_prob is None else tt_prob
    iu, ju = np.triu_indices(ntopic, 1)
    keep = rng.random(iu.size) < p
    iu, ju = iu[keep], ju[keep]
    ww = rng.uniform(0.35, 0.76, iu.size)
    rows += [ndoc + iu, ndoc + ju]
    cols += [ndoc + ju, ndoc + iu]
    vals += [ww, ww]
    n = ndoc + ntopic
    rr, cc, vv = sym_normalize(np.concatenate(rows), np.concatenate(cols),
                               np.concatenate(vals).astype(np.float32), n)
    nfeat = max(ntopic, emb_dim)
    X = np.zeros((n, nfeat), np.float32)
    th_n = theta / (theta.sum(1, keepdims=True) + 1e-8)
    X[:ndoc, :ntopic] = th_n
    X[ndoc:, :emb_dim] = rng.standard_normal((ntopic, emb_dim))
    X /= np.maximum(np.linalg.norm(X, axis=1, keepdims=True), 1e-12)
    target = rng.integers(0, nclass, ndoc).astype(np.int64)
    return {"adj": _coo(rr, cc, vv, (n, n)), "features": dense_to_coo(X), "features_dense": X,
            "nfeat": nfeat, "nclass": nclass, "nodes": n, "target": target}


def uniform_random_csr(n, nnz, seed=0, device="cpu"):
    """BASELINE config 4/5 graph: rows, cols ~ U[0, n) (torch.Generator(seed)),
    values U[0,1), duplicates summed (coalesce) -> (rowptr, colind, val) int32/fp32."""
    g = torch.Generator().manual_seed(seed)
    rows = torch.randint(0, n, (nnz,), generator=g)
    cols = torch.randint(0, n, (nnz,), generator=g)
    vals = torch.rand(nnz, generator=g)
    t = torch.sparse_coo_tensor(torch.stack([rows, cols]), vals, (n, n)).coalesce()
    idx = t.indices()
    rowptr = torch.zeros(n + 1, dtype=torch.int64)
    rowptr[1:] = torch.cumsum(torch.bincount(idx[0], minlength=n), 0)
    return rowptr.to(torch.int32).to(device), idx[1].to(torch.int32).to(device), t.values().to(device)


def rmat_csr(scale, nnz, a=0.57, b=0.19, c=0.19, seed=0, device="cpu", permute=True):
    """Power-law variant of BASELINE config 4 (R-MAT(0.57,
    0.19, 0.19), reported separately): 2^scale nodes, ``nnz`` edges drawn by
    recursive quadrant choice (probabilities a, b, c, 1 - a - b - c per level,
    torch.Generator(seed)), node ids relabelled by a seeded permutation (as
    Graph500 does, so degree is not correlated with id), values U[0, 1),
    duplicates summed (coalesce) -> (rowptr, colind, val) int32/fp32.  At
    scale 20 / 20M edges the largest row holds ~10^5 nonzeros: the heavy-row
    case a uniform graph never has."""
    n = 1 << scale
    g = torch.Generator().manual_seed(seed)
    rows = torch.zeros(nnz, dtype=torch.int64)
    cols = torch.zeros(nnz, dtype=torch.int64)
    for _ in range(scale):
        r = torch.rand(nnz, generator=g)
        rbit = (r >= a + b).to(torch.int64)
        cbit = (((r >= a) & (r < a + b)) | (r >= a + b + c)).to(torch.int64)
        rows.mul_(2).add_(rbit)
        cols.mul_(2).add_(cbit)
        del r, rbit, cbit
    if permute:
        p = torch.randperm(n, generator=g)
        rows, cols = p[rows], p[cols]
    vals = torch.rand(nnz, generator=g)
    t = torch.sparse_coo_tensor(torch.stack([rows, cols]), vals, (n, n)).coalesce()
    del rows, cols, vals
    idx = t.indices()
    rowptr = torch.zeros(n + 1, dtype=torch.int64)
    rowptr[1:] = torch.cumsum(torch.bincount(idx[0], minlength=n), 0)
    return rowptr.to(torch.int32).to(device), idx[1].to(torch.int32).to(device), t.values().to(device)


def reference_coo(rowptr, colind, val, shape):
    """The torch sparse COO the reference would hand th.spmm for this matrix
    (utils.py:196-203: ``sparse_mx.tocoo()`` of the normalised matrix, which
    comes out of normalize_adj's transpose in COLUMN-major order, int64
    indices, fp32 values, not flagged coalesced) -- the CPU baseline's input
    for the synthetic configs."""
    rp = torch.as_tensor(rowptr).to("cpu", torch.int64)
    ci = torch.as_tensor(colind).to("cpu", torch.int64)
    v = torch.as_tensor(val).to("cpu", torch.float32)
    rows = torch.repeat_interleave(torch.arange(shape[0], dtype=torch.int64), rp[1:] - rp[:-1])
    order = torch.argsort(ci * shape[0] + rows, stable=True)
    return torch.sparse_coo_tensor(torch.stack([rows[order], ci[order]]), v[order], shape)


def load_edgelist(path, device=None):
    """The graph file the reference's builder writes (build_graph.py:199,
    "u v weight" lines) -> the symmetric float32 adjacency A that
    trainer.py:98-148 builds from it, as int32 CSR arrays (native loader,
    gcnk_edgelist_*; no networkx).  Returns (rowptr, colind, val) numpy arrays,
    or a device CSR when ``device`` is given (feed it to
    sparse.preprocess_adj for Â)."""
    import ctypes

    from . import _lib
    lib = _lib.load()
    n, nnz = ctypes.c_int64(), ctypes.c_int64()
    bpath = str(path).encode()
    _lib.check(lib.gcnk_edgelist_size(bpath, ctypes.byref(n), ctypes.byref(nnz)), "gcnk_edgelist_size")
    rp = np.empty(n.value + 1, np.int32)
    ci = np.empty(nnz.value, np.int32)
    v = np.empty(nnz.value, np.float32)
    _lib.check(lib.gcnk_edgelist_csr(bpath, n.value, nnz.value, rp.ctypes.data, ci.ctypes.data, v.ctypes.data),
               "gcnk_edgelist_csr")
    if device is None:
        return rp, ci, v
    from .sparse import from_arrays
    return from_arrays(rp, ci, v, (n.value, n.value), device)
