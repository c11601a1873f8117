"""CPU checks of the hub factorisation behind the factored gc1 kernel
(csrc/factor.hip), on its host restatement oracle/factor_host.py (the device
build, factor.py + csrc/factor_build.hip, is pinned to it bit for bit by
tests/test_gpu_parity.py): the operands it builds reproduce A-hat X W1 of the
reference (layer.py:102,106) in float64 on the reference-built R8 graph and on
synthetic doc-topic graphs, the per-block records hold exactly A-hat's
hub-column nonzeros, and graphs without the structure are refused."""
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

import gcn_amd  # noqa: F401
from graph_convolutional_networks_for_text_classification_amd import datasets
from graph_convolutional_networks_for_text_classification_amd.sparse import from_arrays
from oracle import factor_host as factor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _XOp:
    """Operand stand-in on the CPU (ops.Operand needs a GPU tensor)."""

    def __init__(self, csr=None, dense=None):
        self.csr, self.dense = csr, dense

    @property
    def shape(self):
        return self.csr.shape if self.csr is not None else tuple(self.dense.shape)


def _csr(m):
    m = sp.csr_matrix(m)
    m.sort_indices()
    return from_arrays(m.indptr.astype(np.int32), m.indices.astype(np.int32), m.data.astype(np.float32), m.shape, "cpu")


def _check_factor(A, X, F=24, seed=0):
    """float64: U W1[Kc] + A_H (X[hubs] W1) == A (X W1)."""
    A, X = sp.csr_matrix(A), sp.csr_matrix(X)
    f = factor.build(_csr(A), _XOp(csr=_csr(X)))
    assert f is not None
    W1 = np.random.default_rng(seed).standard_normal((X.shape[1], F))
    Af, Xf = A.astype(np.float64), X.astype(np.float64)
    ref = Af @ (Xf @ W1)
    U = f.U.astype(np.float64)
    hubs = f.hubs
    perm = f.perm
    S_T = Xf[hubs] @ W1
    Z = U[:, :f.Kc] @ W1[f.k0:f.k0 + f.Kc]          # block order: position i holds row perm[i]
    rec = f.rec
    M = A.shape[0]
    assert np.array_equal(np.sort(perm), np.arange(M))
    nnz_h = 0
    for b in range(rec.shape[0]):
        off = rec[b, :33]
        items = rec[b, factor.REC_HEAD:].reshape(-1, 2)
        for i in range(32):
            p = 32 * b + i
            assert rec[b, factor.REC_ROW + i] == (perm[p] if p < M else -1)
            if p >= M:
                continue
            for k in range(off[i], off[i + 1]):
                t, bits = items[k]
                Z[p] += np.int32(bits).view(np.float32) * S_T[t]
                nnz_h += 1
    # exactly the hub-column nonzeros of A-hat, each once
    is_hub = np.zeros(M, bool)
    is_hub[hubs] = True
    assert nnz_h == int(is_hub[A.indices].sum())
    err = np.abs(Z - ref[perm]).max() / max(1.0, np.abs(ref).max())
    assert err < 1e-6, err
    # hub rows spread: no block holds more than ceil(H / nblk) + 1 of them
    pos = np.empty(M, np.int64)
    pos[perm] = np.arange(M)
    per_block = np.bincount(pos[hubs] // 32, minlength=rec.shape[0])
    assert per_block.max() <= -(-len(hubs) // rec.shape[0]) + 1, per_block.max()
    return f


def test_factor_reproduces_r8_product():
    g = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    A = g["adj"].coalesce()
    X = g["features"].coalesce()
    Asp = sp.csr_matrix((A.values().numpy(), A.indices().numpy()), shape=A.shape)
    Xsp = sp.csr_matrix((X.values().numpy(), X.indices().numpy()), shape=X.shape)
    f = _check_factor(Asp, Xsp, F=16)
    # R8: the 50 topic rows are the hubs; documents use topic-weight columns 0..49
    assert f.H == 50 and f.k0 == 0 and f.Kc == 50
    assert f.hubs.tolist() == list(range(7674, 7724))


@pytest.mark.parametrize("ndoc,ntopic,seed", [(600, 12, 1), (1500, 40, 3), (333, 7, 5)])
def test_factor_synthetic_doc_topic(ndoc, ntopic, seed):
    g = datasets.doc_topic_graph(ndoc=ndoc, ntopic=ntopic, nclass=4, seed=seed)
    A, X = g["adj"].coalesce(), g["features"].coalesce()
    Asp = sp.csr_matrix((A.values().numpy(), A.indices().numpy()), shape=A.shape)
    Xsp = sp.csr_matrix((X.values().numpy(), X.indices().numpy()), shape=X.shape)
    # small synthetic graphs may have no row past the hub threshold: then no factor
    f = factor.build(_csr(Asp), _XOp(csr=_csr(Xsp)))
    if f is None:
        deg = np.diff(Asp.indptr)
        assert deg.max() < max(64, 8 * -(-Asp.nnz // Asp.shape[0]))
        return
    _check_factor(Asp, Xsp)


def test_factor_dense_features():
    # gensim-shaped X (dense 100-d rows): Kc = all columns
    rng = np.random.default_rng(7)
    nd, nt = 900, 10
    M = nd + nt
    rows, cols = [], []
    for d in range(nd):
        for t in rng.choice(nt, size=rng.integers(1, 4), replace=False):
            rows += [d, nd + t]
            cols += [nd + t, d]
    A = sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(M, M)) + sp.eye(M)
    dinv = 1 / np.sqrt(np.asarray(A.sum(1)).ravel())
    A = sp.diags(dinv) @ A @ sp.diags(dinv)
    X = rng.standard_normal((M, 100)).astype(np.float32)
    f = factor.build(_csr(A), _XOp(dense=torch.from_numpy(X)))
    assert f is not None and f.Kc == 100 and f.k0 == 0
    W1 = rng.standard_normal((100, 8))
    hubs = f.hubs
    ref = A @ (X.astype(np.float64) @ W1)
    perm = f.perm
    Z = f.U[:, :100].astype(np.float64) @ W1       # rows in the block order
    Zh = A[:, hubs] @ (X[hubs].astype(np.float64) @ W1)
    assert np.abs(Z + Zh[perm] - ref[perm]).max() < 1e-5 * max(1, np.abs(ref).max())


def test_factor_refuses_unstructured_graph():
    rng = np.random.default_rng(0)
    M = 400
    A = sp.random(M, M, density=0.05, random_state=1, format="csr") + sp.eye(M)
    A = A + A.T
    X = sp.random(M, 30, density=0.3, random_state=2, format="csr")
    assert factor.build(_csr(A), _XOp(csr=_csr(X))) is None
    # hubs present but a light row references another light row
    nd, nt = 300, 4
    rows = [d for d in range(nd)] + [nd + d % nt for d in range(nd)] + [0, 1]
    cols = [nd + d % nt for d in range(nd)] + [d for d in range(nd)] + [1, 0]
    A = sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(nd + nt, nd + nt)) + sp.eye(nd + nt)
    X = sp.csr_matrix(rng.random((nd + nt, 5)))
    assert factor.build(_csr(A), _XOp(csr=_csr(X))) is None


def test_hub_operand_choice():
    """Which form of X[hubs] the product S_T = X[hubs] W1 takes (factor.py):
    the CSR when no dense copy exists; with both, the dense copy in eval and
    the CSR in a training forward (XHUB_TRAIN_TILE, profiles/r06_xhub_train_ab.log)."""
    from graph_convolutional_networks_for_text_classification_amd import factor
    f = factor.HubFactor()
    f.x_hub, f.x_hub_dense = object(), None
    assert f.hub_operand(False) == "csr" and f.hub_operand(True) == "csr"
    f.x_hub_dense = object()
    assert f.hub_operand(False) == "dense"
    assert f.hub_operand(True) == ("csr" if factor.XHUB_TRAIN_TILE else "dense")
    f.x_hub = None   # a dense X: its hub rows exist only as the dense copy
    assert f.hub_operand(True) == "dense"
