"""ORACLE (test infrastructure only): torch-CPU restatement of the reference GCN.

Issues the same ATen calls, in the same order, as the reference:
  GraphConvolution.forward      layer.py:84-112   th.spmm(infeatn, W); th.spmm(adj, support); + bias
  GraphConvolution init         layer.py:67-82    U(-1/sqrt(out), 1/sqrt(out)), weight then bias
  GCN.forward                   layer.py:164-190  gc1 -> th.relu -> th.dropout(p, train) -> gc2
  preprocess_adj/normalize_adj  utils.py:185-213  D^-1/2 (A+I) D^-1/2 in float64, cast to fp32 COO
  trainer loop                  trainer.py:349-406  Adam(lr), CE on train idx, val each epoch,
                                                    EarlyStopping(patience) utils.py:216-255
  accuracy / macro_f1           utils.py:25-109
so on identical tensors it reproduces the reference's outputs bit for bit
(checked against tests/golden by tests/test_oracle.py).
"""
import math

import numpy as np
import torch as th


class RefGraphConvolution(th.nn.Module):
    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = th.nn.Parameter(th.empty(in_features, out_features))
        self.bias = th.nn.Parameter(th.empty(out_features)) if bias else None
        stdv = 1.0 / math.sqrt(out_features)
        self.weight.data.uniform_(-stdv, stdv)
        if self.bias is not None:
            self.bias.data.uniform_(-stdv, stdv)

    def forward(self, infeatn, adj):
        support = th.spmm(infeatn, self.weight)
        output = th.spmm(adj, support)
        return output + self.bias if self.bias is not None else output


class RefGCN(th.nn.Module):
    def __init__(self, nfeat, nhid, nclass, dropout):
        super().__init__()
        self.gc1 = RefGraphConvolution(nfeat, nhid)
        self.gc2 = RefGraphConvolution(nhid, nclass)
        self.dropout = dropout

    def forward(self, x, adj):
        x = th.relu(self.gc1(x, adj))
        x = th.dropout(x, self.dropout, train=self.training)
        return self.gc2(x, adj)


def normalize_adj_coo(rows, cols, vals, n):
    """Â = D^-1/2 (A+I) D^-1/2 with the reference's arithmetic (utils.py:185-213).

    A+I is formed in float64 (sp.eye is float64, utils.py:188); row sums and
    d = rowsum^-0.5 in float64; each value is d[r] * a * d[c] in float64 and
    rounded to fp32 once (utils.py:198).  Returns CSR-sorted (row, col, val)."""
    import scipy.sparse as sp
    A = sp.coo_matrix((np.asarray(vals, np.float32), (rows, cols)), shape=(n, n), dtype=np.float32)
    A = A + sp.eye(n)
    rowsum = np.asarray(A.sum(1)).flatten()
    with np.errstate(divide="ignore"):
        d = np.power(rowsum, -0.5)
    d[np.isinf(d)] = 0.0
    C = A.tocsr()
    C.sum_duplicates()
    C.sort_indices()
    r = np.repeat(np.arange(n), np.diff(C.indptr))
    v = (d[r] * C.data.astype(np.float64)) * d[C.indices]
    return r.astype(np.int64), C.indices.astype(np.int64), v.astype(np.float32)


def coo_tensor(rows, cols, vals, shape):
    """A torch sparse COO exactly as given (order preserved, NOT coalesced),
    like th.sparse.FloatTensor(indices, values, shape) in utils.py:199-203."""
    idx = th.from_numpy(np.vstack((np.asarray(rows), np.asarray(cols))).astype(np.int64))
    return th.sparse_coo_tensor(idx, th.from_numpy(np.asarray(vals, np.float32)), shape)


def accuracy(pred, targ):
    pred = th.max(pred, 1)[1]
    return ((pred == targ).float()).sum().item() / targ.size()[0]


def macro_f1(pred, targ, num_classes):
    pred = th.max(pred, 1)[1]
    tp, fp, fn = [], [], []
    for i in range(num_classes):
        tp.append(((pred == i) & (targ == i)).sum().item())
        fp.append(((pred == i) & (targ != i)).sum().item())
        fn.append(((pred != i) & (targ == i)).sum().item())
    tp, fp, fn = np.array(tp), np.array(fp), np.array(fn)
    with np.errstate(divide="ignore", invalid="ignore"):
        precision = tp / (tp + fp)
        precision[np.isnan(precision)] = 0
        precision = np.mean(precision)
        recall = tp / (tp + fn)
        recall[np.isnan(recall)] = 0
        recall = np.mean(recall)
        f1 = 2 * (precision * recall) / (precision + recall)
    return f1, precision, recall


class EarlyStopping:
    """utils.py:216-255: strict improvement of val loss, counter to patience."""

    def __init__(self, patience=7, delta=0.0):
        self.patience, self.delta = patience, delta
        self.counter, self.best_score, self.early_stop = 0, None, False

    def __call__(self, val_loss):
        score = -val_loss
        if self.best_score is None:
            self.best_score = score
        elif score < self.best_score + self.delta:
            self.counter += 1
            if self.counter >= self.patience:
                self.early_stop = True
                return True
        else:
            self.best_score = score
            self.counter = 0
        return None


def train_run(model_cls, features, adj, target, train_idx, val_idx, test_idx, nfeat, nclass, seed,
              nhid=200, dropout=0.5, lr=0.02, max_epoch=200, patience=10, device="cpu", model_kwargs=None):
    """trainer.py:294-406 for one seed: returns (history, test_desc, model).

    ``model_cls`` is any class with the reference GCN constructor — the
    reference-equivalent RefGCN here, or the HIP drop-in in the tests."""
    th.manual_seed(seed)                                   # trainer.py:295
    np.random.seed(seed)                                   # trainer.py:296
    model = model_cls(nfeat=nfeat, nhid=nhid, nclass=nclass, dropout=dropout, **(model_kwargs or {}))
    model = model.to(device)
    opt = th.optim.Adam(model.parameters(), lr=lr)
    crit = th.nn.CrossEntropyLoss()
    features, adj = features.to(device), adj.to(device)
    target = th.as_tensor(target).long().to(device)
    tr = th.as_tensor(train_idx).long().to(device)
    va = th.as_tensor(val_idx).long().to(device)
    te = th.as_tensor(test_idx).long().to(device)
    stopper = EarlyStopping(patience)
    history = []

    def evaluate(idx, prefix):
        model.eval()
        with th.no_grad():
            logits = model.forward(features, adj)
            loss = crit(logits[idx], target[idx])
            acc = accuracy(logits[idx], target[idx])
            f1, p, r = macro_f1(logits[idx], target[idx], nclass)
        return {f"{prefix}_loss": loss.item(), "acc": acc, "macro_f1": f1, "precision": p, "recall": r}

    for epoch in range(max_epoch):
        model.train()
        opt.zero_grad()
        logits = model.forward(features, adj)
        loss = crit(logits[tr], target[tr])
        loss.backward()
        opt.step()
        desc = dict(epoch=epoch, train_loss=loss.item(), **evaluate(va, "val"))
        history.append(desc)
        if stopper(desc["val_loss"]):
            break
    return history, evaluate(te, "test"), model
