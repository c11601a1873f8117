"""Generate the committed golden fixtures by running the REFERENCE itself.

Test infrastructure only.  Runs in the build container (never on the GPU box):
it imports the reference from ``$GCN_REFERENCE`` (default ``/root/reference``)
inside a scratch working directory, rebuilds the R8 doc-topic graph with the
reference's own builder, and records the reference's outputs as plain data
(``.npz`` / ``.json``).  No reference source or bytecode is copied anywhere:
``sys.dont_write_bytecode`` is set and only numbers are written.

Call sites exercised (all in the reference):
  build_graph.py:30-206   TopicGraphBuilder("R8", num_topics=50)  (LDA random_state 42)
  trainer.py:83-261       PrepareData  -> .adj (utils.py:185-203), .features (trainer.py:226-238)
  layer.py:126-190        GCN forward, eval and train mode (dropout consumes the CPU RNG)
  trainer.py:264-406      TopicGCNTrainer.fit()/test()  (training-parity goldens; the trained
                          state_dict + eval logits of seed 50494: tie-free labels)
  utils.py:185-213        preprocess_adj on tiny hand-made graphs (known-answer cases)

Usage:  PYTHONHASHSEED=0 python tests/golden/make_golden.py [--skip-train] [--trained-only]
"""
import argparse
import contextlib
import hashlib
import io
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("GCN_REFERENCE", "/root/reference")
SCRATCH = os.environ.get("GCN_ORACLE_SCRATCH", os.path.join(tempfile.gettempdir(), "gcn_oracle_scratch"))

LOGIT_SEEDS = [50494, 99346, 0]
TRAIN_SEEDS = [50494, 99346]

_PRETTYTABLE_STUB = '''
class PrettyTable:
    def __init__(self, *a, **k):
        self.field_names = []
        self.rows = []
    def add_row(self, r):
        self.rows.append(r)
    def __str__(self):
        return "\\n".join(str(r) for r in [self.field_names] + self.rows)
'''


def _sha(t):
    return hashlib.sha256(t.detach().contiguous().numpy().tobytes()).hexdigest()


def _setup():
    os.makedirs(os.path.join(SCRATCH, "data", "graph"), exist_ok=True)
    link = os.path.join(SCRATCH, "data", "text_dataset")
    if not os.path.exists(link):
        os.symlink(os.path.join(REF, "data", "text_dataset"), link)
    stub = os.path.join(SCRATCH, "_stubs")
    os.makedirs(stub, exist_ok=True)
    with open(os.path.join(stub, "prettytable.py"), "w") as f:
        f.write(_PRETTYTABLE_STUB)
    os.chdir(SCRATCH)
    sys.dont_write_bytecode = True
    sys.path.insert(0, stub)
    sys.path.insert(1, REF)
    import numpy as np
    if not hasattr(np, "Inf"):
        np.Inf = np.inf  # utils.py:234 uses the NumPy-1 alias


class _Args:
    pass


def _args(seed=0):
    import torch as th
    a = _Args()
    a.dataset = "R8"
    a.output_dir = os.path.join(SCRATCH, "results")
    a.device = th.device("cpu")
    a.nhid = 200          # trainer.py:426
    a.max_epoch = 200     # trainer.py:427
    a.dropout = 0.5       # trainer.py:428
    a.val_ratio = 0.1     # trainer.py:429
    a.early_stopping = 10  # trainer.py:430
    a.lr = 0.02           # trainer.py:431
    a.seed = seed
    return a


def tiny_cases():
    """Known-answer cases: reference preprocess_adj + GCN on small graphs."""
    import numpy as np
    import scipy.sparse as sp
    import torch as th
    import layer
    import utils
    cases = []
    rng = np.random.default_rng(1234)
    specs = [
        ("path5", 5, [(0, 1, 1.0), (1, 2, 0.5), (2, 3, 2.0), (3, 4, 0.25)], 6, 4, 3),
        ("star7_isolated", 7, [(0, i, 0.1 * i) for i in range(1, 5)] + [(4, 5, 0.7)], 5, 8, 2),
        ("clique4", 4, [(i, j, 1.0) for i in range(4) for j in range(i + 1, 4)], 3, 2, 2),
    ]
    for name, n, edges, nfeat, nhid, ncls in specs:
        r = [e[0] for e in edges] + [e[1] for e in edges]
        c = [e[1] for e in edges] + [e[0] for e in edges]
        v = [e[2] for e in edges] * 2
        A = sp.coo_matrix((np.array(v, np.float32), (r, c)), shape=(n, n), dtype=np.float32).tocsr()
        adj = utils.preprocess_adj(A, is_sparse=True)
        X = rng.random((n, nfeat)).astype(np.float32)
        X[X < 0.35] = 0.0
        Xs = sp.csr_matrix(X).tocoo()
        feats = th.sparse_coo_tensor(th.from_numpy(np.vstack((Xs.row, Xs.col)).astype(np.int64)),
                                     th.from_numpy(Xs.data.astype(np.float32)), (n, nfeat))
        th.manual_seed(7)
        model = layer.GCN(nfeat=nfeat, nhid=nhid, nclass=ncls, dropout=0.5)
        model.eval()
        logits = model(feats, adj)
        th.manual_seed(7)
        model_t = layer.GCN(nfeat=nfeat, nhid=nhid, nclass=ncls, dropout=0.5)
        model_t.train()
        logits_t = model_t(feats, adj)
        ai = adj._indices().numpy()
        cases.append({
            "name": name, "n": n, "nfeat": nfeat, "nhid": nhid, "nclass": ncls,
            "A_rows": r, "A_cols": c, "A_vals": [float(np.float32(x)) for x in v],
            "adj_rows": ai[0].tolist(), "adj_cols": ai[1].tolist(),
            "adj_vals": [float(x) for x in adj._values().numpy()],
            "X": X.tolist(), "init_seed": 7,
            "W1": model.gc1.weight.detach().numpy().tolist(), "b1": model.gc1.bias.detach().numpy().tolist(),
            "W2": model.gc2.weight.detach().numpy().tolist(), "b2": model.gc2.bias.detach().numpy().tolist(),
            "logits_eval": logits.detach().numpy().tolist(),
            "logits_train": logits_t.detach().numpy().tolist(),
        })
    return cases


def trained_golden(trainer, layer, pre, out, quiet):
    """The reference's TRAINED model (trainer.py:349-376, last epoch, the model
    trainer.py:400-406 tests) for TRAIN_SEEDS[0]: its state_dict and its eval
    logits on all nodes.  Trained logits have a clear top-2 gap (SURVEY §7:
    ~2.5e-3), so predicted labels can be compared bit-exactly on EVERY row."""
    import numpy as np
    import torch as th
    seed = TRAIN_SEEDS[0]
    a = _args(seed)
    with contextlib.redirect_stdout(quiet):
        fw = trainer.TopicGCNTrainer(model=layer.GCN, args=a, pre_data=pre)
        fw.fit()
        res = fw.test()
    fw.model.eval()
    with th.no_grad():
        lg = fw.model(fw.features, fw.adj).numpy()
    srt = np.sort(lg, axis=1)
    gap = srt[:, -1] - srt[:, -2]
    sd = {k: v.detach().numpy() for k, v in fw.model.state_dict().items()}
    np.savez_compressed(os.path.join(out, "r8_trained.npz"), logits=lg, seed=np.int64(seed),
                        epochs=np.int64(len(fw.training_history)), test_acc=np.float64(res["acc"]),
                        min_top2_gap=np.float64(gap.min()), **{"sd_" + k: v for k, v in sd.items()})
    print(f"trained golden: seed {seed}, {len(fw.training_history)} epochs, test acc {res['acc']:.4f}, "
          f"min top-2 gap {gap.min():.3e}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-train", action="store_true")
    ap.add_argument("--trained-only", action="store_true",
                    help="only (re)write r8_trained.npz (the trained-weight golden)")
    ap.add_argument("--out", default=HERE)
    opts = ap.parse_args()

    if os.environ.get("PYTHONHASHSEED") != "0":
        # label ids come from set() order (trainer.py:254): pin the hash seed by
        # re-running this script as a CHILD process (CPU only, no GPU touched).
        env = dict(os.environ, PYTHONHASHSEED="0", PYTHONDONTWRITEBYTECODE="1")
        sys.exit(subprocess.call([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))

    out = os.path.abspath(opts.out)
    _setup()
    import numpy as np
    import torch as th
    th.set_num_threads(8)
    quiet = io.StringIO()

    graph_file = os.path.join(SCRATCH, "data", "graph", "R8_topic.txt")
    with contextlib.redirect_stdout(quiet), contextlib.redirect_stderr(quiet):
        import build_graph
        if not os.path.exists(graph_file):
            build_graph.TopicGraphBuilder("R8", num_topics=50)
        import trainer
        import layer
        pre = trainer.PrepareData(_args())

    adj = pre.adj
    feats = pre.features
    assert not adj.is_coalesced()
    if opts.trained_only:
        trained_golden(trainer, layer, pre, out, quiet)
        return
    ai = adj._indices().numpy()
    av = adj._values().numpy()
    N = adj.shape[0]
    nfeat = feats.shape[1]
    num_topics = 50
    ndoc = N - num_topics

    # ---- X: verify it is exactly [doc block | 0] over [topic block] in row-major COO
    fi = feats._indices().numpy()
    fv = feats._values().numpy()
    dense = feats.to_dense().numpy()
    x_doc = np.ascontiguousarray(dense[:ndoc, :num_topics])
    x_topic = np.ascontiguousarray(dense[ndoc:, :])
    assert not dense[:ndoc, num_topics:].any()
    rr, cc = np.nonzero(dense)
    assert np.array_equal(rr, fi[0]) and np.array_equal(cc, fi[1]), "features COO is not row-major nonzero order"
    assert np.array_equal(dense[rr, cc], fv)

    # ---- raw symmetric A (before +I), reproduced with the reference's own steps
    #      (trainer.py:98-148) so device-side normalisation can be checked bit-exactly
    import networkx as nx
    g = nx.read_weighted_edgelist(graph_file, nodetype=int)
    A = nx.adjacency_matrix(g, nodelist=list(range(g.number_of_nodes())), weight="weight", dtype=np.float32)
    A = (A + A.T.multiply(A.T > A) - A.multiply(A.T > A)).tocsr()
    A.sort_indices()
    Acoo = A.tocoo()

    target = np.asarray(pre.target, dtype=np.int64)
    # label names in id order (set() order under PYTHONHASHSEED=0, trainer.py:254)
    import pandas as pd
    names = np.array(pd.read_csv("data/text_dataset/R8.txt", sep="\t", header=None)[2])
    id2name = {}
    for nm, t in zip(names, target):
        id2name[int(t)] = str(nm)
    label_names = [id2name[i] for i in range(pre.nclass)]

    np.savez_compressed(
        os.path.join(out, "r8_graph.npz"),
        adj_row=ai[0].astype(np.int32), adj_col=ai[1].astype(np.int32), adj_val=av.astype(np.float32),
        a_row=Acoo.row.astype(np.int32), a_col=Acoo.col.astype(np.int32), a_val=Acoo.data.astype(np.float32),
        x_doc=x_doc.astype(np.float32), x_topic=x_topic.astype(np.float32),
        target=target, train_lst=np.asarray(pre.train_lst, np.int64), test_lst=np.asarray(pre.test_lst, np.int64),
        shape=np.array([N, nfeat, ndoc, num_topics, pre.nclass], np.int64),
        label_names=np.array(label_names),
    )

    # ---- forward goldens (reference GCN on the reference tensors)
    logit_meta = {}
    arrays = {}
    for seed in LOGIT_SEEDS:
        th.manual_seed(seed)
        m = layer.GCN(nfeat=nfeat, nhid=200, nclass=pre.nclass, dropout=0.5)
        m.eval()
        with th.no_grad():
            lg = m(feats, adj)
        arrays[f"eval_{seed}"] = lg.numpy()
        srt = np.sort(lg.numpy(), axis=1)
        gap = srt[:, -1] - srt[:, -2]
        logit_meta[str(seed)] = {
            "params_sha256": {k: _sha(v) for k, v in m.state_dict().items()},
            "min_top2_gap": float(gap.min()),
        }
    # train-mode forward + backward for the first seed: dropout mask drawn from the CPU RNG
    seed = LOGIT_SEEDS[0]
    th.manual_seed(seed)
    m = layer.GCN(nfeat=nfeat, nhid=200, nclass=pre.nclass, dropout=0.5)
    m.train()
    lg = m(feats, adj)
    arrays[f"train_{seed}"] = lg.detach().numpy()
    tl = th.tensor(pre.train_lst[:2000], dtype=th.long)
    loss = th.nn.CrossEntropyLoss()(lg[tl], th.tensor(target)[tl])
    loss.backward()
    grads = {}
    for k, p in m.named_parameters():
        gg = p.grad.detach().numpy().astype(np.float64)
        grads[k] = {"sum": float(gg.sum()), "abs_sum": float(np.abs(gg).sum()), "shape": list(gg.shape)}
    arrays["grad_gc2.weight"] = m.gc2.weight.grad.numpy()
    arrays["grad_gc2.bias"] = m.gc2.bias.grad.numpy()
    arrays["grad_gc1.bias"] = m.gc1.bias.grad.numpy()
    arrays["grad_gc1.weight_rows0_64"] = m.gc1.weight.grad[:64].numpy()
    arrays["grad_gc1.weight_rows_tail"] = m.gc1.weight.grad[-64:].numpy()
    logit_meta["train_grad"] = {"seed": seed, "loss": float(loss), "n_train_rows": int(len(tl)), "grads": grads}
    np.savez_compressed(os.path.join(out, "r8_logits.npz"), **arrays)

    meta = {
        "generator": "tests/golden/make_golden.py",
        "reference": "anargh-t/Graph-Convolutional-Networks-for-Text-Classification (read-only mount)",
        "env": {"torch": th.__version__, "numpy": np.__version__, "PYTHONHASHSEED": "0"},
        "graph": {"nodes": int(N), "adj_nnz": int(av.size), "x_nnz": int(fv.size), "nfeat": int(nfeat),
                  "ndoc": int(ndoc), "ntopic": num_topics, "nclass": int(pre.nclass), "a_nnz": int(Acoo.nnz)},
        "logit_seeds": LOGIT_SEEDS,
        "logits": logit_meta,
    }

    # ---- training-parity goldens (trainer.py:264-406, CPU, full run)
    if not opts.skip_train:
        runs = {}
        for seed in TRAIN_SEEDS:
            a = _args(seed)
            with contextlib.redirect_stdout(quiet):
                fw = trainer.TopicGCNTrainer(model=layer.GCN, args=a, pre_data=pre)
                fw.fit()
                res = fw.test()
            hist = [{k: (float(v) if not isinstance(v, int) else v) for k, v in h.items()} for h in fw.training_history]
            runs[str(seed)] = {
                "epochs": len(hist),
                "history": hist,
                "test": {k: float(v) for k, v in res.items()},
                "train_idx": [int(x) for x in fw.train_lst.tolist()],
                "val_idx": [int(x) for x in fw.val_lst.tolist()],
            }
        meta["train_runs"] = runs

        trained_golden(trainer, layer, pre, out, quiet)
    meta["tiny_cases"] = tiny_cases()
    with open(os.path.join(out, "r8_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote fixtures to", out)


if __name__ == "__main__":
    main()
