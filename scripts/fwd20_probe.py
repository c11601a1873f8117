"""BASELINE config 3 (20ng-shaped doc-topic graph, gensim-shaped X, hidden 200,
20 classes): eval-forward per-call time, and X W1 through the sparse tile path
against the dense GEMM on the same X.  One JSON line per measurement."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from hub_probe import time_graph
    dev = torch.device("cuda", 0)
    g = datasets.doc_topic_graph(18846, 70, 20, seed=0)
    torch.manual_seed(1)
    m = GCN(nfeat=g["nfeat"], nhid=200, nclass=20, dropout=0.5).to(dev).eval()
    a, x = g["adj"].to(dev), g["features"].to(dev)
    xd = torch.from_numpy(g["features_dense"]).to(dev)
    xc = as_csr(x)
    with torch.no_grad():
        m(x, a)
        us = time_graph([lambda: m(x, a)], 20)
        print(json.dumps({"case": "20ng forward", "us": round(us, 3), "x_nnz": xc.nnz, "x_shape": list(xc.shape),
                          "density": xc.nnz / (xc.shape[0] * xc.shape[1])}), flush=True)
        W1 = m.gc1.weight.detach()
        s1 = ops.spmm(xc, W1)
        s2 = ops.gemm(xd, W1)
        print(json.dumps({"case": "20ng X W1 sparse", "us": round(time_graph([lambda: ops.spmm(xc, W1, out=s1)], 50), 3),
                          "hdr": list(list(xc._plans.values())[-1].header)}), flush=True)
        print(json.dumps({"case": "20ng X W1 dense gemm", "us": round(time_graph([lambda: ops.gemm(xd, W1, out=s2)], 50), 3),
                          "max_diff": float((s1 - s2).abs().max())}), flush=True)
        md = GCN(nfeat=g["nfeat"], nhid=200, nclass=20, dropout=0.5).to(dev).eval()
        md.load_state_dict(m.state_dict())
        md(xd, a)
        print(json.dumps({"case": "20ng forward, dense X", "us": round(time_graph([lambda: md(xd, a)], 20), 3)}),
              flush=True)


if __name__ == "__main__":
    main()
