"""Eval-forward per-call time of R8 (BASELINE config 2) and the 20ng-shaped graph
(config 3) with gc2's H1 W2 fused into the gc1 aggregation (ops.FUSE_PROJECTION)
and without it.  One JSON line per (graph, schedule)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets, ops
    from hub_probe import time_graph
    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    g20 = datasets.doc_topic_graph(18846, 70, 20, seed=0)
    cases = [("r8", r8["nfeat"], r8["nclass"], r8["features"], r8["adj"]),
             ("20ng", g20["nfeat"], 20, torch.from_numpy(g20["features_dense"]), g20["adj"])]
    for name, nfeat, ncls, x, a in cases:
        torch.manual_seed(1)
        m = GCN(nfeat=nfeat, nhid=200, nclass=ncls, dropout=0.5).to(dev).eval()
        x, a = x.to(dev), a.to(dev)
        outs = {}
        with torch.no_grad():
            for fuse in (True, False):
                ops.FUSE_PROJECTION = fuse
                outs[fuse] = m(x, a).clone()
                us = time_graph([lambda: m(x, a)], 20)
                print(json.dumps({"graph": name, "fuse_projection": fuse, "forward_us": round(us, 3)}), flush=True)
        print(json.dumps({"graph": name, "max_diff": float((outs[True] - outs[False]).abs().max())}), flush=True)


if __name__ == "__main__":
    main()
