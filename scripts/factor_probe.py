"""Per-op timing of the factored forward (warm, hipGraph of back-to-back
launches, HIP events per call): X_hubs W1 (tile SpMM or GEMM),
hubfactor_gc1, A-hat S2, and the whole record forward, on R8 and the
20ng-shaped graph.  One JSON line per (graph, op).  Run it under
GCNK_LIB=<variant .so> to compare kernel builds.

  python scripts/factor_probe.py [--graphs r8,20ng] [--reps 200]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", default="r8,20ng")
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, _lib, datasets, factor, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    from hub_probe import time_graph
    dev = torch.device("cuda", 0)
    tag = os.path.basename(os.environ.get("GCNK_LIB", "libgcnk.so"))
    for gname in args.graphs.split(","):
        if gname == "r8":
            g = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
        else:
            g = datasets.doc_topic_graph(18846, 70, 20, seed=0)
        torch.manual_seed(0)
        m = GCN(nfeat=g["nfeat"], nhid=200, nclass=g["nclass"], dropout=0.5).to(dev).eval()
        x, adj = g["features"].to(dev), g["adj"].to(dev)
        a = as_csr(adj)
        xop = ops.Operand(x)
        f = factor.get(a, xop)
        W1, b1 = m.gc1.weight.detach(), m.gc1.bias.detach()
        W2, b2 = m.gc2.weight.detach(), m.gc2.bias.detach()

        def line(op, us, **kw):
            print(json.dumps({"lib": tag, "graph": gname, "op": op, "us": round(us, 3), **kw}), flush=True)

        with torch.no_grad():
            if f is None or not ops.FACTOR_GC1:
                line("forward (record, unfactored)", time_graph([lambda: m(x, adj)], args.reps))
                continue
            S_T = f.hub_times(W1).contiguous()
            if f.x_hub is not None:
                line("X_hubs W1 (tile spmm)", time_graph([lambda: ops.spmm(f.x_hub, W1)], args.reps))
            if f.x_hub_dense is not None:
                line("X_hubs W1 (gemm)", time_graph([lambda: ops.gemm(f.x_hub_dense, W1)], args.reps))
            H1, S2 = ops.hubfactor_gc1(f, W1, b1, W2, store_h1=False, S=S_T)
            line("hubfactor_gc1", time_graph([lambda: ops.hubfactor_gc1(f, W1, b1, W2, store_h1=False, S=S_T)],
                                             args.reps))
            line("A S2", time_graph([lambda: ops.spmm(a, S2, bias=b2, epilogue=_lib.EPI_BIAS)], args.reps))
            line("forward (record)", time_graph([lambda: m(x, adj)], args.reps))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
