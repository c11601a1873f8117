"""Feasibility probe for computing U W1[Kc] in the X_hubs W1 launch: the CSR of
[X_hubs ; U placed in X's columns k0 .. k0 + Kc] (hub rows first, then U's rows
in block order) through the SpMM tile plan, against X_hubs alone (warm,
hipGraph of back-to-back calls).  One JSON line per op.

  python scripts/xu_probe.py [--graphs r8,20ng] [--reps 200]
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
    ap.add_argument("--graphs", default="r8")
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets, factor, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import CSR, as_csr
    from hub_probe import time_graph
    dev = torch.device("cuda", 0)
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
        W1 = m.gc1.weight.detach()

        def line(op, us, **kw):
            print(json.dumps({"graph": gname, "op": op, "us": round(us, 3), **kw}), flush=True)

        if f is None or f.x_hub is None:
            line("no factor / dense X", 0.0)
            continue
        M, H, Kc, k0 = f.M, f.H, f.Kc, f.k0
        xh = f.x_hub
        # U rows as CSR over X's columns (dense over k0 .. k0 + Kc)
        ucol = (torch.arange(Kc, device=dev, dtype=torch.int32) + k0).repeat(M)
        uval = f.U[:, :Kc].contiguous().view(-1)
        urp = torch.arange(M + 1, device=dev, dtype=torch.int32) * Kc
        rp = torch.cat([xh.rowptr, urp[1:] + xh.rowptr[-1]])
        xu = CSR(rp, torch.cat([xh.colind, ucol]), torch.cat([xh.val, uval]), (H + M, xh.shape[1]))
        with torch.no_grad():
            ref_s = ops.spmm(xh, W1)
            out = ops.spmm(xu, W1)
            want_z = f.U[:, :Kc].double() @ W1[k0:k0 + Kc].double()
            line("X_hubs W1 (tile spmm)", time_graph([lambda: ops.spmm(xh, W1)], args.reps))
            line("[X_hubs; U] W1 (tile spmm)", time_graph([lambda: ops.spmm(xu, W1)], args.reps),
                 s_err=float((out[:H] - ref_s).abs().max()), z_err=float((out[H:].double() - want_z).abs().max()),
                 nnz=int(xu.nnz))
            uw = f.U[:, :Kc].contiguous()
            wk = W1[k0:k0 + Kc].contiguous()
            line("U W1[Kc] alone (gemm)", time_graph([lambda: ops.gemm(uw, wk)], args.reps))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
