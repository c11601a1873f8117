"""The R8 forward's ops launched eagerly (no hipGraph), a few times each, for
rocprofv3 --pmc passes (scripts/pmc.sh, and bench.py's live traffic pass):
per-dispatch HBM counters of every kernel of the forward.  Each round starts
behind a 512 MB write, so no round finds its operands in the 256 MB
Infinity Cache (cold, as the roofline is defined).

  python scripts/pmc_ops.py [--op all|XW1|AS1|H1W2|AS2] [--reps 10]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="all")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr

    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    torch.manual_seed(0)
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(dev).eval()
    a, x = as_csr(r8["adj"].to(dev)), as_csr(r8["features"].to(dev))
    W1, b1 = m.gc1.weight.detach(), m.gc1.bias.detach()
    W2, b2 = m.gc2.weight.detach(), m.gc2.bias.detach()
    with torch.no_grad():
        S1 = ops.spmm(x, W1)
        H1 = ops.spmm(a, S1, bias=b1, epilogue=2)
        S2 = ops.gemm(H1, W2)
        Z = ops.spmm(a, S2, bias=b2, epilogue=1)
        steps = {"XW1": lambda: ops.spmm(x, W1, out=S1),
                 "AS1": lambda: ops.spmm(a, S1, bias=b1, epilogue=2, out=H1),
                 "H1W2": lambda: ops.gemm(H1, W2, out=S2),
                 "AS2": lambda: ops.spmm(a, S2, bias=b2, epilogue=1, out=Z)}
        run = list(steps.values()) if args.op == "all" else [steps[args.op]]
        flush = torch.empty(128 * 1024 * 1024, dtype=torch.float32, device=dev)
        for _ in range(args.reps):
            flush.fill_(1.0)
            for f in run:
                f()
    torch.cuda.synchronize()
    print("pmc ops done", flush=True)


if __name__ == "__main__":
    main()
