"""The R8 forward's ops launched eagerly (no hipGraph), a few times each, for
rocprofv3 --pmc passes (scripts/pmc.sh): per-dispatch HBM counters of every
kernel of the forward."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(reps=10):
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
        # 512 MB write between rounds: every round starts from HBM, not the 256 MB MALL
        flush = torch.empty(128 * 1024 * 1024, dtype=torch.float32, device=dev)
        for _ in range(reps):
            flush.fill_(1.0)
            ops.spmm(x, W1, out=S1)
            ops.spmm(a, S1, bias=b1, epilogue=2, out=H1)
            ops.gemm(H1, W2, out=S2)
            ops.spmm(a, S2, bias=b2, epilogue=1, out=Z)
    torch.cuda.synchronize()
    print("pmc ops done", flush=True)


if __name__ == "__main__":
    main()
