"""Diagnostics: per-op times of the R8 forward after a sustained warm-up (clock
ramp), an in-kernel clock estimate, and the SpMM per-workgroup timeline."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def time_graph(fn, reps=200, rounds=5):
    import torch
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(rounds):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / reps)
    return min(res), res


def main():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr

    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    A = as_csr(r8["adj"].to(dev))
    X = as_csr(r8["features"].to(dev))
    torch.manual_seed(0)
    W1 = torch.randn(r8["nfeat"], 200, device=dev)
    S1 = torch.randn(r8["nodes"], 200, device=dev)
    S2 = torch.randn(r8["nodes"], 8, device=dev)
    H = torch.empty(r8["nodes"], 200, device=dev)
    W2 = torch.randn(200, 8, device=dev)
    o8 = torch.empty(r8["nodes"], 8, device=dev)
    z = torch.zeros(1, device=dev)
    ops_ = {
        "trivial_add": lambda: z.add_(1.0),
        "XW1": lambda: ops.spmm(X, W1, out=H),
        "AS1_F200": lambda: ops.spmm(A, S1, out=H),
        "AS1_F200_nodense": lambda: ops.spmm(A, S1, out=H, dense=2.0),
        "AS1_F200_dense05": lambda: ops.spmm(A, S1, out=H, dense=0.05),
        "AS1_F200_proj": lambda: ops.spmm_proj(A, S1, W2, bias=W2[0].repeat(25), epilogue=2, store_main=False),
        "AS1_F200_proj_H": lambda: ops.spmm_proj(A, S1, W2, bias=W2[0].repeat(25), epilogue=2),
        "AS2_F8": lambda: ops.spmm(A, S2, out=o8),
        "gemm_H_W2": lambda: ops.gemm(H, W2, out=o8),
        "torch_mm_H_W2": lambda: torch.mm(H, W2, out=o8),
        "copy_6MB": lambda: H.copy_(S1),
    }
    print(json.dumps({"phase": "cold"}), flush=True)
    for k, fn in ops_.items():
        print(json.dumps({"op": k, "us": round(time_graph(fn, rounds=2)[0], 2)}), flush=True)
    # sustained load: 3 s of back-to-back replays of the forward
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(dev).eval()
    adj, x = r8["adj"].to(dev), r8["features"].to(dev)
    with torch.no_grad():
        m(x, adj)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(g):
        for _ in range(50):
            m(x, adj)
    t0 = time.time()
    n = 0
    while time.time() - t0 < 3.0:
        g.replay()
        n += 1
        if n % 20 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    fwd_us = (time.time() - t0) / (n * 50) * 1e6
    print(json.dumps({"phase": "warm", "forward_us_sustained": round(fwd_us, 2)}), flush=True)
    ops.FUSE_PROJECTION = not ops.FUSE_PROJECTION
    g2 = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(g2):
        for _ in range(50):
            m(x, adj)
    g2.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(40):
        g2.replay()
    e1.record()
    e1.synchronize()
    fwd2 = e0.elapsed_time(e1) * 1e3 / (40 * 50)
    print(json.dumps({"phase": "warm", "fuse_projection": ops.FUSE_PROJECTION, "forward_us": round(fwd2, 2)}),
          flush=True)
    ops.FUSE_PROJECTION = not ops.FUSE_PROJECTION
    for k, fn in ops_.items():
        best, allr = time_graph(fn)
        print(json.dumps({"op": k, "us": round(best, 2), "all": [round(v, 2) for v in allr]}), flush=True)


if __name__ == "__main__":
    main()
