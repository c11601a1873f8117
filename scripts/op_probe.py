"""Warm per-call time (hipGraph of back-to-back launches) of one R8 forward
op, checked against the float64 oracle.  One JSON line.

  python scripts/op_probe.py --op XW1|AS1|AS1P|H1W2|AS2 [--reps 200]

AS1P: A S1 + b1, ReLU with H1 W2 fused into the epilogue (ops.spmm_proj, H1
not stored: the eval forward's schedule under FUSE_PROJECTION).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="XW1")
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import numpy as np
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import _lib, datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    from oracle import csr_ref
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from hub_probe import time_graph

    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    a, x = as_csr(r8["adj"].to(dev)), as_csr(r8["features"].to(dev))
    g = torch.Generator().manual_seed(0)
    W1 = (torch.rand(r8["nfeat"], 200, generator=g) - 0.5).to(dev)
    W2 = (torch.rand(200, r8["nclass"], generator=g) - 0.5).to(dev)
    S1 = torch.rand(r8["nodes"], 200, generator=g).to(dev)
    S2 = torch.rand(r8["nodes"], r8["nclass"], generator=g).to(dev)
    if args.op == "XW1":
        op, B, out = x, W1, torch.empty(r8["nodes"], 200, device=dev)
        fn = lambda: ops.spmm(x, W1, out=out)  # noqa: E731
    elif args.op == "AS1":
        op, B, out = a, S1, torch.empty(r8["nodes"], 200, device=dev)
        fn = lambda: ops.spmm(a, S1, out=out)  # noqa: E731
    elif args.op == "AS1P":
        op, B, out = a, S1, torch.empty(r8["nodes"], r8["nclass"], device=dev)
        b1 = (torch.rand(200, generator=g) - 0.5).to(dev)

        def fn():
            nonlocal out
            _, out = ops.spmm_proj(a, S1, W2, bias=b1, epilogue=_lib.EPI_BIAS_RELU, store_main=False)
    elif args.op == "AS2":
        op, B, out = a, S2, torch.empty(r8["nodes"], r8["nclass"], device=dev)
        fn = lambda: ops.spmm(a, S2, out=out)  # noqa: E731
    else:
        op, B, out = None, None, torch.empty(r8["nodes"], r8["nclass"], device=dev)
        fn = lambda: ops.gemm(S1, W2, out=out)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    if op is not None:
        rp, ci, v = (t.cpu().numpy() for t in (op.rowptr, op.colind, op.val))
        ref = csr_ref.spmm_csr(rp, ci, v, B.cpu().numpy())
        if args.op == "AS1P":
            ref = np.maximum(ref + b1.cpu().double().numpy(), 0.0) @ W2.cpu().double().numpy()
    else:
        ref = S1.cpu().double().numpy() @ W2.cpu().double().numpy()
    err = float(np.abs(out.cpu().double().numpy() - ref).max())
    us = time_graph([fn], args.reps)
    hdr = list(list(op._plans.values())[-1].header) if op is not None else None
    print(json.dumps({"op": args.op, "warm_us": round(us, 3), "max_err": err, "hdr": hdr}), flush=True)


if __name__ == "__main__":
    main()
