"""BASELINE config 4 (uniform 1M nodes / 20M edges, F = 256): the SpMM in one
pass against column-blocked passes (w-column slices of B and C, one launch
per slice; a slice of B is 1M x w x 4 B, so at w <= 64 it fits the 256 MB
Infinity Cache and the gathers of a pass are served on-die).  Event-timed
best of 5, checked against the full-width result.

  python scripts/colblock_probe.py [--widths 256,128,64,32]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--widths", default="256,128,64,32")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--nnz", type=int, default=20_000_000)
    args = ap.parse_args()
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import CSR
    dev = torch.device("cuda", 0)
    rp, ci, v = datasets.uniform_random_csr(args.n, args.nnz, seed=0, device=dev)
    big = CSR(rp, ci, v, (args.n, args.n))
    F = 256
    B = torch.randn(args.n, F, device=dev)
    ref = torch.empty(args.n, F, device=dev)
    ops.spmm(big, B, out=ref)
    torch.cuda.synchronize()
    nbytes = 4 * (args.n + 1) + 8 * big.nnz + 8 * args.n * F
    for w in (int(x) for x in args.widths.split(",")):
        C = torch.empty(args.n, F, device=dev)

        def run():
            for c in range(0, F, w):
                ops.spmm(big, B[:, c:c + w], out=C[:, c:c + w])
        run()
        torch.cuda.synchronize()
        ok = bool(torch.equal(C, ref))
        best = None
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        print(json.dumps({"width": w, "passes": F // w, "ms": round(best, 4), "equal_full": ok,
                          "frac": nbytes / (best * 1e-3) / 8e12,
                          "edges_per_s": big.nnz / (best * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
