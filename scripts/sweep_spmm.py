"""Sweep SpMM schedules (ipc, lanes) on the GPU and time each with HIP events
around a hipGraph of back-to-back launches.  Prints one JSON line per case.

usage: python scripts/sweep_spmm.py [--big] [--reps 50]
"""
import argparse
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def time_graph(fn, reps, rounds=5):
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
    best = None
    for _ in range(rounds):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        best = us if best is None else min(best, us)
    return best


def time_eager(fn, reps, rounds=3):
    import torch
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(rounds):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        best = us if best is None else min(best, us)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--ipcs", default="4,8,16,32,64")
    ap.add_argument("--lanes", default="0,8,16,32")
    args = ap.parse_args()
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr, CSR

    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    cases = []
    A = as_csr(r8["adj"].to(dev))
    X = as_csr(r8["features"].to(dev))
    cases.append(("R8_A_F200", A, 200))
    cases.append(("R8_A_F8", A, 8))
    cases.append(("R8_X_F200", X, 200))
    ng = datasets.doc_topic_graph(18846, 70, 20, seed=0)
    cases.append(("20ng_A_F200", as_csr(ng["adj"].to(dev)), 200))
    if args.big:
        rp, ci, v = datasets.uniform_random_csr(1_000_000, 20_000_000, seed=0, device=dev)
        cases.append(("U1M20M_F256", CSR(rp, ci, v, (1_000_000, 1_000_000)), 256))

    # trivial-kernel floor inside a graph
    z = torch.zeros(1, device=dev)
    floor = time_graph(lambda: z.add_(1.0), args.reps)
    print(json.dumps({"case": "graph_floor_add_", "us": floor}), flush=True)

    for name, a, F in cases:
        M, K = a.shape
        B = torch.randn(K, F, device=dev)
        out = torch.empty(M, F, device=dev)
        bytes_ = 4 * (M + 1) + 8 * a.nnz + 4 * K * F + 4 * M * F
        # stock hipSPARSE through torch, for reference
        try:
            tcsr = torch.sparse_csr_tensor(a.rowptr.long(), a.colind.long(), a.val, (M, K))
            us = time_eager(lambda: torch.sparse.mm(tcsr, B), 20)
            print(json.dumps({"case": name, "impl": "torch.sparse.mm(hipSPARSE)", "us": us,
                              "GBs": bytes_ / us / 1e3}), flush=True)
        except Exception as exc:  # noqa: BLE001
            print(json.dumps({"case": name, "impl": "torch.sparse.mm", "error": str(exc)[:200]}), flush=True)
        for lanes, ipc in itertools.product([int(x) for x in args.lanes.split(",")],
                                            [int(x) for x in args.ipcs.split(",")]):
            try:
                us = time_graph(lambda: ops.spmm(a, B, out=out, ipc=ipc, lanes=lanes), args.reps)
                print(json.dumps({"case": name, "lanes": lanes, "ipc": ipc, "us": us, "GBs": bytes_ / us / 1e3,
                                  "nnz": a.nnz, "M": M, "F": F}), flush=True)
            except Exception as exc:  # noqa: BLE001
                print(json.dumps({"case": name, "lanes": lanes, "ipc": ipc, "error": str(exc)[:200]}), flush=True)


if __name__ == "__main__":
    main()
