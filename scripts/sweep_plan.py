"""Per-op time of the R8 SpMMs under different dense-block thresholds (plan
variants), from a hipGraph of back-to-back launches timed with HIP events."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr

    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    A = as_csr(r8["adj"].to(dev))
    X = as_csr(r8["features"].to(dev))
    reps = 100
    for name, a in (("A", A), ("X", X)):
        for F in (200, 8):
            B = torch.randn(a.shape[1], F, device=dev)
            out = torch.empty(a.shape[0], F, device=dev)
            for thr in (2.0, 0.5, 0.25, 0.1, 0.05):
                fn = lambda: ops.spmm(a, B, out=out, dense=thr)  # noqa: E731
                fn()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(reps):
                        fn()
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                best = 1e9
                for _ in range(5):
                    e0.record(); g.replay(); e1.record(); e1.synchronize()
                    best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
                hdr = [p for k, p in a._plans.items() if k[2] == float(thr)][-1].header
                print(json.dumps({"op": name, "F": F, "thr": thr, "us": round(best, 2), "ntile": hdr[8], "nred": hdr[9],
                                  "nunits": hdr[5], "nhunits": hdr[6], "diag": hdr[12]}), flush=True)
                del g


if __name__ == "__main__":
    main()
