"""Host-side profile (cProfile) of the eager R8 eval forward (trainer.py:357's
pattern, no graph): which Python frames the ~85 us per forward go to."""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets
    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    x, adj = r8["features"].to(dev), r8["adj"].to(dev)
    torch.manual_seed(0)
    model = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(dev).eval()
    with torch.no_grad():
        for _ in range(20):
            model(x, adj)
        torch.cuda.synchronize()
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            model(x, adj)
        torch.cuda.synchronize()
        print(f"eager forward: {(time.perf_counter() - t0) / n * 1e6:.1f} us", flush=True)
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(n):
            model(x, adj)
        torch.cuda.synchronize()
        pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue()[:7000], flush=True)


if __name__ == "__main__":
    main()
