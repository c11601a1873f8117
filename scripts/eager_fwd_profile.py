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
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets, ops
    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    x, adj = r8["features"].to(dev), r8["adj"].to(dev)
    torch.manual_seed(0)
    model = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(dev).eval()
    with torch.no_grad():
        for use in (False, True):          # op by op, then the whole-forward record (record.py)
            ops.USE_RECORD = use
            for _ in range(20):
                model(x, adj)
            torch.cuda.synchronize()
            n = 200
            t0 = time.perf_counter()
            for _ in range(n):
                model(x, adj)
            torch.cuda.synchronize()
            print(f"eager forward ({'record' if use else 'op by op'}): {(time.perf_counter() - t0) / n * 1e6:.1f} us",
                  flush=True)
    # the training-step pattern of trainer.py:353-362 (forward + CE + backward + Adam), eager
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=0.02)
    tgt = torch.zeros(r8["nodes"], dtype=torch.int64, device=dev)
    tgt[:len(r8["target"])] = torch.from_numpy(r8["target"]).to(dev)
    idx = torch.arange(len(r8["target"]), device=dev)
    for use in (False, True):
        ops.USE_RECORD = use
        for rng in ("cpu", "device"):
            model.dropout_rng = rng
            for _ in range(10):
                opt.zero_grad()
                lg = model(x, adj)
                torch.nn.functional.cross_entropy(lg[idx], tgt[idx]).backward()
                opt.step()
            torch.cuda.synchronize()
            n = 100
            t0 = time.perf_counter()
            for _ in range(n):
                opt.zero_grad()
                lg = model(x, adj)
                torch.nn.functional.cross_entropy(lg[idx], tgt[idx]).backward()
                opt.step()
            torch.cuda.synchronize()
            print(f"eager train step ({'record' if use else 'op by op'}, dropout {rng}): "
                  f"{(time.perf_counter() - t0) / n * 1e3:.3f} ms", flush=True)
    model.eval()
    ops.USE_RECORD = True
    with torch.no_grad():
        n = 200
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
