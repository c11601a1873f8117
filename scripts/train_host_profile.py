"""Host-side profile (cProfile) of eager R8 training steps, factored gc1 on and
off (ops.FACTOR_GC1): where the eager step's host time goes."""
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
    tgt = torch.as_tensor(r8["target"]).long().to(dev)
    idx = torch.as_tensor(r8["train_lst"]).long().to(dev)
    for fac in (True, False):
        ops.FACTOR_GC1 = fac
        torch.manual_seed(0)
        model = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5, dropout_rng="device").to(dev)
        opt = torch.optim.Adam(model.parameters(), lr=0.02)
        crit = torch.nn.CrossEntropyLoss()

        def step():
            model.train()
            opt.zero_grad()
            loss = crit(model(x, adj)[idx], tgt[idx])
            loss.backward()
            opt.step()

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        pr.disable()
        print(f"factored={fac}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/step (profiled)", flush=True)
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
        print(s.getvalue()[:6000], flush=True)


if __name__ == "__main__":
    main()
