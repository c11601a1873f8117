"""R8 training-step timing: one step of trainer.py:354-361
(model.train(), zero_grad, forward, cross-entropy on the training nodes,
backward, Adam step) through the HIP drop-in, next to the oracle's torch-CPU
step (the reference's own ATen calls) on this host's cores.

Prints one JSON line per case.  Eager launches (the training loop is eager in
the reference too); GPU times are HIP events around `--steps` steps.

usage: python scripts/bench_train.py [--steps 50] [--cpu-steps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--cpu-steps", type=int, default=5)
    args = ap.parse_args()

    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets
    from oracle import gcn_ref

    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    nfeat, nclass = r8["nfeat"], r8["nclass"]
    target = torch.as_tensor(r8["target"]).long()
    tr = torch.as_tensor(r8["train_lst"]).long()

    def run(model, x, adj, tgt, idx, steps, sync):
        opt = torch.optim.Adam(model.parameters(), lr=0.02)
        crit = torch.nn.CrossEntropyLoss()

        def step():
            model.train()
            opt.zero_grad()
            logits = model(x, adj)
            loss = crit(logits[idx], tgt[idx])
            loss.backward()
            opt.step()
            return loss

        for _ in range(3):
            step()
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        sync()
        return (time.perf_counter() - t0) / steps * 1e3

    x, adj = r8["features"].to(dev), r8["adj"].to(dev)
    for rng in ("cpu", "device"):
        torch.manual_seed(0)
        model = GCN(nfeat=nfeat, nhid=200, nclass=nclass, dropout=0.5, dropout_rng=rng).to(dev)
        ms = run(model, x, adj, target.to(dev), tr.to(dev), args.steps, torch.cuda.synchronize)
        print(json.dumps({"case": "R8 train step (fwd + bwd + Adam)", "impl": f"HIP, dropout_rng={rng}",
                          "ms_per_step": round(ms, 4), "steps": args.steps}), flush=True)

    # the same step (dropout_rng="device") captured once in a hipGraph and replayed:
    # launch-overhead-free kernel time of a training step.  The hash offset lives
    # on the device and the captured forward advances it, so every replay trains
    # on a fresh mask (checked below: the stream position moves one step per replay).
    torch.manual_seed(0)
    model = GCN(nfeat=nfeat, nhid=200, nclass=nclass, dropout=0.5, dropout_rng="device").to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.02, capturable=True)
    crit = torch.nn.CrossEntropyLoss()
    tgt, idx = target.to(dev), tr.to(dev)
    model.train()

    def step():
        opt.zero_grad(set_to_none=False)
        loss = crit(model(x, adj)[idx], tgt[idx])
        loss.backward()
        opt.step()
        return loss

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.cuda.synchronize()
    base0 = int(model._rng_base.item())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        g.replay()
    e1.record()
    e1.synchronize()
    advanced = (int(model._rng_base.item()) - base0) // (r8["nodes"] * 200)
    print(json.dumps({"case": "R8 train step (fwd + bwd + Adam)", "impl": "HIP, dropout_rng=device, hipGraph replay",
                      "ms_per_step": round(e0.elapsed_time(e1) / args.steps, 4), "steps": args.steps,
                      "fresh_masks": advanced == args.steps}), flush=True)

    if args.cpu_steps > 0:
        torch.manual_seed(0)
        ref = gcn_ref.RefGCN(nfeat=nfeat, nhid=200, nclass=nclass, dropout=0.5)
        ms = run(ref, r8["features"], r8["adj"], target, tr, args.cpu_steps, lambda: None)
        print(json.dumps({"case": "R8 train step (fwd + bwd + Adam)", "impl": "oracle torch-CPU (reference ATen calls)",
                          "threads": torch.get_num_threads(), "ms_per_step": round(ms, 2),
                          "steps": args.cpu_steps}), flush=True)


if __name__ == "__main__":
    main()
