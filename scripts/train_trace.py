"""Kernel breakdown of one R8 training step (trainer.py:354-361: train mode,
zero_grad, forward, cross-entropy on the training nodes, backward, Adam) from
a rocprofv3 kernel trace.  Run under

  rocprofv3 --kernel-trace --output-format csv -d DIR -- python scripts/train_trace.py

(EAGER eager steps, then a hipGraph of one step replayed REPLAYS times), then
`python scripts/train_trace.py --report DIR` prints, per launch position of
the step, the median duration in the eager steps and in the graph replays
(graph-replayed kernels can carry a blit's name in the trace: each position is
labelled with the kernel the last eager step launched there), the kernel sum
and span of a step, and the slowest kernels of the backward."""
import argparse
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

EAGER, REPLAYS = 20, 30


def run():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets
    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    x, adj = r8["features"].to(dev), r8["adj"].to(dev)
    tgt = torch.as_tensor(r8["target"]).long().to(dev)
    idx = torch.as_tensor(r8["train_lst"]).long().to(dev)
    torch.manual_seed(0)
    model = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5, dropout_rng="device").to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.02, capturable=True)
    crit = torch.nn.CrossEntropyLoss()
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
        for _ in range(3 + EAGER):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(REPLAYS):
        g.replay()
    torch.cuda.synchronize()


def _period(names, lo=2, hi=400, reps=4):
    for per in range(lo, min(hi, len(names) // reps) + 1):
        tail = names[-reps * per:]
        if all(tail[i] == tail[i % per] for i in range(len(tail))):
            return per
    return None


def _positions(seq, k):
    out = []
    for j in range(k):
        durs = [(int(seq[i]["End_Timestamp"]) - int(seq[i]["Start_Timestamp"])) / 1e3 for i in range(j, len(seq), k)]
        out.append(statistics.median(durs))
    return out


def _spans(seq, k):
    return [(int(seq[i + k - 1]["End_Timestamp"]) - int(seq[i]["Start_Timestamp"])) / 1e3
            for i in range(0, len(seq) - k + 1, k)]


def report(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            import csv
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    k = _period(names)
    if k is None:
        res = {"error": "no periodic graph replay found"}
        print(json.dumps(res))
        return res
    graph = rows[-REPLAYS * k:]
    before = rows[:-REPLAYS * k]
    ke = _period([r["Kernel_Name"] for r in before])
    eager = before[-(EAGER - 2) * ke:] if ke else []
    g_us = _positions(graph, k)
    e_us = _positions(eager, ke) if ke == k else None
    labels = [r["Kernel_Name"] for r in eager[-k:]] if ke == k else [r["Kernel_Name"] for r in graph[:k]]
    kernels = []
    for j in range(k):
        kernels.append({"pos": j, "kernel": labels[j][:150], "graph_us": round(g_us[j], 3),
                        "eager_us": round(e_us[j], 3) if e_us else None})
    res = {"kernels_per_step": k, "eager_kernels_per_step": ke,
           "graph_step_span_us_median": round(statistics.median(_spans(graph, k)), 3),
           "graph_kernel_sum_us": round(sum(g_us), 3),
           "eager_step_span_us_median": round(statistics.median(_spans(eager, ke)), 3) if ke else None,
           "eager_kernel_sum_us": round(sum(e_us), 3) if e_us else None,
           "slowest": sorted(kernels, key=lambda e: -e["graph_us"])[:12], "kernels": kernels}
    print(json.dumps(res, indent=1))
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--report")
    a = ap.parse_args()
    report(a.report) if a.report else run()
