"""One R8 eval forward timeline from a rocprofv3 kernel trace: run under
`rocprofv3 --kernel-trace --output-format csv -d DIR -- python scripts/fwd_trace.py`
(replays a hipGraph of 10 forwards 20 times; GCNK_TRACE_GRAPH=20ng traces the
BASELINE config-3 graph instead), then
`python scripts/fwd_trace.py --report DIR` prints, per kernel position in the
forward, its median duration and the median gap before it (us)."""
import argparse
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


FORWARDS, REPLAYS = 10, 20


def run():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets
    dev = torch.device("cuda", 0)
    if os.environ.get("GCNK_TRACE_GRAPH") == "20ng":
        g = datasets.doc_topic_graph(18846, 70, 20, seed=0)
        torch.manual_seed(1)
    else:
        g = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
        torch.manual_seed(0)
    m = GCN(nfeat=g["nfeat"], nhid=200, nclass=g["nclass"], dropout=0.5).to(dev).eval()
    x, adj = g["features"].to(dev), g["adj"].to(dev)
    with torch.no_grad():
        for _ in range(3):   # plan builds, then eager forwards (their kernel names are the trace's labels)
            m(x, adj)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(FORWARDS):
                m(x, adj)
        for _ in range(REPLAYS):
            g.replay()
        torch.cuda.synchronize()


def report(d):
    import csv
    import statistics
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    # the forward's kernel sequence: the period of the trace's last 50 kernels
    k = None
    for per in range(2, 12):
        tail = names[-5 * per:]
        if all(tail[i] == tail[i % per] for i in range(len(tail))):
            k = per
            break
    if k is None:
        print(json.dumps({"error": "no periodic forward found"}))
        return
    ng = FORWARDS * REPLAYS * k
    seq = rows[-ng:]
    # graph-replayed kernels can carry a blit's name in the trace: label each
    # position with the kernel the last eager forward launched there
    eager = [r["Kernel_Name"] for r in rows[-ng - k:-ng]] if len(rows) >= ng + k else []
    out = []
    for j in range(k):
        durs, gaps = [], []
        for i in range(j, len(seq), k):
            s, e = int(seq[i]["Start_Timestamp"]), int(seq[i]["End_Timestamp"])
            durs.append((e - s) / 1e3)
            if i > 0:
                gaps.append((s - int(seq[i - 1]["End_Timestamp"])) / 1e3)
        name = seq[j]["Kernel_Name"]
        if "rocclr" in name and len(eager) == k and "rocclr" not in eager[j]:
            name = eager[j] + " (by position; trace name: " + name[:40] + ")"
        out.append({"kernel": name[:160], "us": round(statistics.median(durs), 3),
                    "gap_before_us": round(statistics.median(gaps), 3) if gaps else None})
    per_fwd = [(int(seq[i + k - 1]["End_Timestamp"]) - int(seq[i]["Start_Timestamp"])) / 1e3
               for i in range(k, len(seq) - k, k)]
    res = {"kernels_per_forward": k, "forward_span_us_median": round(statistics.median(per_fwd), 3), "kernels": out}
    print(json.dumps(res, indent=1))
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--report")
    a = ap.parse_args()
    report(a.report) if a.report else run()
