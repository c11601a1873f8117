"""Streaming floor for an op of the north-star's size: torch's vectorised copy
of a [7724 x 200] fp32 tensor (6.2 MB read + 6.2 MB written, the compulsory
traffic of R8 A-hat x S1 minus the CSR), warm (one pair) and cold (rotating
> 256 MB of distinct pairs, as the north-star measurement does).  Run under
rocprofv3 --kernel-trace --stats for kernel durations."""
import argparse
import json

import torch


def graph_us(fns, reps):
    for f in fns:
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    n = 0
    with torch.cuda.graph(g):
        for _ in range(reps):
            for f in fns:
                f()
                n += 1
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=7724)
    ap.add_argument("--cols", type=int, default=200)
    ap.add_argument("--mode", default="cold")
    a = ap.parse_args()
    M, F = a.rows, a.cols
    nsets = max(2, -(-300_000_000 // (8 * M * F)))
    Bs = [torch.randn(M, F, device="cuda") for _ in range(nsets)]
    Cs = [torch.empty(M, F, device="cuda") for _ in range(nsets)]
    if a.mode == "cold":
        us = graph_us([(lambda i=i: Cs[i].copy_(Bs[i])) for i in range(nsets)], max(1, 200 // nsets))
    else:
        us = graph_us([lambda: Cs[0].copy_(Bs[0])], 200)
    print(json.dumps({"op": "copy", "rows": M, "cols": F, "mode": a.mode, "hip_events_us": round(us, 3),
                      "bytes": 8 * M * F}))


if __name__ == "__main__":
    main()
