"""Which steps of the hub factor's first build (factor.build on R8, the
largest piece of the first forward: setup_ms.first_forward_breakdown) cost
what in a fresh process: the build's statements re-run one at a time with a
synchronise after each, twice (first use, then warm).  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import _lib, datasets, factor, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    torch.zeros(1, device=dev)
    adj = as_csr(r8["adj"].to(dev))
    xop = ops.Operand(r8["features"].to(dev))
    torch.cuda.synchronize()
    out = []
    for rnd in range(2):
        t = {}

        def step(name, fn):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            t[name] = round((time.perf_counter() - t0) * 1e3, 3)
            return r
        M = adj.shape[0]
        rp, ci, v, nnz = adj.rowptr, adj.colind, adj.val, adj.nnz
        deg = step("deg_diff", lambda: rp[1:] - rp[:-1])
        hubs = step("nonzero", lambda: torch.nonzero(deg >= 64).flatten())
        H = int(hubs.numel())
        is_hub = step("zeros_bool_index_put", lambda: torch.zeros(M, dtype=torch.bool, device=dev).index_fill_(0, hubs, True))
        rows = step("repeat_interleave", lambda: torch.repeat_interleave(torch.arange(M, device=dev, dtype=torch.int32),
                                                                         deg, output_size=nnz))
        step("struct_check_any", lambda: bool((~is_hub[rows] & ~is_hub[ci.long()] & (ci != rows)).any()))
        x = xop.csr
        xrows = step("x_repeat_interleave", lambda: torch.repeat_interleave(
            torch.arange(x.shape[0], device=dev, dtype=torch.int32), x.rowptr[1:] - x.rowptr[:-1], output_size=x.nnz))
        sel = step("x_select", lambda: ~is_hub[xrows.long()] & (x.val != 0))
        cols = step("x_masked_select", lambda: x.colind[sel])
        step("minmax_cpu", lambda: [int(q) for q in torch.stack([cols.min(), cols.max()]).cpu()])
        step("hubs_cpu", lambda: hubs.cpu().numpy())
        step("cumsum_int64", lambda: torch.cumsum(is_hub[ci.long()].to(torch.int32), 0))
        step("index_put_dense", lambda: torch.zeros((M, 52), device=dev).index_put_(
            (xrows[sel].long(), (cols - cols.min()).long()), x.val[sel]))
        step("factor_build_total", lambda: factor.build(adj, xop))
        out.append(t)
        del deg, hubs, is_hub, rows, xrows, sel, cols
    print(json.dumps({"first": out[0], "warm": out[1], "lib": os.path.basename(_lib.LIB_PATH),
                      "np": np.__version__}), flush=True)


if __name__ == "__main__":
    main()
