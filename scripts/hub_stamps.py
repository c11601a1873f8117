"""In-kernel timeline of the hub-plan SpMM (needs a stamps build:
make -C <pkg>/csrc variant NAME=stamps DEFS=-DGCNK_STAMPS, then
GCNK_LIB=_variants/libgcnk_stamps.so).  s_memrealtime (100 MHz) per
workgroup: group kernel entry / loads landed in LDS / outputs stored (after a
barrier); sum kernel entry / partials summed / stored.  Prints percentiles
(us) per phase, times relative to the first group-kernel entry."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(x):
    import numpy as np
    return {k: round(float(np.percentile(x, q)), 3) for k, q in (("p0", 0), ("p10", 10), ("p50", 50), ("p90", 90),
                                                                   ("p100", 100))}


def main():
    import numpy as np
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import _lib, datasets, ops
    from graph_convolutional_networks_for_text_classification_amd import sparse as sp
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    A = sp.as_csr(r8["adj"].to(dev))
    M = A.shape[0]
    for br in [int(x) for x in (sys.argv[1:] or ["0"])]:
        sp.HUB_MIN, sp.HUB_BLOCK_ROWS = 0, br
        for F in [int(x) for x in os.environ.get("STAMP_WIDTHS", "200,8").split(",")]:
            nsets = max(2, -(-300_000_000 // (8 * M * F)))
            Bs = [torch.randn(M, F, device=dev) for _ in range(nsets)]
            Cs = [torch.empty(M, F, device=dev) for _ in range(nsets)]
            bias = torch.randn(F, device=dev)
            for i in range(nsets):
                ops.spmm(A, Bs[i], bias=bias, epilogue=_lib.EPI_BIAS_RELU, out=Cs[i])
            torch.cuda.synchronize()
            plan = [p for k, p in A._plans.items() if k[4] == br and k[1] == lib.gcnk_spmm_groups(F, 0)][-1]
            h = plan.header
            G, H = h[4], h[6]
            buf = torch.zeros(4 * (G * 64 + H * 16), dtype=torch.int64, device=dev)
            rows = []
            for rep in range(5):   # cold: a fresh operand set each time
                buf.zero_()
                assert lib.gcnk_debug_set_stamps(buf.data_ptr()) == 0
                ops.spmm(A, Bs[rep + 1], bias=bias, epilogue=_lib.EPI_BIAS_RELU, out=Cs[rep + 1])
                torch.cuda.synchronize()
                lib.gcnk_debug_set_stamps(None)
                s = buf.view(-1, 4).cpu().numpy().astype(np.float64)
                nz = np.flatnonzero(s[:, 0] > 0)
                rows.append(s)
            s = rows[-1]
            used = s[:, 0] > 0
            # group blocks first (G x slices: ~8 column vectors per slice), then the sum blocks
            Q = F // 4 if F % 4 == 0 else F
            ng = G * max(1, -(-Q // 8))
            gk = s[:ng]
            sk = s[ng:][used[ng:]]
            assert used[:ng].all()
            t0 = gk[:, 0].min()
            res = {"F": F, "block_rows": br, "G": G, "group_blocks": ng, "sum_blocks": len(sk),
                   "g_entry": pct((gk[:, 0] - t0) / 100), "g_loads": pct((gk[:, 1] - gk[:, 0]) / 100),
                   "g_compute": pct((gk[:, 2] - gk[:, 1]) / 100), "g_arrive": pct((gk[:, 2] - t0) / 100),
                   "g_exit": pct((gk[:, 3] - t0) / 100), "g_combine": pct((gk[:, 3] - gk[:, 2]) / 100)}
            # per slice: last arrival and last exit
            ns = max(1, ng // G)
            arr = (gk[:, 2] - t0).reshape(ns, G) / 100
            ext = (gk[:, 3] - t0).reshape(ns, G) / 100
            res["slice_last_arrival"] = [round(float(x), 2) for x in arr.max(1)]
            res["slice_last_exit"] = [round(float(x), 2) for x in ext.max(1)]
            order = np.argsort(arr, axis=1)
            res["combine_us_by_rank_from_last"] = [round(float(np.median((ext - arr)[np.arange(ns), order[:, -1 - k]])), 2)
                                                   for k in range(min(G, 9))]
            if len(sk):
                res.update({"s_entry": pct((sk[:, 0] - t0) / 100), "s_sum": pct((sk[:, 1] - sk[:, 0]) / 100),
                            "s_end": pct((sk[:, 2] - t0) / 100)})
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
