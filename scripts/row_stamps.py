"""In-kernel timeline of the row-unit SpMM on the R8 adjacency (needs the
stamps build: make -C <pkg>/csrc variant NAME=stamps DEFS=-DGCNK_STAMPS, then
GCNK_LIB=_variants/libgcnk_stamps.so).  s_memrealtime (100 MHz) per
workgroup: 0 entry, 1 unit descriptor(s) loaded, 2 gathers summed, 3 stored /
counted in (a heavy row's last arriver overwrites 3 when its row is stored).
Percentiles in us relative to the first entry, heavy-segment blocks and light
blocks apart; one JSON line per width.

  GCNK_LIB=_variants/libgcnk_stamps.so python scripts/row_stamps.py [F ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(x):
    import numpy as np
    if len(x) == 0:
        return None
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
    for F in [int(x) for x in (sys.argv[1:] or ["200"])]:
        # cold: a fresh operand set per timed call (sets span > the 256 MB MALL)
        nsets = max(7, -(-300_000_000 // (8 * A.shape[0] * F)))
        Bs = [torch.randn(A.shape[1], F, device=dev) for _ in range(nsets)]
        outs = [torch.empty(A.shape[0], F, device=dev) for _ in range(nsets)]
        bias = torch.randn(F, device=dev)
        for i in range(nsets):
            ops.spmm(A, Bs[i], bias=bias, epilogue=_lib.EPI_BIAS_RELU, out=outs[i])
        torch.cuda.synchronize()
        plan = list(A._plans.values())[-1]
        h = plan.header
        buf = torch.zeros(4 * 65536, dtype=torch.int64, device=dev)
        runs = []
        for rep in range(5):
            buf.zero_()
            assert lib.gcnk_debug_set_stamps(buf.data_ptr()) == 0
            ops.spmm(A, Bs[rep + 1], bias=bias, epilogue=_lib.EPI_BIAS_RELU, out=outs[rep + 1])
            torch.cuda.synchronize()
            lib.gcnk_debug_set_stamps(None)
            runs.append(buf.view(-1, 4).cpu().numpy().astype(np.float64))
        s = runs[-1]
        used = np.nonzero(s[:, 0] > 0)[0]
        s = s[: used.max() + 1]
        t0 = s[used, 0].min()
        # heavy blocks come first in grid.x: one per heavy unit (whole-wave groups)
        nheavy = int((s[:, 1] > 0).sum())  # placeholder count of blocks with a descriptor stamp
        nhb = int(h[6]) if h[3] == 1 else 0
        hv, lt = s[:nhb], s[nhb:]
        hv = hv[hv[:, 0] > 0]
        lt = lt[lt[:, 0] > 0]
        rel = lambda a, k: (a[:, k] - t0) / 100  # noqa: E731
        res = {"F": F, "hdr": h, "blocks": int(len(used)), "heavy_blocks": int(len(hv)), "light_blocks": int(len(lt)),
               "with_descriptor": nheavy,
               "span_us": round(float((s[used][:, 1:].max() - t0) / 100), 3),
               "heavy": {"entry": pct(rel(hv, 0)), "desc": pct((hv[:, 1] - hv[:, 0]) / 100),
                         "gather": pct((hv[:, 2] - hv[:, 1]) / 100), "to_3": pct((hv[:, 3] - hv[:, 2]) / 100),
                         "end": pct(rel(hv, 3))},
               "light": {"entry": pct(rel(lt, 0)), "desc": pct((lt[:, 1] - lt[:, 0]) / 100),
                         "gather": pct((lt[:, 2] - lt[:, 1]) / 100), "store": pct((lt[:, 3] - lt[:, 2]) / 100),
                         "end": pct(rel(lt, 3))}}
        spans = []
        for r in runs:
            u = r[r[:, 0] > 0]
            spans.append(round(float((u[:, 1:].max() - u[:, 0].min()) / 100), 3))
        res["spans_us"] = spans
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
