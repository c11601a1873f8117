"""In-kernel timeline of the R8 X W1 product (the MFMA tile path: document
blocks + the split-K chunks of the 50 dense topic rows, then the slab reduce).
Needs the stamps build (make -C <pkg>/csrc variant NAME=stamps
DEFS=-DGCNK_STAMPS; GCNK_LIB=_variants/libgcnk_stamps.so).  Tile kernel stamps:
0 entry, 1 B chunk staged in LDS, 2 MFMAs done, 3 stored.  Percentiles in us
relative to the first entry, single-chunk (document) and multi-chunk (topic)
workgroups apart.
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
    X = sp.as_csr(r8["features"].to(dev))
    nsets = 28              # cold: operand sets span > the 256 MB MALL
    Ws = [torch.randn(r8["nfeat"], 200, device=dev) for _ in range(nsets)]
    outs = [torch.empty(X.shape[0], 200, device=dev) for _ in range(nsets)]
    for i in range(nsets):
        ops.spmm(X, Ws[i], out=outs[i])
    torch.cuda.synchronize()
    W, out = Ws[1], outs[1]
    h = list(X._plans.values())[-1].header
    ntile, nsingle = int(h[8]), int(h[15])
    buf = torch.zeros(4 * 65536, dtype=torch.int64, device=dev)
    assert lib.gcnk_debug_set_stamps(buf.data_ptr()) == 0
    ops.spmm(X, W, out=out)
    torch.cuda.synchronize()
    lib.gcnk_debug_set_stamps(None)
    s = buf.view(-1, 4).cpu().numpy().astype(np.float64)
    used = np.nonzero(s[:, 0] > 0)[0]
    s = s[: used.max() + 1]
    idx = np.arange(len(s))
    t0 = s[used, 0].min()
    slices = 2                                         # F = 200: 13 n-tiles in slices of <= 8
    per = 8 * slices
    item = (idx // per) * 8 + (idx % 8)                # the kernel's XCD-aware workgroup order
    single = item < nsingle
    res = {"hdr": h, "workgroups": int(len(used)), "span_us": round(float((s[used][:, 1:].max() - t0) / 100), 3)}
    for name, m in (("doc_single", single), ("topic_multi", ~single)):
        a = s[m & (s[:, 0] > 0)]
        res[name] = {"n": int(len(a)), "entry": pct((a[:, 0] - t0) / 100), "stage": pct((a[:, 1] - a[:, 0]) / 100),
                     "mfma": pct((a[:, 2] - a[:, 1]) / 100), "store": pct((a[:, 3] - a[:, 2]) / 100),
                     "end": pct((a[:, 3] - t0) / 100)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
