"""Time the R8 A-hat SpMM (F = 200) on row subsets: light rows only, heavy rows
only, and all rows, to see which part bounds the launch.  One JSON line each."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr, CSR
    from sweep_spmm import time_graph

    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    A = as_csr(r8["adj"].to(dev))
    rp, ci, v = A.rowptr.cpu().long(), A.colind.cpu(), A.val.cpu()
    deg = rp[1:] - rp[:-1]
    M, K = A.shape
    F = int(os.environ.get("F", 200))

    def subset(keep):
        kk = keep.repeat_interleave(deg)
        nd = torch.where(keep, deg, torch.zeros_like(deg))
        nrp = torch.zeros(M + 1, dtype=torch.long)
        nrp[1:] = torch.cumsum(nd, 0)
        return CSR(nrp.int().to(dev), ci[kk].to(dev), v[kk].to(dev), (M, K))

    B = torch.randn(K, F, device=dev)
    out = torch.empty(M, F, device=dev)
    for thr in (32, 64, 128, 512):
        for name, a in ((f"light<= {thr}", subset(deg <= thr)), (f"heavy> {thr}", subset(deg > thr))):
            us = time_graph(lambda: ops.spmm(a, B, out=out), 100)
            print(json.dumps({"subset": name, "nnz": a.nnz, "rows": int((a.rowptr[1:] != a.rowptr[:-1]).sum()),
                              "us": us}), flush=True)
    us = time_graph(lambda: ops.spmm(A, B, out=out), 100)
    print(json.dumps({"subset": "all", "nnz": A.nnz, "us": us}), flush=True)
    e = torch.empty(0, device=dev)
    print(json.dumps({"degree_hist": torch.histc(deg.float(), bins=16, min=0, max=2048).int().tolist(),
                      "max_deg": int(deg.max())}))


if __name__ == "__main__" and not os.environ.get("STAMPS"):
    main()


def stamps_heavy():
    """Per-workgroup stamps of the heavy-only subset (all its workgroups are heavy segments)."""
    import numpy as np
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import _lib, datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr, CSR
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    A = as_csr(r8["adj"].to(dev))
    rp, ci, v = A.rowptr.cpu().long(), A.colind.cpu(), A.val.cpu()
    deg = rp[1:] - rp[:-1]
    M, K = A.shape
    keep = deg > 32
    kk = keep.repeat_interleave(deg)
    nd = torch.where(keep, deg, torch.zeros_like(deg))
    nrp = torch.zeros(M + 1, dtype=torch.long)
    nrp[1:] = torch.cumsum(nd, 0)
    a = CSR(nrp.int().to(dev), ci[kk].to(dev), v[kk].to(dev), (M, K))
    B = torch.randn(K, 200, device=dev)
    out = torch.empty(M, 200, device=dev)
    for _ in range(5):
        ops.spmm(a, B, out=out)
    torch.cuda.synchronize()
    buf = torch.zeros(4 * 100000, dtype=torch.int64, device=dev)
    lib.gcnk_debug_set_stamps(buf.data_ptr())
    ops.spmm(a, B, out=out)
    torch.cuda.synchronize()
    lib.gcnk_debug_set_stamps(None)
    s = buf.view(-1, 4).cpu().numpy().astype(np.float64)
    s = s[(s[:, 0] > 0) & (s[:, 3] > 0)]
    s = (s - s[:, 0].min()) / 100.0
    d = np.diff(s, axis=1)
    pct = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 50, 90, 100)]
    print(json.dumps({"wgs": len(s), "entry": pct(s[:, 0]), "unit": pct(d[:, 0]), "walk": pct(d[:, 1]),
                      "tail": pct(d[:, 2]), "end": pct(s[:, 3])}))
    order = np.argsort(-s[:, 3])[:8]
    print(json.dumps({"latest": [[round(x, 2) for x in s[i]] for i in order]}))
    # per-workgroup walk time against grid position and segment (plan units: heavy region first)
    pl = list(a._plans.values())[-1]
    hdr = pl.header
    nnz, nh = hdr[13], hdr[6]
    words = pl.buf.view(torch.int32).cpu().numpy() if hasattr(pl, "buf") else None
    raw = buf.view(-1, 4).cpu().numpy().astype(np.float64)[:nh]
    ok = (raw[:, 0] > 0) & (raw[:, 3] > 0)
    t0 = raw[ok, 0].min()
    st = (raw - t0) / 100.0
    walk = st[:, 2] - st[:, 1]
    if words is not None:
        uoff = (16 + 2 * nnz + 3) & ~3
        units = words[uoff:uoff + 4 * nh].reshape(nh, 4)
        seglen = units[:, 2] - units[:, 1]
        idx = np.where(ok)[0]
        slow = idx[np.argsort(-walk[idx])[:12]]
        print(json.dumps({"slowest_walks": [[int(b), int(b % 8), int(units[b, 0]), int(seglen[b]), round(float(st[b, 0]), 2),
                                              round(float(walk[b]), 2)] for b in slow],
                          "walk_by_xcd_p90": [round(float(np.percentile(walk[idx[idx % 8 == c]], 90)), 2) for c in range(8)],
                          "walk_by_position_decile_p50": [round(float(np.median(walk[idx[(idx * 10) // nh == q]])), 2)
                                                          for q in range(10)]}))


if __name__ == "__main__" and os.environ.get("STAMPS"):
    stamps_heavy()
