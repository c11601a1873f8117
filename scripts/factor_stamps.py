"""In-kernel timeline of the hub-factored gc1 kernel (csrc/factor.hip) on R8
(needs the stamps build: make -C <pkg>/csrc variant NAME=stamps DEFS=-DGCNK_STAMPS,
then GCNK_LIB=_variants/libgcnk_stamps.so).  Per workgroup s_memrealtime
(100 MHz): 0 operands staged, 1 U W1 MFMA done, 2 epilogue done, 3 exit; percentiles in
us from the first entry, cold (a fresh W1 / output set per call)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import _lib, datasets, factor, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    if os.environ.get("GCNK_STAMP_GRAPH") == "20ng":     # BASELINE config 3's shape: 70 hubs, 20 classes
        r8 = datasets.doc_topic_graph(18846, 70, 20, seed=0)
    else:
        r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    A, X = r8["adj"].to(dev), r8["features"].to(dev)
    f = factor.get(as_csr(A), ops.Operand(X))
    print(json.dumps({"M": f.M, "H": f.H, "Kc": f.Kc, "rec_words": f.rec_words, "nblk": f.nblk}), flush=True)
    W1s = [torch.randn(r8["nfeat"], 200, device=dev) * 0.05 for _ in range(8)]
    W2 = torch.randn(200, r8["nclass"], device=dev) * 0.1
    b1 = torch.randn(200, device=dev) * 0.1
    for W1 in W1s:
        ops.hubfactor_gc1(f, W1, b1, W2, store_h1=False)
    torch.cuda.synchronize()
    buf = torch.zeros(4 * 8192, dtype=torch.int64, device=dev)
    for rep in range(4):
        S = f.hub_times(W1s[rep + 1])
        torch.cuda.synchronize()
        buf.zero_()
        assert lib.gcnk_debug_set_stamps(buf.data_ptr()) == 0
        ops.hubfactor_gc1(f, W1s[rep + 1], b1, W2, store_h1=False)
        torch.cuda.synchronize()
        lib.gcnk_debug_set_stamps(None)
        s = buf.view(-1, 4).cpu().numpy().astype(np.float64)
        s = s[s[:, 0] > 0]
        t0 = s[:, 0].min()
        rel = (s - t0) / 100.0
        q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 100)]  # noqa: E731
        worst = int(np.argmax(rel[:, 3]))
        print(json.dumps({"rep": rep, "blocks": len(s), "staged": q(rel[:, 0]), "mfma": q(rel[:, 1] - rel[:, 0]),
                          "epilogue": q(rel[:, 2] - rel[:, 1]), "projection": q(rel[:, 3] - rel[:, 2]),
                          "exit": q(rel[:, 3]), "slowest_block": worst, "slowest": rel[worst].round(2).tolist()}),
              flush=True)
    del S


if __name__ == "__main__":
    main()
