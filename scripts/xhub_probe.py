"""X_hubs W1 of the factored R8 forward (the hub rows of layer.py:102, [50 x
7463] x [7463 x 200]) per call in a hipGraph: the tile SpMM on the hub rows'
CSR (the product path) against gcnk_gemm_f32's small-M in-workgroup K-split
GEMM on a dense copy of them (whichever variant of that kernel the loaded
library was built with: GCNK_WK_KBW / GCNK_WK_NTG), results compared.  One
JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import _lib, datasets, factor, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    from hub_probe import time_graph
    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    a = as_csr(r8["adj"].to(dev))
    xop = ops.Operand(r8["features"].to(dev))
    f = factor.build(a, xop)
    H, K = f.x_hub.shape
    d = torch.zeros((H, (K + 3) // 4 * 4), device=dev)
    _lib.check(_lib.load().gcnk_csr_to_dense(f.x_hub.rowptr.data_ptr(), f.x_hub.colind.data_ptr(),
                                             f.x_hub.val.data_ptr(), H, K, d.data_ptr(), d.stride(0),
                                             torch.cuda.current_stream().cuda_stream), "gcnk_csr_to_dense")
    xd = d[:, :K]
    torch.manual_seed(0)
    W1 = torch.rand((K, 200), device=dev) - 0.5
    out_t = torch.empty((H, 200), device=dev)
    out_g = torch.empty((H, 200), device=dev)
    t_tile = time_graph([lambda: ops.spmm(f.x_hub, W1, out=out_t)], 200)
    t_gemm = time_graph([lambda: ops.gemm(xd, W1, out=out_g)], 200)
    err = float((out_t - out_g).abs().max())
    print(json.dumps({"tile_us": round(t_tile, 3), "gemm_us": round(t_gemm, 3), "max_diff": err,
                      "lib": os.path.basename(_lib.LIB_PATH)}), flush=True)


if __name__ == "__main__":
    main()
