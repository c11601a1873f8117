"""In-kernel timeline of gcn_bwd2_kernel (csrc/bwd.hip) at R8's shape (7,724 x
200, 8 classes; needs the stamps build: make -C <pkg>/csrc variant NAME=stamps
DEFS=-DGCNK_STAMPS, then GCNK_LIB=_variants/libgcnk_stamps.so).  Per workgroup
s_memrealtime (100 MHz): 0 entry, 1 operands staged, 2 rows done (gZ1 stored),
3 partial stored; percentiles in us from the first entry."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import _lib, ops
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    M, N, P = 7724, 200, 8
    H1 = torch.relu(torch.randn(M, N, device=dev))
    gS2, G = torch.randn(M, P, device=dev), torch.randn(M, P, device=dev)
    W2 = torch.randn(N, P, device=dev)
    ops.gcn_bwd2(H1, gS2, W2, G=G, scale=2.0)
    torch.cuda.synchronize()
    buf = torch.zeros(4 * 4096, dtype=torch.int64, device=dev)
    q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 100)]  # noqa: E731
    for rep in range(4):
        buf.zero_()
        assert lib.gcnk_debug_set_stamps(buf.data_ptr()) == 0
        ops.gcn_bwd2(H1, gS2, W2, G=G, scale=2.0)
        torch.cuda.synchronize()
        lib.gcnk_debug_set_stamps(None)
        s = buf.view(-1, 4).cpu().numpy().astype(np.float64)
        s = s[s[:, 0] > 0]
        rel = (s - s[:, 0].min()) / 100.0
        print(json.dumps({"rep": rep, "blocks": len(s), "entry": q(rel[:, 0]), "staged": q(rel[:, 1] - rel[:, 0]),
                          "rows": q(rel[:, 2] - rel[:, 1]), "partial": q(rel[:, 3] - rel[:, 2]),
                          "exit": q(rel[:, 3])}), flush=True)


if __name__ == "__main__":
    main()
