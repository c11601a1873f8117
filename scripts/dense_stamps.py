"""In-kernel timeline of gcnk_dense_gc1_f32 (csrc/dense_gc1.hip) on the 20ng shape
(M 18,916, K 100, F 200, P 20) and the gensim R8 shape (7,724, 100, 200, 8); needs
the stamps build (make -C <pkg>/csrc variant NAME=stamps DEFS=-DGCNK_STAMPS, then
GCNK_LIB=_variants/libgcnk_stamps.so).  Per workgroup s_memrealtime (100 MHz):
0 entry, 1 W1 / W2 fragments loaded (all waves), 2 first tile done, 3 exit;
percentiles in us from the first entry."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import _lib
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    g = torch.Generator().manual_seed(0)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for M, K, F, P in ((18916, 100, 200, 20), (7724, 100, 200, 8)):
        AX = torch.zeros((M, K)).normal_(generator=g).to(dev)
        W1 = (torch.zeros((K, F)).normal_(generator=g) * 0.1).to(dev)
        W2 = (torch.zeros((F, P)).normal_(generator=g) * 0.1).to(dev)
        b1 = torch.zeros(F).normal_(generator=g).to(dev)
        S2 = torch.empty((M, P), device=dev)
        buf = torch.zeros(4 * 8192, dtype=torch.int64, device=dev)
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

        def run():
            _lib.check(lib.gcnk_dense_gc1_f32(M, K, F, P, p(AX), K, p(W1), F, p(b1), _lib.EPI_BIAS_RELU, None, 0,
                                              1.0, 1.0, 0, 0, None, p(W2), P, None, 0, p(S2), P, stream),
                       "gcnk_dense_gc1_f32")
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        for rep in range(3):
            buf.zero_()
            torch.cuda.synchronize()
            assert lib.gcnk_debug_set_stamps(buf.data_ptr()) == 0
            run()
            torch.cuda.synchronize()
            lib.gcnk_debug_set_stamps(None)
            s = buf.view(-1, 4).cpu().numpy().astype(np.float64)
            s = s[s[:, 0] > 0]
            rel = (s - s[:, 0].min()) / 100.0
            q = lambda x: [round(float(np.percentile(x, v)), 2) for v in (0, 10, 50, 90, 100)]  # noqa: E731
            print(json.dumps({"M": M, "rep": rep, "blocks": len(s), "entry": q(rel[:, 0]),
                              "fragments": q(rel[:, 1] - rel[:, 0]), "first_tile": q(rel[:, 2] - rel[:, 1]),
                              "rest": q(rel[:, 3] - rel[:, 2]), "exit": q(rel[:, 3])}), flush=True)


if __name__ == "__main__":
    main()
