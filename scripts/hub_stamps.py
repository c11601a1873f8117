"""In-kernel timeline of the hub-split SpMM (needs the stamps variant:
make -C <pkg>/csrc variant NAME=stamps DEFS=-DGCNK_STAMPS, then
GCNK_LIB=_variants/libgcnk_stamps.so).  s_memrealtime (100 MHz) per workgroup:
light kernel: entry / record in LDS / stage in LDS / outputs stored (after a
barrier); finishing kernel: entry / partials summed / stored.  Prints
percentiles (us, relative to the first light-kernel entry) per phase."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(x):
    import numpy as np
    return {k: round(float(np.percentile(x, q)), 3) for k, q in (("p0", 0), ("p50", 50), ("p90", 90), ("p100", 100))}


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
    for br in [int(x) for x in (sys.argv[1:] or ["0"])]:
        sp.HUB_MIN, sp.HUB_BLOCK_ROWS = 0, br
        for F in (200, 8):
            B = torch.randn(A.shape[1], F, device=dev)
            bias = torch.randn(F, device=dev)
            out = torch.empty(A.shape[0], F, device=dev)
            for _ in range(20):
                ops.spmm(A, B, bias=bias, epilogue=_lib.EPI_BIAS_RELU, out=out)
            torch.cuda.synchronize()
            plan = [p for k, p in A._plans.items() if k[4] == br and k[1] == lib.gcnk_spmm_groups(F, 0)][-1]
            h = plan.header
            nb, nhub = h[4], h[6]
            ntiles = (F + 255) // 256 if F > 8 else 1
            buf = torch.zeros(4 * (nb * ntiles + nhub * 16), dtype=torch.int64, device=dev)
            assert lib.gcnk_debug_set_stamps(buf.data_ptr()) == 0
            ops.spmm(A, B, bias=bias, epilogue=_lib.EPI_BIAS_RELU, out=out)
            torch.cuda.synchronize()
            lib.gcnk_debug_set_stamps(None)
            s = buf.view(-1, 4).cpu().numpy().astype(np.float64)
            la = s[: nb * ntiles]
            fb = s[nb * ntiles:]
            fb = fb[fb[:, 0] > 0]
            t0 = la[:, 0].min()
            res = {"F": F, "block_rows": br, "blocks": nb,
                   "light_entry": pct((la[:, 0] - t0) / 100), "record": pct((la[:, 1] - la[:, 0]) / 100),
                   "stage": pct((la[:, 2] - la[:, 1]) / 100), "outputs": pct((la[:, 3] - la[:, 2]) / 100),
                   "light_end": pct((la[:, 3] - t0) / 100),
                   "finish_entry": pct((fb[:, 0] - t0) / 100), "finish_sum": pct((fb[:, 1] - fb[:, 0]) / 100),
                   "finish_end": pct((fb[:, 2] - t0) / 100)}
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
