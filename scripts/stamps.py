"""Debug timeline of the SpMM row kernel: per-workgroup s_memrealtime stamps
(100 MHz, wave 0 of each workgroup) at entry / unit loaded / gathers summed /
stored (heavy segments: counted in; the last arriver restamps after its
combine).  Prints a summary per case and per block kind (heavy-segment blocks
come first in the grid, then light-row blocks)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import _lib, datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr

    dev = torch.device("cuda", 0)
    lib = _lib.load()
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    A = as_csr(r8["adj"].to(dev))
    X = as_csr(r8["features"].to(dev))
    only = sys.argv[1:] or None
    # (column tile 0 only: grid rows of other tiles are not split by kind)
    cases = [("R8_A_F200", A, 200, 0, None), ("R8_A_F8", A, 8, 0, None),
             ("R8_A_F200_i16", A, 200, 0, 16), ("R8_X_F200", X, 200, 0, None)]
    cases = [c for c in cases if only is None or c[0] in only]
    for name, a, F, lanes, ipc in cases:
        B = torch.randn(a.shape[1], F, device=dev)
        out = torch.empty(a.shape[0], F, device=dev)
        for _ in range(3):
            ops.spmm(a, B, out=out, lanes=lanes, ipc=ipc)
        torch.cuda.synchronize()
        buf = torch.zeros(4 * 200000, dtype=torch.int64, device=dev)
        lib.gcnk_debug_set_stamps(buf.data_ptr())
        ops.spmm(a, B, out=out, lanes=lanes, ipc=ipc)
        torch.cuda.synchronize()
        lib.gcnk_debug_set_stamps(None)
        hdr = list(a._plans.values())[-1].header
        if hdr[5] == 0:   # tile-path-only operand (R8 X): chunks of single-chunk blocks vs multi-chunk blocks
            s_all = buf.view(-1, 4).cpu().numpy().astype(np.float64)
            nchunk = hdr[8]
            single = hdr[11] - hdr[9]            # single-chunk blocks come first (R8 X: document rows)
            t0 = s_all[s_all[:, 0] > 0, 0].min()
            idx = np.arange(len(s_all)) % max(nchunk, 1)
            for kind, sel in (("single", idx < single), ("multi", idx >= single)):
                s = s_all[sel & (s_all[:, 0] > 0) & (s_all[:, 3] > 0)]
                if len(s):
                    summarize(f"{name}:tile_{kind}", (s - t0) / 100.0)
            continue
        # heavy blocks: one unit per workgroup at 64 lanes, 4 per 256-thread workgroup
        # for 8..32 lanes, 1 per one-wave workgroup below (hdr[3] = 64 / lanes)
        lpr = 64 // hdr[3]
        nhb = hdr[6] if lpr == 64 else (hdr[6] // 4 if lpr >= 8 else hdr[6])
        s_all = buf.view(-1, 4).cpu().numpy().astype(np.float64)
        t0 = s_all[s_all[:, 0] > 0, 0].min()
        for kind, rows in (("heavy", s_all[:nhb]), ("light", s_all[nhb:]), ("all", s_all)):
            s = rows[(rows[:, 0] > 0) & (rows[:, 3] > 0)]
            if len(s) == 0:
                continue
            s = (s - t0) / 100.0  # µs
            summarize(name + ":" + kind, s)


def summarize(name, s):
    import numpy as np
    span = s[:, 3].max()
    if True:
        res = {
            "case": name, "wgs": int(len(s)), "span_us": round(span, 2),
            "entry_p50_us": round(float(np.median(s[:, 0])), 2), "entry_max_us": round(float(s[:, 0].max()), 2),
            "stage_p50_us": round(float(np.median(s[:, 1] - s[:, 0])), 2),
            "walk_p50_us": round(float(np.median(s[:, 2] - s[:, 1])), 2),
            "walk_p99_us": round(float(np.percentile(s[:, 2] - s[:, 1], 99)), 2),
            "combine_p50_us": round(float(np.median(s[:, 3] - s[:, 2])), 2),
            "wg_p50_us": round(float(np.median(s[:, 3] - s[:, 0])), 2),
            "wg_max_us": round(float((s[:, 3] - s[:, 0]).max()), 2),
            "entry_hist": np.histogram(s[:, 0], bins=8)[0].tolist(),
        }
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
