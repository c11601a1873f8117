"""R8 eval forward per-call time (hipGraph of 10 forwards) under the ops
module's schedule switches (FUSE_PROJECTION, OVERLAP_TILE_PARTS), with the
logits checked against the default schedule.  One JSON line per setting.

  python scripts/fwd_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets, ops
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from hub_probe import time_graph
    dev = torch.device("cuda", 0)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    torch.manual_seed(0)
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(dev).eval()
    x, adj = r8["features"].to(dev), r8["adj"].to(dev)
    saved = ops.FUSE_PROJECTION, ops.OVERLAP_TILE_PARTS
    with torch.no_grad():
        ops.FUSE_PROJECTION, ops.OVERLAP_TILE_PARTS = False, False
        ref = m(x, adj)
        for name, fuse, overlap in (("separate", False, False), ("fuse_projection", True, False),
                                    ("fuse_projection+overlap_tile_parts", True, True)):
            ops.FUSE_PROJECTION, ops.OVERLAP_TILE_PARTS = fuse, overlap
            out = m(x, adj)
            torch.cuda.synchronize()
            err = float((out - ref).abs().max())
            us = time_graph([lambda: m(x, adj)], 20)
            print(json.dumps({"schedule": name, "forward_us": round(us, 3), "max_diff_vs_separate": err}), flush=True)
        ops.FUSE_PROJECTION, ops.OVERLAP_TILE_PARTS = saved


if __name__ == "__main__":
    main()
