"""Per-call time of gcn_bwd2 (kernel + its reduce) at R8's shape, warm, hipGraph
of back-to-back calls, HIP events.  Run under GCNK_LIB=<variant> to compare
builds (e.g. GCNK_BWD_TARGET, the workgroups per column slice)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import ops
    from hub_probe import time_graph
    dev = torch.device("cuda", 0)
    for M, N, P in ((7724, 200, 8), (18916, 200, 20)):
        H1 = torch.relu(torch.randn(M, N, device=dev))
        gS2, G = torch.randn(M, P, device=dev), torch.randn(M, P, device=dev)
        W2 = torch.randn(N, P, device=dev)
        us = time_graph([lambda: ops.gcn_bwd2(H1, gS2, W2, G=G, scale=2.0)], 200)
        print(json.dumps({"lib": os.path.basename(os.environ.get("GCNK_LIB", "libgcnk.so")), "M": M, "N": N, "P": P,
                          "us": round(us, 3)}), flush=True)


if __name__ == "__main__":
    main()
