"""Per-call time (hipGraph of back-to-back launches) of gcnk_gemm_f32 on a
given shape; one JSON line.  python scripts/gemm_probe.py M N K
(GCNK_PROBE_SPLIT=<n> forces split_k)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import ops
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from hub_probe import time_graph
    M, N, K = (int(x) for x in sys.argv[1:4])
    dev = torch.device("cuda", 0)
    A = torch.randn(M, K, device=dev)
    B = torch.randn(K, N, device=dev)
    split = int(os.environ.get("GCNK_PROBE_SPLIT", "0")) or None
    C = ops.gemm(A, B, split_k=split)
    err = float((C - A.double() @ B.double()).abs().max())
    us = time_graph([lambda: ops.gemm(A, B, out=C, split_k=split)], 100)
    print(json.dumps({"M": M, "N": N, "K": K, "split_k": split, "us": round(us, 3),
                      "tflops": 2 * M * N * K / us / 1e6, "max_err": err}), flush=True)


if __name__ == "__main__":
    main()
