"""rocprofv3 probe: the fused projection SpMM (gcnk_spmm_proj_f32) vs the plain one."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import gcn_amd  # noqa: E402,F401
from graph_convolutional_networks_for_text_classification_amd import datasets, ops  # noqa: E402
from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr  # noqa: E402

dev = torch.device("cuda", 0)
r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
A = as_csr(r8["adj"].to(dev))
S1 = torch.randn(r8["nodes"], 200, device=dev)
W2 = torch.randn(200, 8, device=dev)
b = torch.randn(200, device=dev)
for _ in range(20):
    ops.spmm(A, S1, bias=b, epilogue=2)
    ops.spmm_proj(A, S1, W2, bias=b, epilogue=2, store_main=False)
    ops.spmm_proj(A, S1, W2, bias=b, epilogue=2, store_main=True)
torch.cuda.synchronize()
print("probe done")
