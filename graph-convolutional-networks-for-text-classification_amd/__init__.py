"""MI355X-native GCN hot path (gfx950 HIP kernels behind a C-ABI).

Drop-in for the reference's ``layer.py`` (GraphConvolution, GCN) — see
DESIGN.md for the path, the boundary and the kernels.
"""
from . import _lib, datasets, metrics, parallel, sparse
from .layer import GCN, GraphConvolution
from .ops import GCNFn, GraphConvFn, Operand, colsum, gemm, spmm
from .parallel import ColumnShardedSpMM, shard_bounds, sharded_gcn_forward
from .sparse import CSR, as_csr, from_arrays, from_torch, preprocess_adj

__all__ = [
    "datasets", "metrics", "parallel", "sparse",
    "GCN", "GraphConvolution", "GCNFn", "GraphConvFn", "Operand", "CSR",
    "as_csr", "from_arrays", "from_torch", "preprocess_adj", "spmm", "gemm", "colsum",
    "ColumnShardedSpMM", "shard_bounds", "sharded_gcn_forward",
]


def native_library_path():
    """Path of the in-tree libgcnk.so this package runs on."""
    return _lib.LIB_PATH
