"""Feature-column sharding of the graph aggregation over GPUs (SURVEY.md §8(e),
BASELINE.json config 5).

``C = A @ B`` is independent per column block of B.  With P ranks (one process
per GPU, ``torch.distributed`` over RCCL / xGMI) rank p holds the replicated
CSR ``A`` and its own column shard ``B[:, c0_p:c1_p]`` and computes
``C[:, c0_p:c1_p]`` with no communication.  Only a consumer that needs the whole
``C`` pays the one exchange: an all-gather of the ``[M, F/P]`` shards into a
``[P, M, F/P]`` buffer, which is handed over AS IS (``GatheredColumns``:
column block p is a ``[M, F_p]`` view with leading dimension F/P, exactly the
strided operand the SpMM / GEMM kernels take) -- no re-layout copy of the
gathered bytes (16.4 GB for config 5).  ``GatheredColumns.to_dense()`` makes
the row-major copy for a consumer that truly needs one.

For the two-layer GCN (reference layer.py:164-190) the hidden columns of gc1
are sharded the same way and gc2's projection needs a sum over the shards:
``S2 = H1 W2 = sum_p H1[:, p] W2[p, :]`` — an all-reduce of ``[M, nclass]``
(tiny), after which the second aggregation ``A S2 + b2`` runs replicated.

R8 / 20ng graphs do not shard: they run as independent
replicas and never use this module.

The per-shard arithmetic is the HIP kernels (``ops.spmm`` / ``ops.gemm``);
``kernels`` exists only so the collective logic can be exercised on CPU ranks
in the tests (gloo) with a test-side implementation of the same two calls.
"""
import types

import torch
import torch.distributed as dist

from . import _lib


def shard_bounds(F, world, rank):
    """Columns [c0, c1) of rank `rank` when F columns are split over `world` ranks
    (the first F % world ranks take one extra column)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, rem = divmod(int(F), int(world))
    c0 = rank * base + min(rank, rem)
    return c0, c0 + base + (1 if rank < rem else 0)


def _default_kernels():
    from . import ops
    return types.SimpleNamespace(spmm=ops.spmm, gemm=ops.gemm)


def _distributed():
    return dist.is_available() and dist.is_initialized()


def _world(group):
    if _distributed():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def _all_gather(buf, part, group):
    """buf[P, ...] <- every rank's `part` (equal shapes), RCCL's all-gather into one tensor."""
    if buf.device.type == "cuda":
        dist.all_gather_into_tensor(buf, part, group=group)
    else:
        dist.all_gather(list(buf.unbind(0)), part, group=group)


class GatheredColumns:
    """The all-gathered ``[M, F]`` product in the layout the collective wrote:
    ``buf[P, M, width]``, column block p = columns ``bounds[p]`` of C.

    ``block(p)`` is a zero-copy ``[M, c1 - c0]`` view (leading dimension
    ``width``), which the kernels accept as a strided operand; ``spmm(a)``
    runs a consumer product ``A @ C`` block by block into a row-major output;
    ``to_dense()`` is the explicit row-major copy."""

    def __init__(self, buf, bounds):
        self.buf, self.bounds = buf, list(bounds)
        self.shape = (buf.shape[1], self.bounds[-1][1])

    def block(self, p):
        c0, c1 = self.bounds[p]
        return self.buf[p, :, : c1 - c0]

    def blocks(self):
        return [(c0, c1, self.block(p)) for p, (c0, c1) in enumerate(self.bounds)]

    def to_dense(self):
        out = torch.empty(self.shape, dtype=self.buf.dtype, device=self.buf.device)
        for c0, c1, blk in self.blocks():
            out[:, c0:c1].copy_(blk)
        return out

    def spmm(self, a, bias=None, epilogue=_lib.EPI_NONE, out=None, kernels=None):
        """``epi(A @ C)`` for the gathered C, one launch per column block (each
        reads its block in place; the output is row-major ``[M_a, F]``)."""
        k = kernels or _default_kernels()
        if out is None:
            out = torch.empty((a.shape[0], self.shape[1]), dtype=self.buf.dtype, device=self.buf.device)
        for c0, c1, blk in self.blocks():
            k.spmm(a, blk, bias=bias[c0:c1] if bias is not None else None, epilogue=epilogue, out=out[:, c0:c1])
        return out


class ColumnShardedSpMM:
    """``C = epi(A @ B)`` with B's F columns split over the ranks of `group`.

    ``local(B_shard)`` computes this rank's ``[M, F_p]`` block (no exchange);
    ``gather(C_block)`` returns the full result on every rank (one RCCL
    all-gather into a ``GatheredColumns``; no re-layout).  Shards are padded to
    the widest one so every rank contributes equal bytes; the padded block is
    what ``local`` writes (its leading dimension is the padded width), so the
    kernel's output is already the send buffer."""

    def __init__(self, a, F, group=None, kernels=None):
        self.a = a
        self.F = int(F)
        self.group = group
        self.world, self.rank = _world(group)
        self.bounds = [shard_bounds(self.F, self.world, r) for r in range(self.world)]
        self.width = max(c1 - c0 for c0, c1 in self.bounds)
        self.kernels = kernels or _default_kernels()

    @property
    def columns(self):
        return self.bounds[self.rank]

    def shard(self, B):
        """This rank's column block of a full ``[K, F]`` operand (a contiguous copy)."""
        c0, c1 = self.columns
        return B[:, c0:c1].contiguous()

    def local(self, B_shard, bias=None, epilogue=_lib.EPI_NONE):
        c0, c1 = self.columns
        if B_shard.shape[1] != c1 - c0:
            raise RuntimeError(f"rank {self.rank}: shard has {B_shard.shape[1]} columns, expected {c1 - c0}")
        M = self.a.shape[0]
        alloc = torch.zeros if c1 - c0 < self.width else torch.empty   # pad columns are sent, so defined
        block = alloc((M, self.width), dtype=torch.float32, device=B_shard.device)
        view = block[:, : c1 - c0]
        b = bias[c0:c1] if bias is not None else None
        self.kernels.spmm(self.a, B_shard, bias=b, epilogue=epilogue, out=view)
        return block

    def gather(self, block):
        """All ranks' blocks -> ``GatheredColumns`` (RCCL all-gather over xGMI,
        whenever a process group exists -- a 1-rank group included)."""
        M = block.shape[0]
        buf = torch.empty((self.world, M, self.width), dtype=block.dtype, device=block.device)
        if _distributed():
            _all_gather(buf, block.contiguous(), self.group)
        else:
            buf[0].copy_(block)
        return GatheredColumns(buf, self.bounds)

    def __call__(self, B_shard, bias=None, epilogue=_lib.EPI_NONE, gather=True):
        block = self.local(B_shard, bias=bias, epilogue=epilogue)
        return self.gather(block) if gather else block


def sharded_gcn_forward(model, x, adj, group=None, kernels=None):
    """Eval forward of the two-layer GCN (reference layer.py:164-190) with the
    hidden columns of gc1 split over ranks:

        S1_p = X W1[:, p]                      no exchange        layer.py:102
        H1_p = relu(A S1_p + b1[p])            no exchange        layer.py:106,110,182
        S2   = all_reduce_p(H1_p W2[p, :])     [M x nclass] sum   layer.py:102 (gc2)
        Z    = A S2 + b2                       replicated         layer.py:106,110

    `model` holds the full parameters on every rank (each rank slices its own
    columns); dropout is the identity in eval mode (layer.py:185)."""
    k = kernels or _default_kernels()
    world, rank = _world(group)
    W1, b1 = model.gc1.weight.detach(), model.gc1.bias
    W2, b2 = model.gc2.weight.detach(), model.gc2.bias
    c0, c1 = shard_bounds(W1.shape[1], world, rank)
    from .ops import Operand
    from .sparse import as_csr
    a = adj if not isinstance(adj, torch.Tensor) else as_csr(adj)
    xop = x if not isinstance(x, torch.Tensor) else Operand(x)
    W1p = W1[:, c0:c1].contiguous()
    S1 = k.spmm(xop.csr, W1p) if xop.csr is not None else k.gemm(xop.dense, W1p)
    H1 = k.spmm(a, S1, bias=(b1.detach()[c0:c1].contiguous() if b1 is not None else None),
                epilogue=_lib.EPI_BIAS_RELU)   # a null bias adds 0 in the epilogue
    S2 = k.gemm(H1, W2[c0:c1].contiguous())
    if _distributed():
        dist.all_reduce(S2, op=dist.ReduceOp.SUM, group=group)
    return k.spmm(a, S2, bias=(b2.detach() if b2 is not None else None),
                  epilogue=_lib.EPI_BIAS if b2 is not None else _lib.EPI_NONE)
