"""Multi-process CPU checks of the feature-column sharding (parallel.py,
SURVEY.md §8(e)): world_size 2 over gloo, the per-shard SpMM / GEMM supplied by
the oracle's CSR restatement so the collective logic (shard bounds, padded
all-gather, re-layout, all-reduce of gc2's partial projection) is exercised
without a GPU.  On the GPU the same module runs the HIP kernels over RCCL."""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import gcn_amd  # noqa: F401
from graph_convolutional_networks_for_text_classification_amd import _lib
from graph_convolutional_networks_for_text_classification_amd.parallel import (
    ColumnShardedSpMM, shard_bounds, sharded_gcn_forward)
from oracle import csr_ref


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Csr:
    def __init__(self, rp, ci, v, shape):
        self.rp, self.ci, self.v, self.shape = rp, ci, v, shape


def _cpu_kernels():
    """spmm / gemm with the signatures parallel.py calls, on the oracle."""

    def spmm(a, B, bias=None, epilogue=_lib.EPI_NONE, out=None):
        acc = csr_ref.spmm_csr(a.rp, a.ci, a.v, B.double().numpy())
        if epilogue in (_lib.EPI_BIAS, _lib.EPI_BIAS_RELU) and bias is not None:
            acc = acc + bias.double().numpy()
        if epilogue == _lib.EPI_BIAS_RELU:
            acc = np.maximum(acc, 0.0)
        res = torch.from_numpy(acc.astype(np.float32))
        if out is None:
            return res
        out.copy_(res)
        return out

    def gemm(A, B):
        return torch.from_numpy((A.double().numpy() @ B.double().numpy()).astype(np.float32))

    return types.SimpleNamespace(spmm=spmm, gemm=gemm)


def _graph(seed=0, M=300, K=300, nnz=2500):
    rng = np.random.default_rng(seed)
    rows = np.concatenate([rng.integers(0, M, nnz), np.full(400, 7)])   # one heavy row
    cols = rng.integers(0, K, rows.size)
    rp, ci, v = csr_ref.coo_to_csr(rows, cols, rng.standard_normal(rows.size).astype(np.float32), (M, K))
    return _Csr(rp, ci, v, (M, K)), rng


def _model(nfeat, nhid=10, ncls=3):
    torch.manual_seed(3)
    return types.SimpleNamespace(
        gc1=types.SimpleNamespace(weight=torch.randn(nfeat, nhid), bias=torch.randn(nhid)),
        gc2=types.SimpleNamespace(weight=torch.randn(nhid, ncls), bias=torch.randn(ncls)))


def _worker(rank, world, port, F, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        k = _cpu_kernels()
        a, rng = _graph()
        B = torch.from_numpy(rng.standard_normal((a.shape[1], F)).astype(np.float32))
        bias = torch.from_numpy(rng.standard_normal(F).astype(np.float32))
        op = ColumnShardedSpMM(a, F, kernels=k)
        gathered = op(op.shard(B), bias=bias, epilogue=_lib.EPI_BIAS_RELU)
        full = gathered.to_dense()
        # a consumer reading the gathered blocks in place: A @ C, block by block
        consumer = gathered.spmm(a, kernels=k)
        assert gathered.block(op.rank).data_ptr() == gathered.buf[op.rank].data_ptr()   # zero-copy view
        block = op(op.shard(B), bias=bias, epilogue=_lib.EPI_BIAS_RELU, gather=False)
        # GCN eval forward with gc1's hidden columns sharded (all-reduce of H1 W2)
        logits = sharded_gcn_forward(_model(a.shape[1]), types.SimpleNamespace(csr=a, dense=None), a, kernels=k)
        q.put((rank, full.numpy(), block.numpy(), op.columns, logits.numpy(), consumer.numpy()))
    finally:
        dist.destroy_process_group()


def test_shard_bounds_cover_columns_exactly():
    for F in (1, 7, 8, 200, 4096):
        for world in (1, 2, 3, 8):
            b = [shard_bounds(F, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == F
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            assert max(c1 - c0 for c0, c1 in b) - min(c1 - c0 for c0, c1 in b) <= 1
    with pytest.raises(ValueError):
        shard_bounds(8, 2, 2)


@pytest.mark.parametrize("F", [8, 13])
def test_column_sharded_spmm_and_gcn_world2_gloo(F):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, F, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, full, block, cols, logits, consumer = q.get(timeout=180)
        res[rank] = (full, block, cols, logits, consumer)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference of the same products
    k = _cpu_kernels()
    a, rng = _graph()
    B = torch.from_numpy(rng.standard_normal((a.shape[1], F)).astype(np.float32))
    bias = torch.from_numpy(rng.standard_normal(F).astype(np.float32))
    ref = k.spmm(a, B, bias=bias, epilogue=_lib.EPI_BIAS_RELU).numpy()
    m = _model(a.shape[1])
    H1 = k.spmm(a, k.spmm(a, m.gc1.weight), bias=m.gc1.bias, epilogue=_lib.EPI_BIAS_RELU)
    ref_logits = k.spmm(a, k.gemm(H1, m.gc2.weight), bias=m.gc2.bias, epilogue=_lib.EPI_BIAS).numpy()
    ref_consumer = k.spmm(a, torch.from_numpy(ref)).numpy()
    assert sorted(res) == [0, 1]
    for rank in range(world):
        full, block, (c0, c1), logits, consumer = res[rank]
        np.testing.assert_array_equal(full, ref)                        # the gathered blocks are exact
        np.testing.assert_allclose(consumer, ref_consumer, rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(block[:, : c1 - c0], ref[:, c0:c1])
        np.testing.assert_allclose(logits, ref_logits, rtol=1e-5, atol=1e-4)


def test_bench_gpus_n_spawns_n_ranks():
    """`python bench.py --gpus 2` outside a launcher starts 2 rank processes
    (torch.distributed.run, 127.0.0.1 rendezvous) before any GPU call; each sees
    world 2.  --dry-run stops every rank before it touches the GPU."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    import re
    views = [json.loads(m) for m in re.findall(r"\{[^{}]*\"rank\"[^{}]*\}", r.stdout)]
    assert sorted(v["rank"] for v in views) == [0, 1]
    assert all(v["world"] == 2 for v in views)
    assert sorted(v["local_rank"] for v in views) == [0, 1]
    # one rank and --gpus 1: no launcher, world 1
    r1 = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--dry-run"],
                        capture_output=True, text=True, timeout=120, cwd=root)
    one = [json.loads(m) for m in re.findall(r"\{[^{}]*\"rank\"[^{}]*\}", r1.stdout)]
    assert r1.returncode == 0 and [v["world"] for v in one] == [1]
