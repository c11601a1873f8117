"""CPU checks of the SpMM plan builders (gcnk_spmm_plan_build_host: the same
host code the device build runs, writing into host memory).

The hub-split plan (include/gcnk.h, csrc/hub.hip) is executed here by a numpy
interpreter of its two kernels — light blocks reading staged rows / gathering
the rest, hub rows summed from per-block partials plus leftover nonzeros —
and compared with the float64 oracle, so the plan's bookkeeping (row
ownership, staging, partial indices, leftovers) is checked without a GPU.
The kernels themselves are checked on the GPU (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest

import gcn_amd  # noqa: F401
from graph_convolutional_networks_for_text_classification_amd import _lib
from oracle import csr_ref

HUB_MAGIC = 0x474E4831
ROW_MAGIC = 0x474E4B35


def build_host_plan(rp, ci, v, shape, hub_min=0, block_rows=0, groups=1, ipc=12, dense=0.25):
    lib = _lib.load()
    M, K = shape
    rp = np.ascontiguousarray(rp, np.int32)
    ci = np.ascontiguousarray(ci, np.int32)
    v = np.ascontiguousarray(v, np.float32)
    nnz = len(ci)
    nbytes = lib.gcnk_spmm_plan_bytes_host(rp.ctypes.data, ci.ctypes.data, M, K, nnz, ipc, groups, dense, hub_min,
                                           block_rows)
    assert nbytes > 0, lib.gcnk_last_error()
    buf = np.zeros(nbytes // 4, np.int32)
    rc = lib.gcnk_spmm_plan_build_host(rp.ctypes.data, ci.ctypes.data, v.ctypes.data, M, K, nnz, ipc, groups, dense,
                                       hub_min, block_rows, buf.ctypes.data, nbytes)
    assert rc == 0, lib.gcnk_last_error()
    return buf


def _a4(x):
    return (x + 3) & ~3


def exec_hub_plan(plan, B):
    """numpy interpreter of hub_light_kernel + hub_finish_kernel (float64)."""
    h = plan[:16]
    assert h[0] == HUB_MAGIC
    M, nblocks, R, nhub, npart, smax = int(h[1]), int(h[4]), int(h[5]), int(h[6]), int(h[7]), int(h[14])
    F = B.shape[1]
    B = B.astype(np.float64)
    C = np.full((M, F), np.nan)
    written = np.zeros(M, np.int64)
    part = np.full((npart, F), np.nan)
    for b in range(nblocks):
        rec = plan[16 + b * R: 16 + (b + 1) * R]
        nstage, nl, ng, nit = (int(x) for x in rec[:4])
        assert nstage <= smax and nstage <= int(h[8])
        scols = rec[4:4 + nstage]
        o_out = _a4(4 + nstage)
        o_it = _a4(o_out + 2 * (nl + ng))
        assert o_it + 2 * nit <= R
        ib = 0
        for o in range(nl + ng):
            dest, ie = int(rec[o_out + 2 * o]), int(rec[o_out + 2 * o + 1])
            items = rec[o_it + 2 * ib: o_it + 2 * ie].reshape(-1, 2)
            slots = items[:, 0]
            vals = items[:, 1].copy().view(np.float32).astype(np.float64)
            assert (ie - ib) % 4 == 0, "items padded to a multiple of 4"
            pad = slots == nstage                      # {zero row, 0} padding
            assert np.all(vals[pad] == 0) and np.all((slots >= 0) & (slots <= nstage)), "items read staged rows"
            cols = scols[np.clip(slots[~pad], 0, max(nstage - 1, 0))]
            acc = vals[~pad] @ B[cols] if len(cols) else np.zeros(F)
            if dest >= 0:
                assert o < nl, "light rows come first"
                C[dest] = acc
                written[dest] += 1
            else:
                assert o >= nl
                part[-dest - 1] = acc
            ib = ie
        assert ib == nit
    hubs = plan[16 + nblocks * R: 16 + nblocks * R + 4 * (nhub + 1)].reshape(-1, 4)
    left = plan[16 + nblocks * R + 4 * (nhub + 1):].reshape(-1, 2)
    assert len(left) == int(h[10])
    for i in range(nhub):
        row, pb, npr, lb = (int(x) for x in hubs[i])
        le = int(hubs[i + 1][3])
        lv = left[lb:le, 1].copy().view(np.float32).astype(np.float64)
        acc = part[pb:pb + npr].sum(0) + (lv @ B[left[lb:le, 0]] if le > lb else 0.0)
        C[row] = acc
        written[row] += 1
    assert np.all(written == 1), "every output row exactly once"
    assert not np.isnan(part).any(), "every partial row written"
    return C


def _hubby(rng, M, K, nhub, hub_deg, light_deg, symmetric_block=False):
    rows, cols = [], []
    hubs = rng.choice(M, nhub, replace=False)
    for r in range(M):
        if r in hubs:
            c = rng.choice(K, min(K, hub_deg), replace=False)
        else:
            d = int(rng.integers(0, light_deg + 1))
            c = np.concatenate([[r % K], rng.choice(hubs % K, min(d, nhub), replace=False)]) if d else np.zeros(0, int)
        rows.append(np.full(len(c), r))
        cols.append(c)
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    return csr_ref.coo_to_csr(rows, cols, rng.standard_normal(rows.size).astype(np.float32), (M, K))


def _check(rp, ci, v, shape, F=24, **kw):
    plan = build_host_plan(rp, ci, v, shape, **kw)
    B = np.random.default_rng(1).standard_normal((shape[1], F)).astype(np.float32)
    got = exec_hub_plan(plan, B)
    want = csr_ref.spmm_csr(rp, ci, v.astype(np.float32).astype(np.float64), B)
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-10)
    return plan


def test_r8_adjacency_gets_the_hub_plan(r8):
    adj = r8["adj"].coalesce()
    idx = adj.indices().numpy()
    rp, ci, v = csr_ref.coo_to_csr(idx[0], idx[1], adj.values().numpy(), adj.shape)
    plan = _check(rp, ci, v, adj.shape, F=16)
    h = plan[:16]
    assert h[6] == r8["ntopic"], "the 50 topic rows are the hubs"
    assert h[11] == r8["ndoc"], "every document row is a light row"
    assert 200 <= h[4] <= 300, "about one light block per CU"
    assert h[8] <= 64
    assert h[10] == 2 * 237 + 50, "leftovers: the 237 topic-topic edges both ways + the topic self loops"


def test_hub_plan_square_nonsquare_and_overflowing_stage():
    rng = np.random.default_rng(0)
    # square: sparse hub rows, light rows self + a few hubs (automatic threshold)
    rp, ci, v = _hubby(rng, 3000, 3000, 40, 300, 6)
    plan = _check(rp, ci, v, (3000, 3000))
    assert plan[0] == HUB_MAGIC
    # hub rows dense enough for the MFMA tile path keep the row-unit + tile plan
    rp, ci, v = _hubby(rng, 900, 900, 12, 700, 6)
    assert build_host_plan(rp, ci, v, (900, 900))[0] == ROW_MAGIC
    # rectangular (K < M): columns >= K are never owned; light rows j >= K own nothing
    rp, ci, v = _hubby(rng, 1200, 700, 30, 150, 5)
    _check(rp, ci, v, (1200, 700), hub_min=100)
    # light rows referencing many distinct columns: blocks are cut before their
    # staged rows would exceed the 64 stage slots
    rows = np.repeat(np.arange(1000), 10)
    cols = rng.integers(0, 1000, rows.size)
    hub_r = np.full(3000, 7)
    hub_c = rng.choice(1000, 3000)
    rp, ci, v = csr_ref.coo_to_csr(np.concatenate([rows, hub_r]), np.concatenate([cols, hub_c]),
                                   rng.standard_normal(rows.size + 3000).astype(np.float32), (1000, 1000))
    plan = _check(rp, ci, v, (1000, 1000), hub_min=200, block_rows=64)
    R = plan[5]
    recs = plan[16:16 + plan[4] * R].reshape(plan[4], R)
    assert recs[:, 0].max() <= 64 and recs[:, 1].max() < 64, "stage-bound blocks hold fewer than block_rows rows"
    assert plan[8] == recs[:, 0].max()


def test_hub_plan_empty_rows_and_explicit_block_rows():
    rng = np.random.default_rng(3)
    rp, ci, v = _hubby(rng, 1500, 1500, 30, 200, 4)
    for br in (1, 4, 64):
        _check(rp, ci, v, (1500, 1500), F=8, block_rows=br)


def test_row_plan_when_no_hubs_or_forced():
    rng = np.random.default_rng(4)
    rows = rng.integers(0, 2000, 20000)
    cols = rng.integers(0, 2000, 20000)
    rp, ci, v = csr_ref.coo_to_csr(rows, cols, rng.standard_normal(20000).astype(np.float32), (2000, 2000))
    plan = build_host_plan(rp, ci, v, (2000, 2000))
    assert plan[0] == ROW_MAGIC, "uniform graph: no hubs -> row-unit plan"
    rp, ci, v = _hubby(rng, 900, 900, 12, 700, 6)
    assert build_host_plan(rp, ci, v, (900, 900), hub_min=-1)[0] == ROW_MAGIC
    # items are packed {col, value bits} right after the header in CSR order
    plan = build_host_plan(rp, ci, v, (900, 900), hub_min=-1)
    items = plan[16:16 + 2 * len(ci)].reshape(-1, 2)
    assert np.array_equal(items[:, 0], ci)
    assert np.array_equal(items[:, 1].view(np.float32), v.astype(np.float32))


def test_plan_rejects_bad_csr():
    lib = _lib.load()
    rp = np.array([0, 2, 1], np.int32)
    ci = np.array([0, 1], np.int32)
    n = lib.gcnk_spmm_plan_bytes_host(rp.ctypes.data, ci.ctypes.data, 2, 2, 2, 8, 1, 0.25, 0, 0)
    assert n == _lib.EARG and b"rowptr" in lib.gcnk_last_error()
    rp = np.array([0, 1, 2], np.int32)
    ci = np.array([0, 5], np.int32)
    n = lib.gcnk_spmm_plan_bytes_host(rp.ctypes.data, ci.ctypes.data, 2, 2, 2, 8, 1, 0.25, 0, 0)
    assert n == _lib.EARG and b"out of range" in lib.gcnk_last_error()


@pytest.mark.parametrize("kind", ["random", "mixed", "hub"])
def test_plan_bytes_is_exactly_the_built_image(kind):
    """gcnk_spmm_plan_bytes_host sizes a row-unit plan from its header alone
    (no light-row sort, no image): the build must write exactly that many
    bytes -- none past them, the last one included."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_gpu_parity import _mixed_density_csr, _random_csr
    lib = _lib.load()
    rng = np.random.default_rng(17)
    if kind == "mixed":
        rp, ci, v = _mixed_density_csr(rng, 900, 900)
        M = K = 900
    else:
        M, K = 3001, 2003
        rp, ci, v = _random_csr(M, K, 20000, rng, heavy_rows=(5, 1700), heavy_deg=2500, empty_frac=0.2)
    hub_min = 0 if kind == "hub" else -1
    rp, ci, v = (np.ascontiguousarray(a, t) for a, t in ((rp, np.int32), (ci, np.int32), (v, np.float32)))
    nbytes = lib.gcnk_spmm_plan_bytes_host(rp.ctypes.data, ci.ctypes.data, M, K, len(ci), 12, 1, 0.25, hub_min, 0)
    assert nbytes > 0 and nbytes % 4 == 0
    buf = np.full(nbytes // 4 + 64, -7, np.int32)
    rc = lib.gcnk_spmm_plan_build_host(rp.ctypes.data, ci.ctypes.data, v.ctypes.data, M, K, len(ci), 12, 1, 0.25,
                                       hub_min, 0, buf.ctypes.data, buf.nbytes)
    assert rc == 0, lib.gcnk_last_error()
    assert np.all(buf[nbytes // 4:] == -7), "the build wrote past the size plan_bytes reported"
    # no plan word is -7 (ids >= -1, counts >= 0, float bits of -7 would be a NaN),
    # so a sentinel left in the last reported word means the size was too large
    assert buf[nbytes // 4 - 1] != -7, "plan_bytes reported more than the build wrote"
