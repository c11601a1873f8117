"""CPU checks of the SpMM plan builders (gcnk_spmm_plan_build_host: the same
host code the device build runs, writing into host memory).

The hub plan (include/gcnk.h, csrc/hub.hip) is executed here by a numpy
interpreter of its two kernels — row groups computing their light rows and
one partial per hub from their LDS image, hub rows summed from the groups'
partials — and compared with the float64 oracle, so the plan's bookkeeping
(groups, slots, item order, hub x hub placement) is checked without a GPU.
The kernels themselves are checked on the GPU (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest

import gcn_amd  # noqa: F401
from graph_convolutional_networks_for_text_classification_amd import _lib
from oracle import csr_ref

HUB_MAGIC = 0x474E4832
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
    """numpy interpreter of hub_group_kernel + hub_sum_kernel (float64; the
    column slices of a launch do not change what is summed, so whole rows).

    Checks the plan's bookkeeping: every light row and every hub partial
    written exactly once, slots inside the group's LDS image, items in CSR
    (column) order with padding only at the ends of rows / hubs, light rows
    sorted by batch count, hub x hub nonzeros in group t % G."""
    h = plan[:16]
    assert h[0] == HUB_MAGIC
    M, G, R, H, h0, nL, gs, max_hb = (int(h[i]) for i in (1, 4, 5, 6, 7, 8, 10, 13))
    assert M == H + nL and G == -(-nL // gs)
    F = B.shape[1]
    B = B.astype(np.float64)

    def light_row(l):
        return l if l < h0 else l + H

    C = np.full((M, F), np.nan)
    written = np.zeros(M, np.int64)
    part = np.full((H, G, F), np.nan)
    for g in range(G):
        rec = plan[16 + g * R: 16 + (g + 1) * R]
        n, nhb, nit, o_it = (int(x) for x in rec[:4])
        assert n == min(gs, nL - g * gs) and nhb <= max_hb
        assert o_it % 4 == 0 and o_it + 2 * nit <= R
        light = rec[4:4 + 2 * n].reshape(-1, 2)
        hb = rec[4 + 2 * n:4 + 2 * n + 2 * nhb].reshape(-1, 2)
        hoff = rec[4 + 2 * n + 2 * nhb:4 + 2 * n + 2 * nhb + H + 1]
        items = rec[o_it:o_it + 2 * nit].reshape(-1, 2)
        slots = items[:, 0]
        vals = items[:, 1].copy().view(np.float32).astype(np.float64)
        assert np.all((slots >= 0) & (slots <= H + n)), "items read the group's LDS image"
        zero = slots == H + n                    # padding: the zero row, value 0
        assert np.all(vals[zero] == 0)
        srows = np.array([h0 + s if s < H else light_row(g * gs + s - H) for s in range(H + n)], np.int64)

        def walk(k0, k1):
            real = ~zero[k0:k1]
            assert np.all(real[:real.sum()]), "padding only at the end"
            sl = slots[k0:k1][real]
            cols = srows[sl]
            assert np.all(np.diff(cols) > 0), "CSR column order"
            acc = vals[k0:k1][real] @ B[cols] if len(cols) else np.zeros(F)
            return sl, acc

        nbs = light[:, 0] >> 16
        assert np.all(np.diff(nbs) <= 0), "light rows sorted by batch count"
        seen = set()
        for (word, ib), nb in zip(light, nbs):
            i = int(word & 0xffff)
            seen.add(i)
            r = light_row(g * gs + i)
            sl, acc = walk(int(ib), int(ib) + 4 * int(nb))
            assert np.all((sl < H) | (srows[sl] == r)), "a light row reads hub rows and itself"
            C[r] = acc
            written[r] += 1
        assert seen == set(range(n))
        assert hoff[0] == 0 and hoff[-1] == nhb and np.all(np.diff(hoff) >= 0)
        for t in range(H):
            bs = range(int(hoff[t]), int(hoff[t + 1]))
            assert all(int(hb[b, 0]) == t for b in bs)
            if len(bs):
                k0 = int(hb[bs[0], 1])
                assert all(int(hb[b, 1]) == k0 + 8 * (b - bs[0]) for b in bs), "hub batches of 8, contiguous"
                sl, acc = walk(k0, k0 + 8 * len(bs))
            else:
                sl, acc = np.zeros(0, np.int64), np.zeros(F)
            assert not (sl < H).any() or t % G == g, "hub x hub nonzeros ride in group t % G"
            part[t, g] = acc
    assert not np.isnan(part).any(), "every partial written"
    for t in range(H):
        C[h0 + t] = part[t].sum(0)
        written[h0 + t] += 1
    assert np.all(written == 1), "every output row exactly once"
    return C


def _doc_topic(rng, below, H, above, hub_deg, light_deg, hub_hub=0.2, empty_frac=0.05, no_diag_frac=0.05):
    """Square doc-topic-like operand: `below` light rows, H contiguous hub rows,
    `above` light rows; light rows = own diagonal + a few hub columns, hub rows =
    light columns + some hub columns (+ diagonal)."""
    M = below + H + above
    h0 = below
    hubs = np.arange(h0, h0 + H)
    light = np.concatenate([np.arange(below), np.arange(h0 + H, M)])
    rows, cols = [], []
    for r in light:
        if rng.random() < empty_frac:
            continue
        d = int(rng.integers(0, light_deg + 1))
        c = list(rng.choice(hubs, min(d, H), replace=False))
        if rng.random() >= no_diag_frac:
            c.append(r)
        rows += [r] * len(c)
        cols += c
    for r in hubs:
        c = list(rng.choice(light, min(len(light), hub_deg), replace=False))
        c += [x for x in hubs if rng.random() < hub_hub]
        rows += [r] * len(c)
        cols += c
    rows, cols = np.array(rows), np.array(cols)
    return csr_ref.coo_to_csr(rows, cols, rng.standard_normal(rows.size).astype(np.float32), (M, M))


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
    assert h[7] == r8["ndoc"] and h[8] == r8["ndoc"], "topics follow the documents; every document is a light row"
    assert h[4] == 32 and h[10] == 240, "wide F: 32 groups of 240 documents (x 7 column slices at F = 200)"
    # narrow widths (F = 8: 32 lane groups per wavefront): ~256 groups, one slice
    plan8 = _check(rp, ci, v, adj.shape, F=8, groups=32)
    assert 240 <= plan8[4] <= 264


def test_hub_plan_hubs_in_the_middle_with_hub_hub_entries():
    rng = np.random.default_rng(0)
    rp, ci, v = _doc_topic(rng, 1700, 40, 1300, 300, 6)
    plan = _check(rp, ci, v, (3040, 3040))
    assert plan[0] == HUB_MAGIC and plan[6] == 40 and plan[7] == 1700
    for br in (1, 7, 64, 512):   # explicit rows per group, groups straddling the hub range
        _check(rp, ci, v, (3040, 3040), F=8, block_rows=br)
    # hubs first / last
    for below, above in ((0, 900), (900, 0)):
        rp, ci, v = _doc_topic(rng, below, 16, above, 120, 4)
        plan = _check(rp, ci, v, (below + 16 + above,) * 2, F=5)
        assert plan[0] == HUB_MAGIC and plan[7] == below


def test_hub_plan_not_applicable_falls_back_to_row_plan():
    rng = np.random.default_rng(1)
    # a light row referencing another light row
    rp, ci, v = _doc_topic(rng, 800, 20, 200, 150, 4)
    M = 1020
    rows = np.repeat(np.arange(M), np.diff(rp))
    rows, cols = np.append(rows, 3), np.append(ci, 5)
    rp2, ci2, v2 = csr_ref.coo_to_csr(rows, cols, np.append(v, 1.0).astype(np.float32), (M, M))
    assert build_host_plan(rp2, ci2, v2, (M, M))[0] == ROW_MAGIC
    assert build_host_plan(rp, ci, v, (M, M))[0] == HUB_MAGIC
    # hub rows not contiguous: swap a hub row's nonzeros into a light row's place
    perm = np.arange(M)
    perm[[805, 100]] = perm[[100, 805]]
    rows3 = perm[np.repeat(np.arange(M), np.diff(rp))]
    rp3, ci3, v3 = csr_ref.coo_to_csr(rows3, perm[ci], v, (M, M))
    assert build_host_plan(rp3, ci3, v3, (M, M))[0] == ROW_MAGIC
    # rectangular operands never get it
    rp4, ci4, v4 = _doc_topic(rng, 500, 10, 0, 100, 3)
    assert build_host_plan(rp4[:401], ci4[:rp4[400]], v4[:rp4[400]], (400, 510))[0] == ROW_MAGIC


def test_row_plan_when_no_hubs_or_forced():
    rng = np.random.default_rng(4)
    rows = rng.integers(0, 2000, 20000)
    cols = rng.integers(0, 2000, 20000)
    rp, ci, v = csr_ref.coo_to_csr(rows, cols, rng.standard_normal(20000).astype(np.float32), (2000, 2000))
    plan = build_host_plan(rp, ci, v, (2000, 2000))
    assert plan[0] == ROW_MAGIC, "uniform graph: no hubs -> row-unit plan"
    rp, ci, v = _doc_topic(rng, 600, 12, 288, 500, 6)
    assert build_host_plan(rp, ci, v, (900, 900))[0] == HUB_MAGIC
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
    elif kind == "hub":
        rp, ci, v = _doc_topic(rng, 2000, 30, 900, 400, 5)
        M = K = 2930
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
    assert (buf[0] == HUB_MAGIC) == (kind == "hub")
    assert np.all(buf[nbytes // 4:] == -7), "the build wrote past the size plan_bytes reported"
    # no plan word is -7 (ids >= -1, counts >= 0, float bits of -7 would be a NaN),
    # so a sentinel left in the last reported word means the size was too large
    assert buf[nbytes // 4 - 1] != -7, "plan_bytes reported more than the build wrote"


SPLIT_MAGIC = 0x474E5831


def exec_split_plan(plan, B):
    """numpy interpreter of the split plan (csrc/xw.hip): light rows = dense
    values over the hot columns, heavy rows = dense rows (float64)."""
    h = plan[:16]
    assert h[0] == SPLIT_MAGIC
    M, K, nl, nhot, nhp, nh, h0, o_hot, o_xl, o_xh, ldxh = (int(h[i]) for i in (1, 2, 4, 5, 6, 7, 8, 10, 11, 12, 13))
    assert M == nl + nh and nhp % 4 == 0 and nhot <= nhp and ldxh % 4 == 0 and ldxh >= K
    hot = plan[o_hot:o_hot + nhp]
    assert np.all(np.diff(hot[:nhot]) > 0), "hot columns sorted"
    xl = plan[o_xl:o_xl + nl * nhp].view(np.float32).reshape(nl, nhp).astype(np.float64)
    assert np.all(xl[:, nhot:] == 0)
    xh = plan[o_xh:o_xh + nh * ldxh].view(np.float32).reshape(nh, ldxh).astype(np.float64)
    B = B.astype(np.float64)
    C = np.zeros((M, B.shape[1]))
    light = np.array([l if l < h0 else l + nh for l in range(nl)], np.int64)
    C[light] = xl[:, :nhot] @ B[hot[:nhot]]
    C[h0:h0 + nh] = xh[:, :K] @ B
    return C


def test_r8_features_get_the_split_plan(r8):
    x = r8["features"].coalesce()
    idx = x.indices().numpy()
    rp, ci, v = csr_ref.coo_to_csr(idx[0], idx[1], x.values().numpy(), x.shape)
    plan = build_host_plan(rp, ci, v, x.shape)
    assert plan[0] == SPLIT_MAGIC and plan[7] == 50 and plan[8] == r8["ndoc"] and plan[5] == 50
    B = np.random.default_rng(3).standard_normal((x.shape[1], 16)).astype(np.float32)
    np.testing.assert_allclose(exec_split_plan(plan, B), csr_ref.spmm_csr(rp, ci, v, B), rtol=1e-12, atol=1e-9)
    # the transpose (X^T g of the backward): dense rows first
    rt, ct, vt = csr_ref.coo_to_csr(idx[1], idx[0], x.values().numpy(), (x.shape[1], x.shape[0]))
    pt = build_host_plan(rt, ct, vt, (x.shape[1], x.shape[0]))
    assert pt[0] == SPLIT_MAGIC and pt[7] == 50 and pt[8] == 0
    G = np.random.default_rng(4).standard_normal((x.shape[0], 8)).astype(np.float32)
    np.testing.assert_allclose(exec_split_plan(pt, G), csr_ref.spmm_csr(rt, ct, vt, G), rtol=1e-12, atol=1e-9)
    # a negative threshold keeps the tile path (no split plan)
    assert build_host_plan(rp, ci, v, x.shape, dense=-0.25)[0] == ROW_MAGIC


def test_split_plan_duplicates_and_fallbacks():
    rng = np.random.default_rng(8)
    M, K = 900, 700
    hot = np.sort(rng.choice(K, 20, replace=False))
    rows, cols = [], []
    for r in range(M):
        if 100 <= r < 110:
            c = rng.choice(K, 400, replace=False)
        else:
            c = rng.choice(hot, 8, replace=True)          # duplicates: summed in CSR order
        rows.append(np.full(len(c), r))
        cols.append(c)
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    vals = rng.standard_normal(rows.size).astype(np.float32)
    rp, ci, v = csr_ref.coo_to_csr(rows, cols, vals, (M, K))
    plan = build_host_plan(rp, ci, v, (M, K), hub_min=-1)
    assert plan[0] == SPLIT_MAGIC and plan[7] == 10 and plan[8] == 100
    B = rng.standard_normal((K, 12)).astype(np.float32)
    v32 = v.astype(np.float32).astype(np.float64)             # the plan stores fp32 values
    np.testing.assert_allclose(exec_split_plan(plan, B), csr_ref.spmm_csr(rp, ci, v32, B), rtol=1e-9, atol=1e-9)
    # dense rows not contiguous -> not the split plan
    rows2 = np.where(rows == 105, 500, np.where(rows == 500, 105, rows))
    rp2, ci2, v2 = csr_ref.coo_to_csr(rows2, cols, vals, (M, K))
    assert build_host_plan(rp2, ci2, v2, (M, K), hub_min=-1)[0] == ROW_MAGIC
