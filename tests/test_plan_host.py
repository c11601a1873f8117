"""CPU checks of the SpMM plan builder (gcnk_spmm_plan_build_host: the same
host code the device build runs, writing into host memory): the row-unit +
tile plan's layout and its size query.  The kernels themselves are checked
on the GPU (tests/test_gpu_parity.py); the row-unit control logic by the
Python model in tests/path_model.py.
"""
import numpy as np
import pytest

import gcn_amd  # noqa: F401
from graph_convolutional_networks_for_text_classification_amd import _lib
from oracle import csr_ref

ROW_MAGIC = 0x474E4B35


def build_host_plan(rp, ci, v, shape, groups=1, ipc=12, dense=0.25):
    lib = _lib.load()
    M, K = shape
    rp = np.ascontiguousarray(rp, np.int32)
    ci = np.ascontiguousarray(ci, np.int32)
    v = np.ascontiguousarray(v, np.float32)
    nnz = len(ci)
    nbytes = lib.gcnk_spmm_plan_bytes_host(rp.ctypes.data, ci.ctypes.data, M, K, nnz, ipc, groups, dense)
    assert nbytes > 0, lib.gcnk_last_error()
    buf = np.zeros(nbytes // 4, np.int32)
    rc = lib.gcnk_spmm_plan_build_host(rp.ctypes.data, ci.ctypes.data, v.ctypes.data, M, K, nnz, ipc, groups, dense,
                                       buf.ctypes.data, nbytes)
    assert rc == 0, lib.gcnk_last_error()
    return buf


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


def test_row_plan_layout():
    rng = np.random.default_rng(4)
    rows = rng.integers(0, 2000, 20000)
    cols = rng.integers(0, 2000, 20000)
    rp, ci, v = csr_ref.coo_to_csr(rows, cols, rng.standard_normal(20000).astype(np.float32), (2000, 2000))
    plan = build_host_plan(rp, ci, v, (2000, 2000))
    assert plan[0] == ROW_MAGIC and plan[1] == 2000 and plan[13] == len(ci)
    rp, ci, v = _doc_topic(rng, 600, 12, 288, 500, 6)
    # items are packed {col, value bits} right after the header in CSR order
    plan = build_host_plan(rp, ci, v, (900, 900))
    assert plan[0] == ROW_MAGIC
    items = plan[16:16 + 2 * len(ci)].reshape(-1, 2)
    assert np.array_equal(items[:, 0], ci)
    assert np.array_equal(items[:, 1].view(np.float32), v.astype(np.float32))


def test_plan_rejects_bad_csr():
    lib = _lib.load()
    rp = np.array([0, 2, 1], np.int32)
    ci = np.array([0, 1], np.int32)
    n = lib.gcnk_spmm_plan_bytes_host(rp.ctypes.data, ci.ctypes.data, 2, 2, 2, 8, 1, 0.25)
    assert n == _lib.EARG and b"rowptr" in lib.gcnk_last_error()
    rp = np.array([0, 1, 2], np.int32)
    ci = np.array([0, 5], np.int32)
    n = lib.gcnk_spmm_plan_bytes_host(rp.ctypes.data, ci.ctypes.data, 2, 2, 2, 8, 1, 0.25)
    assert n == _lib.EARG and b"out of range" in lib.gcnk_last_error()


@pytest.mark.parametrize("kind", ["random", "mixed", "doc_topic"])
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
    elif kind == "doc_topic":
        rp, ci, v = _doc_topic(rng, 2000, 30, 900, 400, 5)
        M = K = 2930
    else:
        M, K = 3001, 2003
        rp, ci, v = _random_csr(M, K, 20000, rng, heavy_rows=(5, 1700), heavy_deg=2500, empty_frac=0.2)
    rp, ci, v = (np.ascontiguousarray(a, t) for a, t in ((rp, np.int32), (ci, np.int32), (v, np.float32)))
    nbytes = lib.gcnk_spmm_plan_bytes_host(rp.ctypes.data, ci.ctypes.data, M, K, len(ci), 12, 1, 0.25)
    assert nbytes > 0 and nbytes % 4 == 0
    buf = np.full(nbytes // 4 + 64, -7, np.int32)
    rc = lib.gcnk_spmm_plan_build_host(rp.ctypes.data, ci.ctypes.data, v.ctypes.data, M, K, len(ci), 12, 1, 0.25,
                                       buf.ctypes.data, buf.nbytes)
    assert rc == 0, lib.gcnk_last_error()
    assert buf[0] == ROW_MAGIC
    assert np.all(buf[nbytes // 4:] == -7), "the build wrote past the size plan_bytes reported"
    # no plan word is -7 (ids >= -1, counts >= 0, float bits of -7 would be a NaN),
    # so a sentinel left in the last reported word means the size was too large
    assert buf[nbytes // 4 - 1] != -7, "plan_bytes reported more than the build wrote"




def test_power_law_hub_keeps_short_segments_two_levels():
    """on an R-MAT graph whose hub rows hold ~10^4
    nonzeros the plan keeps every heavy segment at the base length (ipc x the
    workgroup's lane groups; it used to double it past 64 segments) and gives
    such a row a top heavy entry (.w = -2) over groups of <= 64 segments, each
    group's .w the top's slot for its sum; no heavy entry
    has more than 64 slots, slots never overlap, and the units cover every
    nonzero of the heavy rows exactly once."""
    from graph_convolutional_networks_for_text_classification_amd import datasets
    rp, ci, v = (t.numpy() for t in datasets.rmat_csr(16, 1_300_000, seed=2))
    n = len(rp) - 1
    ipc, groups = 12, 1                      # whole-wavefront groups (F > 128): 4-wave segments
    plan = build_host_plan(rp, ci, v, (n, n), groups=groups, ipc=ipc, dense=2.0)
    hdr = plan[:16]
    nnz, nunits, nh, nheavy = hdr[13], hdr[5], hdr[6], hdr[7]
    units = plan[16 + 2 * nnz:16 + 2 * nnz + 4 * nunits].reshape(-1, 4)
    heavy = plan[16 + 2 * nnz + 4 * nunits:16 + 2 * nnz + 4 * nunits + 4 * nheavy].reshape(-1, 4)
    seg = ipc * 4
    deg = np.diff(rp)
    hub = int(np.argmax(deg))
    assert deg[hub] > 64 * seg
    hu = units[:nh][units[:nh, 0] == hub]
    assert len(hu) > 64 and (hu[:, 2] - hu[:, 1]).max() <= seg
    assert (heavy[:, 2] <= 64).all() and (heavy[:, 2] >= 1).all()
    assert (hdr[12] >> 30) & 1, "the plan flags its two-level rows"
    tops = heavy[(heavy[:, 0] == hub) & (heavy[:, 3] == -2)]
    assert len(tops) == 1 and tops[0, 2] > 1
    groups_of_hub = heavy[(heavy[:, 0] == hub) & (heavy[:, 3] >= 0)]
    assert len(groups_of_hub) == tops[0, 2]
    assert groups_of_hub[:, 3].tolist() == list(range(tops[0, 1], tops[0, 1] + tops[0, 2]))
    assert groups_of_hub[:, 2].sum() == len(hu)
    slots = np.concatenate([np.arange(h[1], h[1] + h[2]) for h in heavy])
    assert len(np.unique(slots)) == len(slots) == hdr[14]
    for r in np.unique(units[:nh, 0][units[:nh, 0] >= 0])[:200]:
        u = units[:nh][units[:nh, 0] == r]
        got = np.sort(np.concatenate([np.arange(a, b) for a, b in u[:, 1:3]]))
        assert np.array_equal(got, np.arange(rp[r], rp[r + 1]))
