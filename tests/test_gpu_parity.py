"""GPU parity: the HIP path (through the C-ABI) against the oracle and the
reference's golden vectors.

Tolerances (BASELINE.json north_star: logits within 1e-4 fp32, labels
bit-exact):
  * SpMM / GEMM / colsum vs the float64 oracle: |err| <= 1e-5 * (1 + |ref|)
    scaled by the reduction length where stated;
  * GCN logits vs the reference's golden logits: max |err| <= 1e-4;
  * predicted labels: identical on EVERY row for the reference's trained model
    (tests/golden/r8_trained.npz); for random-init weights, identical on every
    row whose golden top-2 gap exceeds twice the measured max logit error
    (the rows below it are counted and bounded).
"""
import os

import numpy as np
import pytest
import torch

import gcn_amd  # noqa: F401
from graph_convolutional_networks_for_text_classification_amd import (
    GCN, _lib, colsum, datasets, from_arrays, gemm, spmm)
from graph_convolutional_networks_for_text_classification_amd.sparse import from_torch
from oracle import csr_ref, gcn_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
LOGIT_TOL = 1e-4
TRAINED_LOGIT_TOL = 3e-4   # absolute, trained-model logits up to |190| (see the test)


def _close(got, ref, rtol=1e-5, atol=1e-5):
    got = got.detach().double().cpu().numpy() if isinstance(got, torch.Tensor) else got
    err = np.abs(got - ref)
    bound = atol + rtol * np.abs(ref)
    assert np.all(err <= bound), f"max err {err.max():.3e} (bound at worst {bound.flat[np.argmax(err - bound)]:.3e})"


def _grads_close(got, want, name, rtol=1e-4, kink_frac=1e-3):
    """Gradients of two fp32 associations of the same forward (e.g. (A-hat X) W1
    against A-hat (X W1)): every element within rtol (atol 1e-5 of the largest),
    except where an element of Z1 that sits within rounding of 0 took the other
    side of the ReLU in one of them (its whole gZ1 entry then differs, and so do
    the gW1 / gb1 terms it feeds): at most `kink_frac` of the elements (or 2),
    each still within 1e-2 relative / 10x the absolute bound."""
    atol = 1e-5 * max(1.0, float(np.abs(want).max()))
    bad = np.abs(got - want) > atol + rtol * np.abs(want)
    assert bad.sum() <= max(2, kink_frac * bad.size), f"{name}: {int(bad.sum())} of {bad.size} elements off"
    np.testing.assert_allclose(got, want, rtol=1e-2, atol=10 * atol, err_msg=name)


def _random_csr(M, K, nnz, rng, heavy_rows=(), heavy_deg=0, empty_frac=0.0):
    rows = rng.integers(0, M, nnz)
    if empty_frac > 0:
        allowed = np.flatnonzero(rng.random(M) >= empty_frac)
        rows = allowed[rng.integers(0, len(allowed), nnz)]
    cols = rng.integers(0, K, nnz)
    for h in heavy_rows:
        rows = np.concatenate([rows, np.full(heavy_deg, h)])
        cols = np.concatenate([cols, rng.integers(0, K, heavy_deg)])
    vals = rng.standard_normal(len(rows)).astype(np.float32)
    return csr_ref.coo_to_csr(rows, cols, vals, (M, K))


def test_native_library_is_loaded():
    lib = _lib.load()
    assert lib.gcnk_abi_version() == _lib.ABI_VERSION
    with open("/proc/self/maps") as f:
        assert _lib.LIB_PATH in f.read()


@pytest.mark.parametrize("F", [200, 8])
def test_spmm_r8_adjacency(r8, F):
    adj = r8["adj"].to(DEV)
    a = from_torch(adj)
    rp, ci, v = (x.cpu().numpy() for x in (a.rowptr, a.colind, a.val))
    B = torch.randn(r8["nodes"], F, generator=torch.Generator().manual_seed(F))
    got = spmm(a, B.to(DEV))
    ref = csr_ref.spmm_csr(rp, ci, v, B.numpy())
    _close(got, ref)
    # low dense threshold: document rows run as MFMA tiles over the 50 topic
    # columns with the self loop kept aside (diagonal epilogue)
    got_t = spmm(a, B.to(DEV), dense=0.05)
    _close(got_t, ref)
    hdr = [p for k, p in a._plans.items() if abs(k[2]) == 0.05][0].header
    assert hdr[8] > 0 and (hdr[12] & 1) == 1, "R8 document rows: MFMA tiles over the topic columns + diagonal"


@pytest.mark.parametrize("F", [1, 3, 7, 8, 16, 64, 100, 200, 256, 257, 1000, 4096])
def test_spmm_widths_with_heavy_and_empty_rows(F):
    rng = np.random.default_rng(F)
    M, K = 3001, 2003
    rp, ci, v = _random_csr(M, K, 20000, rng, heavy_rows=(5, 1700, 3000), heavy_deg=2500, empty_frac=0.2)
    a = from_arrays(rp, ci, v, (M, K), DEV)
    B = rng.standard_normal((K, F)).astype(np.float32)
    got = spmm(a, torch.from_numpy(B).to(DEV))
    _close(got, csr_ref.spmm_csr(rp, ci, v, B), rtol=1e-5, atol=2e-5 * np.sqrt(2500))


@pytest.fixture(scope="module")
def rmat17():
    """A power-law graph (SURVEY §8(d) row 4's R-MAT(0.57, 0.19, 0.19), scale 17:
    131,072 nodes, 2.6M edges drawn; its heaviest rows hold ~10^4 nonzeros,
    far beyond 64 segments of ipc) as host CSR arrays."""
    rp, ci, v = datasets.rmat_csr(17, 2_621_440, seed=5)
    return rp.numpy(), ci.numpy(), v.numpy()


@pytest.mark.parametrize("F", [8, 64, 256])
def test_spmm_power_law_rows_and_linearity(rmat17, F):
    """The SpMM on the R-MAT graph: its 16 heaviest rows, every empty-row kind
    and 400 random rows against the float64 oracle (csr_ref.spmm_csr on the
    sampled rows), the whole product linear (A (B1 + 2 B2) = A B1 + 2 A B2
    to fp32 reassociation), bitwise reproducible."""
    rp, ci, v = rmat17
    n = len(rp) - 1
    deg = np.diff(rp)
    assert deg.max() > 64 * 32, deg.max()   # a row past 64 segments of the largest ipc
    a = from_arrays(rp, ci, v, (n, n), DEV)
    rng = np.random.default_rng(F)
    B1 = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(DEV)
    B2 = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(DEV)
    C1 = spmm(a, B1)
    if F == 256:   # rows past 64 segments: groups + the top-entry launch (spmm_heavy_top_kernel)
        assert any((p.header[12] >> 30) & 1 for p in a._plans.values())
    rows = np.unique(np.concatenate([np.argsort(deg)[-16:], rng.choice(n, 400, replace=False),
                                     np.flatnonzero(deg == 0)[:8]]))
    sub_rp = np.concatenate([[0], np.cumsum(deg[rows])])
    sub_ci = np.concatenate([ci[rp[r]:rp[r + 1]] for r in rows])
    sub_v = np.concatenate([v[rp[r]:rp[r + 1]] for r in rows])
    want = csr_ref.spmm_csr(sub_rp, sub_ci, sub_v, B1.cpu().numpy())
    _close(C1[torch.from_numpy(rows).to(DEV)], want, rtol=1e-5, atol=2e-5 * np.sqrt(deg.max()))
    lin = spmm(a, B1 + 2 * B2)
    both = C1 + 2 * spmm(a, B2)
    scale = float(both.abs().max())
    assert float((lin - both).abs().max()) <= 1e-5 * max(1.0, scale) * np.sqrt(deg.max() / 100)
    assert torch.equal(spmm(a, B1), C1)


@pytest.mark.parametrize("F,ipc,lanes", [(64, 4, 64), (64, None, None), (8, 4, 0), (200, None, None)])
def test_spmm_heavy_rows_at_the_combine_boundaries(F, ipc, lanes):
    """Rows around the plan's combine boundaries (csrc/spmm.hip: 64 segments
    per combine, groups of <= 64 under a top entry past that, segment length
    doubled only past 4,096 segments): degrees one below / at / above 64 and
    128 segments of the smallest segment (ipc 4 x 4 waves = 16), a row of
    70,000 nonzeros (4,375 segments of 16: the doubling), empty and light
    rows; against the float64 oracle, bitwise reproducible."""
    rng = np.random.default_rng(F + (ipc or 0))
    K = 80_000
    degs = [1023, 1024, 1025, 2047, 2049, 70_000, 0, 5, 1, 300]
    rows, cols = [], []
    for r, d in enumerate(degs):
        span = K // 8 if r < 5 else K   # (one column class: one run, exact segment counts)
        c = np.sort(rng.choice(span, d, replace=False)) if d else np.zeros(0, np.int64)
        rows.append(np.full(d, r))
        cols.append(c)
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    rp, ci, v = csr_ref.coo_to_csr(rows, cols, rng.standard_normal(rows.size), (len(degs), K))
    a = from_arrays(rp, ci, v, (len(degs), K), DEV)
    B = rng.standard_normal((K, F)).astype(np.float32)
    Bt = torch.from_numpy(B).to(DEV)
    kw = {} if ipc is None else {"ipc": ipc, "lanes": lanes}
    got = spmm(a, Bt, **kw)
    _close(got, csr_ref.spmm_csr(rp, ci, v, B), rtol=1e-5, atol=2e-5 * np.sqrt(70_000))
    assert torch.equal(spmm(a, Bt, **kw), got)


@pytest.mark.parametrize("ipc", [4, 8, 12, 16, 32, 64])
@pytest.mark.parametrize("lanes", [0, 16, 32])
def test_spmm_schedule_variants(ipc, lanes):
    """Every light-row limit / lane layout computes the same product (light
    units, single- and multi-segment heavy rows and the last-arriver combine
    are exercised)."""
    rng = np.random.default_rng(ipc * 100 + lanes)
    M, K, F = 1500, 900, 200
    rp, ci, v = _random_csr(M, K, 9000, rng, heavy_rows=(0, 749, 1499), heavy_deg=700, empty_frac=0.1)
    a = from_arrays(rp, ci, v, (M, K), DEV)
    B = rng.standard_normal((K, F)).astype(np.float32)
    got = spmm(a, torch.from_numpy(B).to(DEV), ipc=ipc, lanes=lanes)
    _close(got, csr_ref.spmm_csr(rp, ci, v, B), atol=2e-5 * np.sqrt(700))


def _mixed_density_csr(rng, M, K):
    """Row blocks of every kind the hybrid plan distinguishes: a dense band over
    few columns (R8 X's document rows; contiguous, and strided so the tile
    kernel's column-list path runs too), fully dense rows spanning several
    64-column chunks (X's topic rows), heavy sparse rows, light rows, empty rows."""
    rows, cols = [], []
    for r in range(M):
        if r < 130:                       # dense over columns 0..49 (+ the diagonal past 50)
            c = np.arange(50) if r < 50 else np.concatenate([np.arange(50), [r]])
        elif 200 <= r < 264:              # dense over a strided column set (a non-contiguous condensed chunk)
            c = 100 + 3 * np.arange(60)
        elif 300 <= r < 341:              # fully dense
            c = np.arange(K)
        elif 400 <= r < 600:              # self loop + 4 of 50 "topic" columns (Â's document rows)
            c = np.concatenate([[r], 800 + rng.choice(50, 4, replace=False)])
        elif r % 97 == 5:                 # heavy sparse
            c = rng.choice(K, 400, replace=False)
        elif r % 7 == 0:                  # empty
            c = np.zeros(0, np.int64)
        else:
            c = rng.choice(K, int(rng.integers(1, 9)), replace=False)
        rows.append(np.full(len(c), r))
        cols.append(c)
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    return csr_ref.coo_to_csr(rows, cols, rng.standard_normal(rows.size).astype(np.float32), (M, K))


@pytest.mark.parametrize("F", [1, 7, 8, 64, 200, 256, 300])
@pytest.mark.parametrize("M", [700, 900])
def test_spmm_hybrid_dense_blocks(F, M):
    """Tile path (single- and multi-chunk dense blocks + slab reduce) beside the
    row kernel; a square operand keeps its diagonal aside (added in the tile
    epilogue), a rectangular one has none."""
    rng = np.random.default_rng(F + 1)
    K = 900
    rp, ci, v = _mixed_density_csr(rng, M, K)
    a = from_arrays(rp, ci, v, (M, K), DEV)
    B = rng.standard_normal((K, F)).astype(np.float32)
    bias = rng.standard_normal(F).astype(np.float32)
    mask = (rng.random((M, F)) < 0.6).astype(np.uint8)
    got = spmm(a, torch.from_numpy(B).to(DEV), bias=torch.from_numpy(bias).to(DEV),
               epilogue=_lib.EPI_BIAS_RELU_DROP, mask=torch.from_numpy(mask).to(DEV), scale=1.5)
    acc = csr_ref.spmm_csr(rp, ci, v, B)
    _close(got, csr_ref.spmm_epilogue(acc, bias, relu=True, mask=mask, scale=1.5), atol=2e-5 * np.sqrt(K))
    hdr = list(a._plans.values())[0].header
    assert hdr[8] > 0 and hdr[9] > 0, "dense blocks (single and multi-chunk) expected on the tile path"
    assert (hdr[12] & 1) == (1 if M == K else 0), "diagonal entries of a square operand's tile rows are kept aside"
    # tile path disabled: the row kernel alone gives the same product
    got2 = spmm(a, torch.from_numpy(B).to(DEV), dense=2.0)
    _close(got2, acc, atol=2e-5 * np.sqrt(K))


def test_csr_to_dense_sums_duplicates_in_order():
    """gcnk_csr_to_dense: every element once, duplicates summed in CSR order,
    columns past K untouched (ld > K)."""
    from graph_convolutional_networks_for_text_classification_amd import _lib
    from graph_convolutional_networks_for_text_classification_amd.ops import _ptr, _stream
    rng = np.random.default_rng(9)
    M, K = 300, 150
    rows = rng.integers(0, M, 6000)
    cols = rng.integers(0, K, 6000)
    order = np.lexsort((cols, rows))
    rows, cols = rows[order], cols[order]                 # sorted, duplicates kept
    vals = rng.standard_normal(6000).astype(np.float32)
    rp = np.zeros(M + 1, np.int32)
    np.add.at(rp, rows + 1, 1)
    rp = np.cumsum(rp).astype(np.int32)
    want = np.zeros((M, K + 8), np.float32)
    for r, c, v in zip(rows, cols, vals):
        want[r, c] = np.float32(want[r, c] + v)
    want[:, K:] = 7.0
    out = torch.full((M, K + 8), 7.0, device=DEV)
    t = [torch.from_numpy(x).to(DEV) for x in (rp, cols.astype(np.int32), vals)]
    rc = _lib.load().gcnk_csr_to_dense(_ptr(t[0]), _ptr(t[1]), _ptr(t[2]), M, K, _ptr(out), out.stride(0),
                                       _stream(out.device))
    assert rc == 0
    assert np.array_equal(out.cpu().numpy(), want)
    # strictly increasing columns (the fast scatter path), rows of every length
    rp2, ci2, v2 = _random_csr(M, K, 20000, rng, empty_frac=0.1)
    want2 = np.zeros((M, K + 8), np.float32)
    for r in range(M):
        want2[r, ci2[rp2[r]:rp2[r + 1]]] = v2[rp2[r]:rp2[r + 1]]
    want2[:, K:] = 7.0
    out2 = torch.full((M, K + 8), 7.0, device=DEV)
    t2 = [torch.from_numpy(np.ascontiguousarray(x)).to(DEV) for x in (rp2.astype(np.int32), ci2.astype(np.int32),
                                                                       v2.astype(np.float32))]
    assert _lib.load().gcnk_csr_to_dense(_ptr(t2[0]), _ptr(t2[1]), _ptr(t2[2]), M, K, _ptr(out2), out2.stride(0),
                                         _stream(out2.device)) == 0
    assert np.array_equal(out2.cpu().numpy(), want2)




@pytest.mark.parametrize("P", [1, 8, 20, 33])
@pytest.mark.parametrize("store_main", [True, False])
def test_spmm_fused_projection(r8, P, store_main):
    """H = relu(A S + b) * dropout, S2 = H W2 in one pass (gcnk_spmm_proj_f32,
    [M, P]); wider P exercises the unfused fallback.  Then the consumer:
    A S2 + b2 against the oracle."""
    from graph_convolutional_networks_for_text_classification_amd.ops import spmm_proj
    a = from_torch(r8["adj"].to(DEV))
    rng = np.random.default_rng(P)
    N, F = r8["nodes"], 200
    S = rng.standard_normal((N, F)).astype(np.float32)
    W = rng.standard_normal((F, P)).astype(np.float32)
    b = rng.standard_normal(F).astype(np.float32)
    b2 = rng.standard_normal(P).astype(np.float32)
    mask = (rng.random((N, F)) < 0.5).astype(np.uint8)
    H, S2 = spmm_proj(a, torch.from_numpy(S).to(DEV), torch.from_numpy(W).to(DEV), bias=torch.from_numpy(b).to(DEV),
                      epilogue=_lib.EPI_BIAS_RELU_DROP, mask=torch.from_numpy(mask).to(DEV), scale=2.0,
                      store_main=store_main)
    rp, ci, v = (t.cpu().numpy() for t in (a.rowptr, a.colind, a.val))
    Href = csr_ref.spmm_epilogue(csr_ref.spmm_csr(rp, ci, v, S), b, relu=True, mask=mask, scale=2.0)
    if store_main:
        _close(H, Href, atol=2e-5)
    else:
        assert H is None
    S2ref = Href @ W.astype(np.float64)
    _close(S2, S2ref, atol=2e-4)
    Z = spmm(a, S2, bias=torch.from_numpy(b2).to(DEV), epilogue=_lib.EPI_BIAS)
    _close(Z, csr_ref.spmm_epilogue(csr_ref.spmm_csr(rp, ci, v, S2ref), b2), atol=4e-4)
    assert torch.equal(Z, spmm(a, S2, bias=torch.from_numpy(b2).to(DEV), epilogue=_lib.EPI_BIAS))


def test_spmm_deterministic():
    rng = np.random.default_rng(7)
    rp, ci, v = _random_csr(2000, 2000, 30000, rng, heavy_rows=(3,), heavy_deg=9000)
    a = from_arrays(rp, ci, v, (2000, 2000), DEV)
    B = torch.randn(2000, 200, device=DEV)
    o1, o2 = spmm(a, B), spmm(a, B)
    assert torch.equal(o1, o2)


@pytest.mark.parametrize("kind", ["r8", "random"])
def test_spmm_two_streams_share_one_plan_concurrently(r8, kind):
    """Reentrancy (gcnk.h threading contract): two streams run SpMMs on the same
    cached operand at the same time, with different inputs and outputs.  The
    heavy-row arrival counters live in a per-stream region
    (sparse.Plan.counters), so neither can corrupt the other: every output
    equals the single-stream result bit for bit."""
    rng = np.random.default_rng(17)
    if kind == "r8":
        a, K = from_torch(r8["adj"].to(DEV)), r8["nodes"]
    else:   # multi-segment heavy rows (tile path off)
        M, K = 3001, 20003
        rp, ci, v = _random_csr(M, K, 20000, rng, heavy_rows=(5, 1700, 3000), heavy_deg=2500)
        a = from_arrays(rp, ci, v, (M, K), DEV)
    F = 200
    Bs = [torch.from_numpy(rng.standard_normal((K, F)).astype(np.float32)).to(DEV) for _ in range(2)]
    dense = 2.0
    ref = [spmm(a, B, dense=dense) for B in Bs]
    plan = list(a._plans.values())[-1]
    assert plan.counter_bytes() > 0, "multi-segment heavy rows use arrival counters"
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [[torch.empty_like(ref[i]) for _ in range(24)] for i in range(2)]
    torch.cuda.synchronize()
    for it in range(24):
        for i in range(2):
            with torch.cuda.stream(streams[i]):
                spmm(a, Bs[i], out=outs[i][it], dense=dense)
    torch.cuda.synchronize()
    for i in range(2):
        for o in outs[i]:
            assert torch.equal(o, ref[i])
    assert len(plan._counters) >= 3, "one counter region per stream"


def test_spmm_epilogues_and_strided_operands():
    rng = np.random.default_rng(11)
    M, K, F = 700, 500, 64
    rp, ci, v = _random_csr(M, K, 5000, rng, heavy_rows=(1,), heavy_deg=400)
    a = from_arrays(rp, ci, v, (M, K), DEV)
    Bfull = rng.standard_normal((K, 3 * F)).astype(np.float32)
    Bt = torch.from_numpy(Bfull).to(DEV)[:, F:2 * F]          # ldb = 3F > F
    bias = rng.standard_normal(F).astype(np.float32)
    mask = (rng.random((M, F)) < 0.5).astype(np.uint8)
    acc = csr_ref.spmm_csr(rp, ci, v, Bfull[:, F:2 * F])
    bt = torch.from_numpy(bias).to(DEV)
    _close(spmm(a, Bt, bias=bt, epilogue=_lib.EPI_BIAS), csr_ref.spmm_epilogue(acc, bias))
    _close(spmm(a, Bt, bias=bt, epilogue=_lib.EPI_BIAS_RELU), csr_ref.spmm_epilogue(acc, bias, relu=True))
    _close(spmm(a, Bt, bias=bt, epilogue=_lib.EPI_BIAS_RELU_DROP, mask=torch.from_numpy(mask).to(DEV), scale=2.0),
           csr_ref.spmm_epilogue(acc, bias, relu=True, mask=mask, scale=2.0))
    out = torch.full((M, 2 * F), 7.0, device=DEV)[:, :F]       # ldc = 2F
    spmm(a, Bt, out=out)
    _close(out, acc)
    # hash-RNG dropout: kept fraction ~ keep_prob and kept values == relu(.)*scale
    h = spmm(a, Bt, bias=bt, epilogue=_lib.EPI_BIAS_RELU_HASH, scale=2.0, keep_prob=0.5, seed=123).cpu().numpy()
    relu = csr_ref.spmm_epilogue(acc, bias, relu=True)
    pos = relu > 1e-3
    kept = h[pos] != 0
    assert 0.45 < kept.mean() < 0.55
    np.testing.assert_allclose(h[pos][kept], 2 * relu[pos][kept], rtol=1e-5, atol=1e-5)


def test_spmm_coo_input_with_duplicates_and_shuffled_order():
    rng = np.random.default_rng(5)
    M, K, F = 400, 300, 8
    rows = rng.integers(0, M, 3000)
    cols = rng.integers(0, K, 3000)
    rows = np.concatenate([rows, rows[:500]])   # duplicates
    cols = np.concatenate([cols, cols[:500]])
    vals = rng.standard_normal(len(rows)).astype(np.float32)
    perm = rng.permutation(len(rows))
    t = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows[perm], cols[perm]])),
                                torch.from_numpy(vals[perm]), (M, K)).to(DEV)
    B = rng.standard_normal((K, F)).astype(np.float32)
    rp, ci, v = csr_ref.coo_to_csr(rows, cols, vals, (M, K))
    _close(spmm(t, torch.from_numpy(B).to(DEV)), csr_ref.spmm_csr(rp, ci, v, B))


def test_coo_to_csr_matches_aten_coalesce(r8):
    """gcnk_coo_to_csr (sparse.from_torch) against ATen's own coalesce -- what
    th.spmm does to the reference's uncoalesced COO on every call -- bit for
    bit: R8's column-major A-hat (utils.py:196-203), R8's row-major X
    (trainer.py:226-238), and a shuffled COO with duplicates; an out-of-range
    index raises."""
    rng = np.random.default_rng(21)
    M, K = 900, 700
    rows = rng.integers(0, M, 9000)
    cols = rng.integers(0, K, 9000)
    rows = np.concatenate([rows, rows[:3000], rows[:100]])
    cols = np.concatenate([cols, cols[:3000], cols[:100]])
    vals = rng.standard_normal(rows.size).astype(np.float32)
    perm = rng.permutation(rows.size)
    dup = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows[perm], cols[perm]])),
                                  torch.from_numpy(vals[perm]), (M, K))
    for t in (r8["adj"], r8["features"], dup):
        c = t.coalesce()
        a = from_torch(t.to(DEV))
        want_rp = np.concatenate([[0], np.cumsum(np.bincount(c.indices()[0].numpy(), minlength=t.shape[0]))])
        assert np.array_equal(a.rowptr.cpu().numpy(), want_rp)
        assert np.array_equal(a.colind.cpu().numpy(), c.indices()[1].numpy())
        if t is dup:
            # >= 3 duplicates: we sum in input order; ATen's CPU coalesce sorts
            # unstably, so its fp32 order (hence the last bit) is not defined
            np.testing.assert_allclose(a.val.cpu().numpy(), c.values().numpy(), rtol=1e-6, atol=1e-6)
        else:   # the reference's own tensors (no duplicates): bit for bit
            assert np.array_equal(a.val.cpu().numpy().view(np.uint32), c.values().numpy().view(np.uint32))
    bad = torch.sparse_coo_tensor(torch.tensor([[0, 5], [1, 2]]), torch.tensor([1.0, 2.0]), (4, 4))
    with pytest.raises(RuntimeError, match="outside its shape"):
        from_torch(bad.to(DEV))


def test_empty_graph_and_empty_rows_only():
    a = from_arrays(np.zeros(11, np.int32), np.zeros(0, np.int32), np.zeros(0, np.float32), (10, 5), DEV)
    bias = torch.arange(8, dtype=torch.float32, device=DEV)
    out = spmm(a, torch.randn(5, 8, device=DEV), bias=bias, epilogue=_lib.EPI_BIAS)
    assert torch.equal(out, bias.expand(10, 8))


def test_csr_transpose_matches_oracle():
    rng = np.random.default_rng(3)
    M, K = 1200, 777
    rp, ci, v = _random_csr(M, K, 15000, rng, heavy_rows=(9,), heavy_deg=500, empty_frac=0.3)
    a = from_arrays(rp, ci, v, (M, K), DEV)
    t = a.t()
    rpt, cit, vt = csr_ref.csr_transpose(rp, ci, v, (M, K))
    assert np.array_equal(t.rowptr.cpu().numpy(), rpt)
    assert np.array_equal(t.colind.cpu().numpy(), cit)
    assert np.array_equal(t.val.cpu().numpy(), vt.astype(np.float32))


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("shape", [(7724, 8, 200), (200, 8, 7724), (7724, 200, 8), (33, 70, 5), (1, 1, 1),
                                   (18916, 200, 100), (7724, 20, 200), (1000, 40, 200), (257, 332, 97),
                                   (1000, 124, 128), (77, 68, 4), (130, 336, 64),
                                   (18916, 20, 200), (16400, 64, 256), (16385, 8, 100)])
def test_gemm_mfma(ta, tb, shape):
    """Every GEMM kernel against the float64 oracle: the LDS-tiled MFMA kernel
    (with transposes), the short-K wide-N one (NN, K <= 128, N > 64: a dense
    gensim-style X W1 at 18916 x 100 x 200; K = 4 .. 128, partial row blocks and
    column slices) and the skinny-N K-split one (N <= 64: gc2's H1 W2 at 8, 20
    and 40 classes; 20ng-sized and partial workgroups)."""
    M, N, K = shape
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    got = gemm(A.to(DEV), B.to(DEV), transA=ta, transB=tb)
    ref = csr_ref.gemm(A.numpy(), B.numpy(), ta, tb)
    _close(got, ref, rtol=1e-5, atol=2e-6 * np.sqrt(K) * 4)


@pytest.mark.parametrize("shape", [(50, 200, 7463), (64, 200, 8192), (1, 4, 512), (17, 116, 1000),
                                   (63, 332, 4099)])
@pytest.mark.parametrize("split", [None, 8, 117, 234, 600])
def test_gemm_small_m_split_k(shape, split):
    """The small-M long-K split-K kernel + its slab reduce (X[hubs] W1 of the
    factored gc1: R8 [50 x 7463] x [7463 x 200]) against the float64 oracle, on
    A rows padded to a multiple of 4 (garbage in the padding, never
    multiplied), every k chunk size and ragged M, N, K; bitwise reproducible."""
    M, N, K = shape
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    Ap = torch.full((M, (K + 3) // 4 * 4), float("nan"))
    Ap[:, :K] = A
    Ad = Ap.to(DEV)[:, :K]
    assert Ad.stride(0) % 4 == 0
    got = gemm(Ad, B.to(DEV), split_k=split)
    _close(got, A.double().numpy() @ B.double().numpy(), rtol=1e-5, atol=2e-6 * np.sqrt(K) * 4)
    assert torch.equal(got, gemm(Ad, B.to(DEV), split_k=split))


def test_gemm_epilogues_and_split_k():
    g = torch.Generator().manual_seed(1)
    A = torch.randn(500, 96, generator=g)
    B = torch.randn(96, 40, generator=g)
    bias = torch.randn(40, generator=g)
    R = torch.relu(torch.randn(500, 40, generator=g))
    ref = A.double().numpy() @ B.double().numpy()
    d = {k: v.to(DEV) for k, v in dict(A=A, B=B, bias=bias, R=R).items()}
    _close(gemm(d["A"], d["B"], bias=d["bias"], epilogue=_lib.GEMM_EPI_BIAS), ref + bias.double().numpy())
    _close(gemm(d["A"], d["B"], bias=d["bias"], epilogue=_lib.GEMM_EPI_BIAS_RELU),
           np.maximum(ref + bias.double().numpy(), 0))
    _close(gemm(d["A"], d["B"], epilogue=_lib.GEMM_EPI_MASK_POS, R=d["R"], scale=2.0),
           np.where(R.numpy() > 0, 2 * ref, 0.0))
    for s in (1, 2, 3, 8):
        _close(gemm(d["A"], d["B"], split_k=s), ref, atol=1e-4)
    # the same epilogues on the short-K wide-N kernel (K = 100, N = 200)
    A2 = torch.randn(300, 100, generator=g)
    B2 = torch.randn(100, 200, generator=g)
    b2 = torch.randn(200, generator=g)
    R2 = torch.relu(torch.randn(300, 200, generator=g))
    ref2 = A2.double().numpy() @ B2.double().numpy()
    d2 = {k: v.to(DEV) for k, v in dict(A=A2, B=B2, bias=b2, R=R2).items()}
    _close(gemm(d2["A"], d2["B"], bias=d2["bias"], epilogue=_lib.GEMM_EPI_BIAS_RELU),
           np.maximum(ref2 + b2.double().numpy(), 0), atol=1e-4)
    _close(gemm(d2["A"], d2["B"], epilogue=_lib.GEMM_EPI_MASK_POS, R=d2["R"], scale=2.0),
           np.where(R2.numpy() > 0, 2 * ref2, 0.0), atol=1e-4)


@pytest.mark.parametrize("M,N,P,ldpad", [(7724, 200, 8, 0), (18916, 200, 20, 0), (1000, 7, 3, 0),
                                          (3001, 300, 16, 4), (50, 1030, 5, 2), (70000, 64, 8, 0)])
def test_gcn_bwd2_fused_backward(M, N, P, ldpad):
    """gcnk_gcn_bwd2_f32 (gc2 + ReLU/dropout backward in one pass over H1)
    against float64: gZ1 = (H1 > 0) ? scale * gS2 W2^T : 0, gW2 = H1^T gS2,
    gb1 = colsum(gZ1), gb2 = colsum(G); float4 / float2 / scalar column paths,
    several 256-column slices, strided H1, more rows than one LDS stage.
    Bitwise identical on a second call."""
    from graph_convolutional_networks_for_text_classification_amd.ops import gcn_bwd2
    rng = np.random.default_rng(M + N + P)
    Hf = rng.standard_normal((M, N + ldpad)).astype(np.float32)
    Hf[rng.random((M, N + ldpad)) < 0.4] = 0.0          # dropped / non-positive entries
    Hf = np.maximum(Hf, 0) * 2.0
    gS = rng.standard_normal((M, P)).astype(np.float32)
    W = rng.standard_normal((N, P)).astype(np.float32)
    G = rng.standard_normal((M, P)).astype(np.float32)
    Ht = torch.from_numpy(Hf).to(DEV)[:, :N]
    args = [torch.from_numpy(x).to(DEV) for x in (gS, W, G)]
    gZ, gW, gb1, gb2 = gcn_bwd2(Ht, args[0], args[1], G=args[2], scale=2.0)
    H = Hf[:, :N].astype(np.float64)
    zref = np.where(H > 0, 2.0 * (gS.astype(np.float64) @ W.astype(np.float64).T), 0.0)
    _close(gZ, zref, atol=1e-4)
    _close(gW, H.T @ gS.astype(np.float64), atol=2e-5 * np.sqrt(M) * 4)
    _close(gb1, zref.sum(0), atol=2e-5 * np.sqrt(M) * 4)
    _close(gb2, G.astype(np.float64).sum(0), atol=2e-5 * np.sqrt(M))
    again = gcn_bwd2(Ht, args[0], args[1], G=args[2], scale=2.0)
    assert all(torch.equal(x, y) for x, y in zip((gZ, gW, gb1, gb2), again))
    z2, w2, b1, b2 = gcn_bwd2(Ht, args[0], args[1], scale=1.0, want_gw=False, want_gb1=False)
    assert w2 is None and b1 is None and b2 is None
    _close(z2, zref / 2.0, atol=1e-4)


def test_colsum():
    X = torch.randn(7724, 200, generator=torch.Generator().manual_seed(2))
    _close(colsum(X.to(DEV)), csr_ref.colsum(X.numpy()), atol=1e-4)


# ------------------------------------------------------------------------------ GCN level

def _labels_check(got, golden):
    """Labels must agree on every row whose golden top-2 gap exceeds twice the
    MEASURED max logit error (no error that small can reorder two logits
    further apart); returns the number of rows below that gap."""
    err = float(np.abs(got - golden).max())
    srt = np.sort(golden, axis=1)
    gap = srt[:, -1] - srt[:, -2]
    decided = gap > 2 * err
    same = got.argmax(1) == golden.argmax(1)
    assert np.all(same[decided]), f"{np.sum(~same[decided])} rows with top-2 gap > 2 x max err {err:.2e} changed label"
    return int(np.sum(~decided))


@pytest.mark.parametrize("seed", [50494, 99346, 0])
def test_gcn_eval_logits_match_reference(r8, golden_logits, seed):
    """Random-init weights (the reference init for the seed): logits within
    1e-4; labels identical wherever the golden gap exceeds 2x the measured
    error (random-init logits have near-ties down to 1.25e-6)."""
    torch.manual_seed(seed)
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(DEV)
    m.eval()
    with torch.no_grad():
        lg = m(r8["features"].to(DEV), r8["adj"].to(DEV)).cpu().numpy()
    gold = golden_logits[f"eval_{seed}"]
    err = float(np.abs(lg - gold).max())
    assert err <= LOGIT_TOL
    undecided = _labels_check(lg, gold)
    flips = int(np.sum(lg.argmax(1) != gold.argmax(1)))
    print(f"seed {seed}: max err {err:.2e}; labels bit-exact on {len(gold) - undecided} rows; "
          f"{undecided} rows within 2x that error of a tie; {flips} labels differ")
    assert undecided <= 3 and flips <= undecided


def test_trained_model_labels_bit_exact_on_every_row(r8, trained_golden):
    """The reference's TRAINED model (seed 50494, 72 epochs; its min top-2 gap
    is 5.1e-3) loaded into the HIP GCN: the predicted label of EVERY node is
    the reference's -- no exclusions -- so the test accuracy is the
    reference's to the last document.

    Logits: trained logits reach |190|, where fp32 itself is coarse -- the
    reference's own CPU result is 1.9e-4 away from the float64 forward (its
    7,463-term dot products accumulate in one serial fp32 chain).  A 1e-4
    bound against the reference would demand reproducing its rounding
    sequence; instead the HIP forward must be at least as close to the
    float64 truth as the reference is, and within TRAINED_LOGIT_TOL of the
    reference's logits in absolute terms (observed on MI355X: 1.83e-4, printed
    below; the reference's own distance to float64 is 1.9e-4)."""
    import scipy.sparse as ssp
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(DEV)
    m.load_state_dict(trained_golden["state_dict"])
    m.eval()
    with torch.no_grad():
        lg = m(r8["features"].to(DEV), r8["adj"].to(DEV)).cpu().numpy()
    gold = trained_golden["logits"]
    sd = {k: v.double().numpy() for k, v in trained_golden["state_dict"].items()}
    x = r8["features"].coalesce()
    X = ssp.csr_matrix((x.values().double().numpy(), x.indices().numpy()), shape=tuple(x.shape))
    a = r8["adj"].coalesce()
    A = ssp.csr_matrix((a.values().double().numpy(), a.indices().numpy()), shape=tuple(a.shape))
    H1 = np.maximum(A @ (X @ sd["gc1.weight"]) + sd["gc1.bias"], 0.0)
    truth = A @ (H1 @ sd["gc2.weight"]) + sd["gc2.bias"]
    err_ref = float(np.abs(gold - truth).max())
    err_hip = float(np.abs(lg - truth).max())
    err = float(np.abs(lg - gold).max())
    scale = float(np.abs(gold).max())
    print(f"trained model: |logit| <= {scale:.1f}; max err vs reference {err:.2e}; vs float64: reference "
          f"{err_ref:.2e}, HIP {err_hip:.2e}")
    assert err_hip <= err_ref and err <= TRAINED_LOGIT_TOL
    assert np.array_equal(lg.argmax(1), gold.argmax(1)), f"{int(np.sum(lg.argmax(1) != gold.argmax(1)))} labels differ"
    test = np.asarray(r8["test_lst"])
    acc = float(np.mean(lg[test].argmax(1) == np.asarray(r8["target"])[test]))
    assert acc == trained_golden["test_acc"]


def test_graph_convolution_without_bias_forward_backward(r8):
    """GraphConvolution(bias=False) (layer.py:62 registers bias=None and :111-112
    returns the product alone) through the HIP path: forward and the gradients
    of W and of a dense input against the oracle's reference module."""
    from graph_convolutional_networks_for_text_classification_amd import GraphConvolution
    torch.manual_seed(4)
    gc = GraphConvolution(200, 16, bias=False).to(DEV)
    assert gc.bias is None and "bias" not in dict(gc.named_parameters())
    ref = gcn_ref.RefGraphConvolution(200, 16, bias=False)
    ref.load_state_dict({k: v.cpu() for k, v in gc.state_dict().items()})
    H = torch.randn(r8["nodes"], 200, generator=torch.Generator().manual_seed(5))
    Hd = H.clone().to(DEV).requires_grad_(True)
    Hc = H.clone().requires_grad_(True)
    out = gc(Hd, r8["adj"].to(DEV))
    out_ref = ref(Hc, r8["adj"])
    assert (out.detach().cpu() - out_ref.detach()).abs().max() < 1e-4
    w = torch.randn_like(out_ref)
    (out * w.to(DEV)).sum().backward()
    (out_ref * w).sum().backward()
    np.testing.assert_allclose(gc.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(Hd.grad.cpu().numpy(), Hc.grad.numpy(), rtol=1e-4, atol=1e-4)
    # sparse input too (X of the reference, layer.py:102 with sparse infeatn)
    gc1 = GraphConvolution(r8["nfeat"], 8, bias=False).to(DEV)
    ref1 = gcn_ref.RefGraphConvolution(r8["nfeat"], 8, bias=False)
    ref1.load_state_dict({k: v.cpu() for k, v in gc1.state_dict().items()})
    o = gc1(r8["features"].to(DEV), r8["adj"].to(DEV))
    o_ref = ref1(r8["features"], r8["adj"])
    assert (o.detach().cpu() - o_ref.detach()).abs().max() < 1e-4
    o.sum().backward()
    o_ref.sum().backward()
    np.testing.assert_allclose(gc1.weight.grad.cpu().numpy(), ref1.weight.grad.numpy(), rtol=1e-4, atol=1e-5)


def test_gcn_gensim_shaped_r8_forward_backward(r8):
    """SURVEY §8(d) config 1's feature shape: R8 with the 100-d gensim-style X
    the README's 94.11 % run used (documents: the reference's LDA theta in
    columns 0-49; topics: N(0,1) 100-d rows, L2-normalised; default_rng(0);
    nnz 388,700) -- X is 50 % full, so it is multiplied as a dense copy on the
    MFMA GEMM (ops.DENSE_OPERAND_FILL).  Eval logits and one train-mode step's
    gradients against the oracle."""
    ndoc, ntopic = r8["ndoc"], r8["ntopic"]
    X = np.zeros((r8["nodes"], 100), np.float32)
    X[:ndoc, :ntopic] = r8["x_doc"] if "x_doc" in r8 else r8["features_dense"][:ndoc, :ntopic]
    X[ndoc:] = np.random.default_rng(0).standard_normal((ntopic, 100))
    X /= np.maximum(np.linalg.norm(X, axis=1, keepdims=True), 1e-12)
    Xs = datasets.dense_to_coo(X)
    assert Xs._nnz() == 388_700
    from graph_convolutional_networks_for_text_classification_amd.ops import Operand
    assert Operand(Xs.to(DEV)).dense is not None, "a 50 % full X goes to the dense GEMM"
    torch.manual_seed(50494)
    m = GCN(nfeat=100, nhid=200, nclass=r8["nclass"], dropout=0.5).to(DEV)
    ref = gcn_ref.RefGCN(nfeat=100, nhid=200, nclass=r8["nclass"], dropout=0.5)
    ref.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    m.eval()
    ref.eval()
    with torch.no_grad():
        lg = m(Xs.to(DEV), r8["adj"].to(DEV)).cpu().numpy()
        want = ref(Xs, r8["adj"]).numpy()
    assert np.abs(lg - want).max() <= LOGIT_TOL
    _labels_check(lg, want)
    m.train()
    ref.train()
    torch.manual_seed(7)
    out = m(Xs.to(DEV), r8["adj"].to(DEV))
    torch.manual_seed(7)
    out_ref = ref(Xs, r8["adj"])                    # same CPU dropout stream (dropout_rng="cpu")
    assert (out.detach().cpu() - out_ref.detach()).abs().max() <= LOGIT_TOL
    tgt = torch.from_numpy(np.concatenate([r8["target"], np.zeros(ntopic, np.int64)]))
    torch.nn.functional.cross_entropy(out, tgt.to(DEV)).backward()
    torch.nn.functional.cross_entropy(out_ref, tgt).backward()
    for (k, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        np.testing.assert_allclose(p.grad.cpu().numpy(), q.grad.numpy(), rtol=1e-4,
                                   atol=1e-4 * max(1.0, float(q.grad.abs().max())), err_msg=k)


@pytest.mark.parametrize("nhid", [50, 36, 300])
@pytest.mark.parametrize("gensim", [False, True])
def test_gcn_hidden_widths_outside_the_fused_kernels(r8, nhid, gensim):
    """GCN widths the fused / factored / narrow-feature kernels refuse (nhid % 4
    != 0 -- no 16-B rows -- or nhid > 256): the forward record falls back to the
    SpMM + GEMM launches (a record must never pick a kernel that then
    refuses), on R8's X and on the gensim-shaped 100-d X.  Eval logits and a
    train-mode step's gradients (reference CPU dropout stream) against the
    oracle's torch-CPU restatement of layer.py."""
    if gensim:
        X = _gensim_r8_x(r8)
        Xs = datasets.dense_to_coo(X)
        nfeat = 100
    else:
        Xs, nfeat = r8["features"], r8["nfeat"]
    torch.manual_seed(nhid)
    m = GCN(nfeat=nfeat, nhid=nhid, nclass=r8["nclass"], dropout=0.5).to(DEV)
    ref = gcn_ref.RefGCN(nfeat=nfeat, nhid=nhid, nclass=r8["nclass"], dropout=0.5)
    ref.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    m.eval()
    ref.eval()
    with torch.no_grad():
        lg = m(Xs.to(DEV), r8["adj"].to(DEV)).cpu().numpy()
        again = m(Xs.to(DEV), r8["adj"].to(DEV)).cpu().numpy()
        want = ref(Xs, r8["adj"]).numpy()
    assert np.abs(lg - want).max() <= LOGIT_TOL * max(1.0, float(np.abs(want).max()))
    assert np.array_equal(lg, again)
    m.train()
    ref.train()
    torch.manual_seed(11)
    out = m(Xs.to(DEV), r8["adj"].to(DEV))
    torch.manual_seed(11)
    out_ref = ref(Xs, r8["adj"])
    assert float((out.detach().cpu() - out_ref.detach()).abs().max()) <= \
        LOGIT_TOL * max(1.0, float(out_ref.detach().abs().max()))
    out.square().sum().backward()
    out_ref.square().sum().backward()
    for (k, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        _grads_close(p.grad.cpu().numpy(), q.grad.numpy(), k)


def test_gcn_dense_features_path(r8, golden_logits):
    """Dense infeatn (th.spmm falls through to mm) -> MFMA GEMM path."""
    torch.manual_seed(0)
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(DEV).eval()
    with torch.no_grad():
        lg = m(torch.from_numpy(r8["features_dense"]).to(DEV), r8["adj"].to(DEV)).cpu().numpy()
    assert np.abs(lg - golden_logits["eval_0"]).max() <= LOGIT_TOL


def test_gcn_train_forward_backward_match_reference(r8, golden_meta, golden_logits):
    """Train mode with the reference's CPU dropout RNG stream: identical masks,
    logits within 1e-4, gradients vs the oracle's autograd."""
    meta = golden_meta["logits"]["train_grad"]
    seed = meta["seed"]
    torch.manual_seed(seed)
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(DEV)
    m.train()
    lg = m(r8["features"].to(DEV), r8["adj"].to(DEV))
    assert np.abs(lg.detach().cpu().numpy() - golden_logits[f"train_{seed}"]).max() <= LOGIT_TOL
    tl = torch.tensor(r8["train_lst"][: meta["n_train_rows"]], dtype=torch.long)
    tgt = torch.tensor(r8["target"])
    loss = torch.nn.CrossEntropyLoss()(lg[tl.to(DEV)], tgt[tl].to(DEV))
    assert abs(float(loss) - meta["loss"]) < 1e-5
    loss.backward()
    np.testing.assert_allclose(m.gc2.weight.grad.cpu().numpy(), golden_logits["grad_gc2.weight"], rtol=1e-4,
                               atol=1e-6)
    np.testing.assert_allclose(m.gc2.bias.grad.cpu().numpy(), golden_logits["grad_gc2.bias"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(m.gc1.bias.grad.cpu().numpy(), golden_logits["grad_gc1.bias"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(m.gc1.weight.grad[:64].cpu().numpy(), golden_logits["grad_gc1.weight_rows0_64"],
                               rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(m.gc1.weight.grad[-64:].cpu().numpy(), golden_logits["grad_gc1.weight_rows_tail"],
                               rtol=1e-4, atol=1e-7)
    for k, st in meta["grads"].items():
        gsum = float(dict(m.named_parameters())[k].grad.double().sum())
        assert abs(gsum - st["sum"]) <= 1e-4 * max(1.0, st["abs_sum"]), k


def test_graph_convolution_single_layer_autograd(r8):
    """GraphConvolution alone (layer.py:84-112) incl. dense-input gradient."""
    torch.manual_seed(1)
    from graph_convolutional_networks_for_text_classification_amd import GraphConvolution
    gc = GraphConvolution(200, 8).to(DEV)
    ref = gcn_ref.RefGraphConvolution(200, 8)
    ref.load_state_dict({k: v.cpu() for k, v in gc.state_dict().items()})
    H = torch.randn(r8["nodes"], 200)
    Hd = H.clone().to(DEV).requires_grad_(True)
    Hc = H.clone().requires_grad_(True)
    out = gc(Hd, r8["adj"].to(DEV))
    out_ref = ref(Hc, r8["adj"])
    assert (out.detach().cpu() - out_ref.detach()).abs().max() < 1e-4
    w = torch.randn_like(out_ref)
    (out * w.to(DEV)).sum().backward()
    (out_ref * w).sum().backward()
    for p, q in ((gc.weight.grad, ref.weight.grad), (gc.bias.grad, ref.bias.grad), (Hd.grad, Hc.grad)):
        np.testing.assert_allclose(p.cpu().numpy(), q.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("seed", [50494, 99346])
def test_r8_training_accuracy_parity(r8, golden_meta, seed):
    """trainer.py:349-406 on the GPU path with the reference's dropout stream:
    test accuracy within ±0.1% of the reference run for the same seed."""
    run = golden_meta["train_runs"][str(seed)]
    hist, test, _ = gcn_ref.train_run(
        GCN, r8["features"], r8["adj"], r8["target"], run["train_idx"], run["val_idx"], r8["test_lst"],
        r8["nfeat"], r8["nclass"], seed, device=DEV)
    assert abs(test["acc"] - run["test"]["acc"]) <= 0.001 + 1e-12, (test["acc"], run["test"]["acc"], len(hist))
    # the loss trajectory follows the reference's closely for the first epochs
    for h, g in list(zip(hist, run["history"]))[:10]:
        assert abs(h["train_loss"] - g["train_loss"]) < 1e-3


# ------------------------------------------------------------------------------ BASELINE configs 3-5 at full size

@pytest.mark.parametrize("mode", ["eval", "train_hash"])
def test_gcn_20ng_shaped_forward_matches_oracle(mode, monkeypatch):
    """BASELINE config 3: 20ng-shaped doc-topic graph (18,846 docs, 70 topics,
    nclass 20, gensim-shaped nfeat 100 -> dense X).  The default forward takes
    the narrow-feature first layer (ops.dense_ax_for: the cached A-hat X, one
    gcnk_dense_gc1_f32 launch); eval logits of every path vs the oracle's
    reference-equivalent forward on the same tensors; logits and every gradient
    of a train-mode step (device dropout) of the dense-AX path and of the
    hub-factored path (70 hubs, Kc = 70, P = 20) vs the SpMM path."""
    from graph_convolutional_networks_for_text_classification_amd import factor, ops, record
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    g = datasets.doc_topic_graph(18846, 70, 20, seed=0)
    X, A = g["features"].to(DEV), g["adj"].to(DEV)
    f = factor.get(as_csr(A), ops.Operand(X))
    assert f is not None and f.H == 70 and f.Kc == 70
    outs, want = {}, None
    paths = {"dense_ax": (True, False, record.DENSE_AX), "factored": (False, True, record.FACTORED),
             "spmm": (False, False, record.SPMM_GEMM)}
    for name, (dax, fac, kind) in paths.items():
        monkeypatch.setattr(ops, "DENSE_AX", dax)
        monkeypatch.setattr(ops, "FACTOR_GC1", fac)
        torch.manual_seed(11)
        m = GCN(nfeat=g["nfeat"], nhid=200, nclass=20, dropout=0.5,
                dropout_rng="device" if mode == "train_hash" else "cpu").to(DEV)
        m.train(mode != "eval")
        if mode == "eval":
            with torch.no_grad():
                got = m(X, A)
            outs[name] = (got.cpu().numpy(), {})
            kinds = {r[2].kind for k, r in as_csr(A)._records.items()
                     if isinstance(r[2], record.ForwardRecord) and k[5] == ops.FACTOR_GC1 and k[7] == ops.DENSE_AX}
            assert kind in kinds, (name, kinds)
            if want is None:
                ref = gcn_ref.RefGCN(nfeat=g["nfeat"], nhid=200, nclass=20, dropout=0.5).eval()
                ref.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
                with torch.no_grad():
                    want = ref(g["features"], g["adj"]).numpy()
            assert np.abs(outs[name][0] - want).max() <= LOGIT_TOL, name
            _labels_check(outs[name][0], want)
        else:
            lg = m(X, A)
            lg.square().sum().backward()
            outs[name] = (lg.detach().cpu().numpy(), {k: p.grad.cpu().numpy() for k, p in m.named_parameters()})
    lb, gb = outs["spmm"]
    for name in ("dense_ax", "factored"):
        la, ga = outs[name]
        scale = max(1.0, float(np.abs(lb).max()))
        assert np.abs(la - lb).max() <= 1e-5 * scale, (name, float(np.abs(la - lb).max()))
        for k in ga:
            _grads_close(ga[k], gb[k], f"{name} {k}")


@pytest.fixture(scope="module")
def big_graph():
    """BASELINE config 4: uniform random 1M nodes / 20M edges (coalesced), int32 CSR."""
    rp, ci, v = datasets.uniform_random_csr(1_000_000, 20_000_000, seed=0, device=DEV)
    return from_arrays(rp, ci, v, (1_000_000, 1_000_000), DEV), (rp.cpu().numpy(), ci.cpu().numpy(), v.cpu().numpy())


def test_spmm_1m_20m_f256_sampled_rows_and_linearity(big_graph):
    """Full-size F = 256 product: 4,096 sampled rows against the float64 oracle
    (row slices of the CSR), and linearity A(B1 + B2) = A B1 + A B2 over every
    row (a size-independent property)."""
    a, (rp, ci, v) = big_graph
    M, F = a.shape[0], 256
    g = torch.Generator(device=DEV).manual_seed(5)
    B1 = torch.randn(M, F, device=DEV, generator=g)
    C1 = spmm(a, B1)
    rows = np.sort(np.random.default_rng(1).choice(M, 4096, replace=False))
    B1h = B1.cpu().numpy()
    sub = C1[torch.from_numpy(rows).to(DEV)].cpu().numpy()
    for i, r in enumerate(rows):
        b, e = rp[r], rp[r + 1]
        want = v[b:e].astype(np.float64) @ B1h[ci[b:e]].astype(np.float64)
        _close(sub[i], want, atol=2e-5 * np.sqrt(max(e - b, 1)))
    del B1h
    B2 = torch.randn(M, F, device=DEV, generator=g)
    lhs = spmm(a, B1 + B2)
    rhs = C1 + spmm(a, B2)
    assert torch.allclose(lhs, rhs, rtol=1e-5, atol=1e-4)
    assert torch.equal(spmm(a, B1), C1)   # bitwise reproducible at full size


def test_column_sharded_spmm_single_rank_on_gpu(big_graph):
    """BASELINE config 5's sharding module on one rank through the HIP kernels
    (no process group: the shard is the whole operand): F = 512 block of a
    4096-wide operand on the 1M/20M graph, equal to the unsharded product."""
    from graph_convolutional_networks_for_text_classification_amd.parallel import ColumnShardedSpMM
    a, _ = big_graph
    F = 512
    B = torch.randn(a.shape[0], F, device=DEV, generator=torch.Generator(device=DEV).manual_seed(2))
    op = ColumnShardedSpMM(a, F)
    full = op(op.shard(B))
    assert full.shape == (a.shape[0], F)
    assert torch.equal(full.block(0), spmm(a, B))


def test_rccl_process_group_collectives_on_gpu(r8):
    """The sharded path over a real RCCL (torch "nccl") process group of one
    rank on this GPU: ColumnShardedSpMM's all_gather_into_tensor and
    sharded_gcn_forward's all_reduce run through RCCL; results equal the
    unsharded HIP products bit for bit and the oracle within tolerance.  (N > 1
    is covered by the gloo world-2 tests; the driver's 8-GPU runs use RCCL.)"""
    import socket
    import torch.distributed as dist
    from graph_convolutional_networks_for_text_classification_amd.parallel import (
        ColumnShardedSpMM, sharded_gcn_forward)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device(DEV, 0))
    try:
        assert dist.get_backend() == "nccl"
        a = from_torch(r8["adj"].to(DEV))
        rp, ci, v = (t.cpu().numpy() for t in (a.rowptr, a.colind, a.val))
        F = 256
        B = torch.randn(r8["nodes"], F, device=DEV, generator=torch.Generator(device=DEV).manual_seed(9))
        bias = torch.randn(F, device=DEV, generator=torch.Generator(device=DEV).manual_seed(10))
        op = ColumnShardedSpMM(a, F)
        gathered = op(op.shard(B), bias=bias, epilogue=_lib.EPI_BIAS_RELU)      # RCCL all-gather
        want = spmm(a, B, bias=bias, epilogue=_lib.EPI_BIAS_RELU)
        assert torch.equal(gathered.to_dense(), want)
        _close(gathered.block(0), csr_ref.spmm_epilogue(csr_ref.spmm_csr(rp, ci, v, B.cpu().numpy()),
                                                        bias.cpu().numpy(), relu=True))
        # a consumer product reading the gathered blocks in place
        assert torch.equal(gathered.spmm(a), spmm(a, want))
        torch.manual_seed(0)
        m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(DEV).eval()
        with torch.no_grad():
            got = sharded_gcn_forward(m, r8["features"].to(DEV), r8["adj"].to(DEV))   # RCCL all-reduce
            ref = m(r8["features"].to(DEV), r8["adj"].to(DEV))
        assert (got - ref).abs().max().item() <= 1e-5
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


# ------------------------------------------------------------------------------ device adjacency preparation

def test_preprocess_adj_on_device_bit_exact_r8(r8):
    """gcnk_sym_normalize on R8's raw symmetric A (the adjacency trainer.py:148
    hands to utils.preprocess_adj) reproduces the reference's normalised
    values bit for bit, in CSR order."""
    from graph_convolutional_networks_for_text_classification_amd import preprocess_adj
    n = r8["nodes"]
    A = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([r8["a_rows"], r8["a_cols"]]).astype(np.int64)),
                                torch.from_numpy(np.asarray(r8["a_vals"], np.float32)), (n, n)).to(DEV)
    ah = preprocess_adj(A)
    ref = r8["adj"].coalesce()
    assert np.array_equal(ah.rowptr.cpu().numpy(), np.concatenate([[0], np.cumsum(np.bincount(
        ref.indices()[0].numpy(), minlength=n))]))
    assert np.array_equal(ah.colind.cpu().numpy(), ref.indices()[1].numpy())
    assert np.array_equal(ah.val.cpu().numpy().view(np.uint32), ref.values().numpy().view(np.uint32))
    # and it drives the forward directly
    torch.manual_seed(0)
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(DEV).eval()
    with torch.no_grad():
        a = m(r8["features"].to(DEV), ah)
        b = m(r8["features"].to(DEV), r8["adj"].to(DEV))
    assert torch.equal(a, b)


def test_preprocess_adj_known_answers(golden_meta):
    """The reference's own preprocess_adj outputs on tiny graphs with isolated
    nodes and explicit diagonal entries (tests/golden known-answer cases)."""
    from graph_convolutional_networks_for_text_classification_amd import preprocess_adj
    for case in golden_meta["tiny_cases"]:
        n = case["n"]
        A = torch.sparse_coo_tensor(torch.tensor([case["A_rows"], case["A_cols"]], dtype=torch.int64),
                                    torch.tensor(case["A_vals"], dtype=torch.float32), (n, n)).to(DEV)
        ah = preprocess_adj(A)
        rows = np.repeat(np.arange(n), np.diff(ah.rowptr.cpu().numpy()))
        got = {(int(r), int(c)): v for r, c, v in zip(rows, ah.colind.cpu().numpy(), ah.val.cpu().numpy())}
        want = {(int(r), int(c)): np.float32(v) for r, c, v in zip(case["adj_rows"], case["adj_cols"],
                                                                   case["adj_vals"])}
        assert got.keys() == want.keys(), case["name"]
        assert all(got[k].view(np.uint32) == want[k].view(np.uint32) for k in want), case["name"]
    # an explicit self loop gets + 1 (A + I) and stays one entry
    A = torch.sparse_coo_tensor(torch.tensor([[0, 0, 1], [0, 1, 0]]), torch.tensor([2.0, 1.0, 1.0]), (3, 3)).to(DEV)
    ah = preprocess_adj(A)
    assert ah.nnz == 5 and ah.rowptr.cpu().tolist() == [0, 2, 4, 5]
    assert ah.colind.cpu().tolist() == [0, 1, 0, 1, 2]
    d = np.array([4.0, 2.0, 1.0]) ** -0.5
    want = np.float32([(d[0] * 3.0) * d[0], (d[0] * 1.0) * d[1], (d[1] * 1.0) * d[0], (d[1] * 1.0) * d[1], 1.0])
    assert np.array_equal(ah.val.cpu().numpy(), want)


def test_preprocess_adj_rejects_unsorted_or_asymmetric_input():
    """gcnk_sym_normalize assumes sorted, duplicate-free rows and a symmetric A
    (the reference's (A D)^T D); preprocess_adj checks both and raises."""
    from graph_convolutional_networks_for_text_classification_amd import preprocess_adj
    from graph_convolutional_networks_for_text_classification_amd.sparse import CSR
    i32 = dict(dtype=torch.int32, device=DEV)
    # unsorted row 0 (columns 2, 1) of a symmetric pattern
    a = CSR(torch.tensor([0, 2, 3, 4], **i32), torch.tensor([2, 1, 0, 0], **i32),
            torch.ones(4, device=DEV), (3, 3))
    with pytest.raises(RuntimeError, match="sorted"):
        preprocess_adj(a)
    # a directed edge 0 -> 1 only
    A = torch.sparse_coo_tensor(torch.tensor([[0], [1]]), torch.tensor([1.0]), (2, 2)).to(DEV)
    with pytest.raises(RuntimeError, match="not symmetric"):
        preprocess_adj(A)


# ------------------------------------------------------------------------------ evaluation metrics

@pytest.mark.parametrize("nclass", [8, 20])
def test_metrics_match_reference_restatement(nclass):
    """metrics.evaluate / accuracy / macro_f1 (one launch, one copy) equal the
    reference's utils.py:25-109 arithmetic (oracle restatement) on logits with
    exact ties and NaNs, with and without a row subset, with num_classes given
    and inferred from the targets."""
    from graph_convolutional_networks_for_text_classification_amd import metrics
    g = torch.Generator().manual_seed(nclass)
    rows = 5000
    logits = torch.randn(rows, nclass, generator=g)
    logits[::97, 3] = logits[::97, 1]                  # ties: first maximum wins
    logits[::97, 1] = logits[::97].max(1).values + 1
    logits[::97, 3] = logits[::97, 1]
    logits[5::503, 2] = float("nan")                   # NaN is maximal (th.max)
    targ = torch.randint(0, nclass - 1, (rows,), generator=g)   # the last class never a target
    idx = torch.randperm(rows, generator=g)[:1700]
    for sub in (None, idx):
        p_c = logits if sub is None else logits[sub]
        t_c = targ if sub is None else targ[sub]
        want_acc = gcn_ref.accuracy(p_c, t_c)
        want = gcn_ref.macro_f1(p_c, t_c, nclass)
        acc, f1, p, r = metrics.evaluate(logits.to(DEV), targ.to(DEV), None if sub is None else sub.to(DEV),
                                         num_classes=nclass)
        assert acc == want_acc
        assert (f1, p, r) == pytest.approx(want, rel=0, abs=0)
    # num_classes=None: only the classes present in the targets (utils.py:53-54)
    pred = logits.argmax(1)
    present = sorted(set(targ.tolist()))
    tp = np.array([((pred == i) & (targ == i)).sum().item() for i in present])
    fp = np.array([((pred == i) & (targ != i)).sum().item() for i in present])
    fn = np.array([((pred != i) & (targ == i)).sum().item() for i in present])
    with np.errstate(divide="ignore", invalid="ignore"):
        pr = tp / (tp + fp)
        pr[np.isnan(pr)] = 0
        rc = tp / (tp + fn)
        rc[np.isnan(rc)] = 0
    pm, rm = np.mean(pr), np.mean(rc)
    f1, p, r = metrics.macro_f1(logits.to(DEV), targ.to(DEV))
    assert (f1, p, r) == (2 * pm * rm / (pm + rm), pm, rm)
    assert metrics.accuracy(logits.to(DEV), targ.to(DEV)) == gcn_ref.accuracy(logits, targ)


@pytest.mark.gpu
def test_spmm_two_part_launch_matches_single(monkeypatch, r8):
    """gcnk_spmm_csr_f32_part: the single-chunk tile blocks on a side stream and
    the rest on the caller's stream give the one-launch result bit for bit."""
    from graph_convolutional_networks_for_text_classification_amd import ops
    rng = np.random.default_rng(7)
    for a, K in ((from_torch(r8["features"].to(DEV)), r8["nfeat"]), (None, 900)):
        if a is None:
            rp, ci, v = _mixed_density_csr(rng, 700, K)
            a = from_arrays(rp, ci, v, (700, K), DEV)
        B = torch.from_numpy(rng.standard_normal((K, 200)).astype(np.float32)).to(DEV)
        one = ops.spmm(a, B)
        hdr = list(a._plans.values())[-1].header
        assert hdr[15] > 0 and hdr[8] > hdr[15], "both single- and multi-chunk tile blocks expected"
        monkeypatch.setattr(ops, "OVERLAP_TILE_PARTS", True)
        two = ops.spmm(a, B)
        torch.cuda.synchronize()
        monkeypatch.setattr(ops, "OVERLAP_TILE_PARTS", False)
        assert torch.equal(one, two)


def test_device_dropout_draws_a_fresh_mask_on_every_graph_replay(r8):
    """dropout_rng="device": the hash offset is read from and advanced on the
    device (GCN._rng_base), so a train-mode forward captured in a hipGraph
    draws a new mask per replay, and each replay equals the eager forward at
    the same stream position bit for bit."""
    torch.manual_seed(3)
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5, dropout_rng="device").to(DEV).train()
    x, adj = r8["features"].to(DEV), r8["adj"].to(DEV)
    step = r8["nodes"] * 200
    with torch.no_grad():
        m(x, adj)                                   # plans built outside the capture
        torch.cuda.synchronize()
        base0 = int(m._rng_base.item())
        assert base0 == step
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y = m(x, adj)
        outs = []
        for _ in range(3):
            g.replay()
            outs.append(y.clone())
        torch.cuda.synchronize()
        assert int(m._rng_base.item()) == base0 + 3 * step, "one advance per replay (none at capture)"
        assert not torch.equal(outs[0], outs[1]) and not torch.equal(outs[1], outs[2])
        m._rng_base.fill_(base0 + step)
        eager = m(x, adj)
        assert torch.equal(eager, outs[1])


@pytest.mark.parametrize("kind", ["random", "r8"])
def test_graph_capture_takes_a_prezeroed_counter_region(r8, kind):
    """Captured SpMMs whose plan needs a counter region (heavy-row arrival
    counters) share ONE of the plan's pre-zeroed spare regions per capturing
    stream -- however many calls and graphs -- so no graph holds a memset
    node; eager calls keep their stream's region; replays interleaved with
    eager calls stay exact."""
    rng = np.random.default_rng(23)
    if kind == "random":
        M, K, F = 3001, 20003, 200
        rp, ci, v = _random_csr(M, K, 20000, rng, heavy_rows=(5, 1700), heavy_deg=2500)
        a = from_arrays(rp, ci, v, (M, K), DEV)
    else:
        a, K, F = from_torch(r8["adj"].to(DEV)), r8["nodes"], 200
    B = torch.from_numpy(rng.standard_normal((K, F)).astype(np.float32)).to(DEV)
    ref = spmm(a, B, dense=2.0)
    plan = list(a._plans.values())[-1]
    assert plan.counter_bytes() > 0
    spares = len(plan._spares)
    outs = [torch.empty_like(ref) for _ in range(6)]
    graphs = [torch.cuda.CUDAGraph() for _ in range(2)]
    for gi, g in enumerate(graphs):
        with torch.cuda.graph(g):
            for o in outs[3 * gi:3 * gi + 3]:
                spmm(a, B, out=o, dense=2.0)
    assert len(plan._spares) == spares - 1, "one region for the capturing stream, not one per call"
    for _ in range(4):
        for o in outs:
            o.zero_()
        graphs[0].replay()
        eager = spmm(a, B, dense=2.0)
        graphs[1].replay()
        torch.cuda.synchronize()
        assert torch.equal(eager, ref)
        for o in outs:
            assert torch.equal(o, ref)


@pytest.mark.parametrize("dense", [0.25, 0.3])
def test_tile_path_repeat_streams_and_graph_replay_are_exact(r8, dense, monkeypatch):
    """R8 X W1 on the tile path (single-chunk document blocks, the multi-chunk
    topic block and its slab reduce): back-to-back calls, two streams at once
    on one cached plan and graph replays all give the one-call bits, and the
    product matches the oracle."""
    from graph_convolutional_networks_for_text_classification_amd import ops
    x = from_torch(r8["features"].to(DEV))
    W = torch.randn(r8["nfeat"], 200, generator=torch.Generator().manual_seed(11)).to(DEV)
    one = ops.spmm(x, W, dense=dense)
    plan = list(x._plans.values())[-1]
    assert plan.header[9] > 0, "R8 X's topic rows form a multi-chunk tile block"
    ops_spmm = ops.spmm
    def spmm_d(*a, **k):
        return ops_spmm(*a, dense=dense, **k)
    monkeypatch.setattr(ops, "spmm", spmm_d)
    for _ in range(4):
        assert torch.equal(ops.spmm(x, W), one)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    W2 = W * 0.5
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        o1 = [ops.spmm(x, W) for _ in range(3)]
    with torch.cuda.stream(s2):
        o2 = [ops.spmm(x, W2) for _ in range(3)]
    torch.cuda.synchronize()
    half = ops.spmm(x, W2)
    assert all(torch.equal(o, one) for o in o1) and all(torch.equal(o, half) for o in o2)
    out = torch.empty_like(one)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.spmm(x, W, out=out)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, one)
    rp, ci, v = (t.cpu().numpy() for t in (x.rowptr, x.colind, x.val))
    _close(one, csr_ref.spmm_csr(rp, ci, v, W.cpu().numpy()), atol=1e-4)


# ------------------------------------------------------------------------------ hub-factored gc1

@pytest.mark.parametrize("mode", ["eval", "train_mask", "train_hash"])
def test_factored_gc1_matches_spmm_path(r8, mode):
    """GCN.forward through the hub factorisation (factor.py + gcnk_hubfactor_gc1_f32:
    A-hat X W1 as U W1[Kc] + A_H (X_hubs W1)) against the SpMM path
    (ops.FACTOR_GC1 = False: X W1 then A-hat S1, layer.py:102,106) on R8 with
    the same weights and the same dropout masks: logits and every gradient
    within fp32 reassociation error; H1 kept for the backward only when
    needed; the factored launch bitwise reproducible."""
    from graph_convolutional_networks_for_text_classification_amd import factor, ops
    X, A = r8["features"].to(DEV), r8["adj"].to(DEV)
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    f = factor.get(as_csr(A), ops.Operand(X))
    assert f is not None and f.H == 50 and f.Kc == 50
    outs = {}
    for fac in (True, False):
        saved = ops.FACTOR_GC1
        ops.FACTOR_GC1 = fac
        try:
            torch.manual_seed(123)
            m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5,
                    dropout_rng="device" if mode == "train_hash" else "cpu").to(DEV)
            m.train(mode != "eval")
            torch.manual_seed(9)
            lg = m(X, A)
            if mode == "eval":
                again = m(X, A)
                assert torch.equal(lg, again)
            lg.square().sum().backward()
            outs[fac] = (lg.detach().cpu().numpy(), {k: p.grad.cpu().numpy() for k, p in m.named_parameters()})
        finally:
            ops.FACTOR_GC1 = saved
    (la, ga), (lb, gb) = outs[True], outs[False]
    scale = max(1.0, float(np.abs(lb).max()))
    assert np.abs(la - lb).max() <= 1e-5 * scale, float(np.abs(la - lb).max())
    for k in ga:
        _grads_close(ga[k], gb[k], k)


def test_xhub_product_per_mode(r8):
    """S_T = X[hubs] W1 of the factored forward takes R8's dense hub rows
    through the K-split GEMM in eval and their CSR through the tile plan in
    training (factor.hub_operand; profiles/r06_xhub_train_ab.log): both within
    fp32 reassociation error of float64, and the forward records follow the
    same choice."""
    from graph_convolutional_networks_for_text_classification_amd import factor, ops, record
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    X, A = r8["features"].to(DEV), r8["adj"].to(DEV)
    adj, xop = as_csr(A), ops.Operand(X)
    f = factor.get(adj, xop)
    assert f is not None and f.x_hub is not None and f.x_hub_dense is not None
    assert f.hub_operand(False) == "dense"
    assert f.hub_operand(True) == ("csr" if factor.XHUB_TRAIN_TILE else "dense")
    W1 = torch.randn(r8["nfeat"], 200, generator=torch.Generator().manual_seed(5)).to(DEV) * 0.05
    want = f.x_hub_dense.double().cpu().numpy() @ W1.double().cpu().numpy()
    for train in (False, True):
        got = f.hub_times(W1, train=train).cpu().double().numpy()
        assert np.abs(got - want).max() <= 1e-5 * max(1.0, np.abs(want).max()), train
    rec_e, _ = record.get(adj, xop, 200, r8["nclass"], DEV)
    rec_t, _ = record.get(adj, xop, 200, r8["nclass"], DEV, train=True)
    assert rec_e.kind == rec_t.kind == record.FACTORED
    assert rec_e.s.x_dense and not rec_e.s.x.plan
    assert bool(rec_t.s.x.plan) == (f.hub_operand(True) == "csr")


@pytest.mark.parametrize("F,P,ndoc", [(52, 3, 2000), (200, 20, 2000), (36, 32, 2000), (200, 20, 12000)])
def test_factored_gc1_kernel_against_float64(F, P, ndoc):
    """gcnk_hubfactor_gc1_f32 alone on a synthetic doc-topic graph with hub x
    hub nonzeros, F not a multiple of 16 (and F < 64, where the n-tiles past F
    read the zero pad after W1[Kc]), P of one and two MFMA n-tiles, H1 stored:
    H1 and S2 = H1 W2 against float64 (every epilogue code but the dropout
    ones), rows written through the block order's row ids (hub rows spread over
    the blocks, factor.py).  Every launch follows one that filled all LDS with
    NaN bits (gcnk_debug_poison_lds): a read of LDS the kernel did not write
    would surface as NaN."""
    import ctypes
    import scipy.sparse as ssp
    from graph_convolutional_networks_for_text_classification_amd import factor, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    g = datasets.doc_topic_graph(ndoc, 40, 5, seed=4, tt_prob=0.3)
    A, X = g["adj"].to(DEV), g["features"].to(DEV)
    xop = ops.Operand(X)
    f = factor.get(as_csr(A), xop)
    assert f is not None
    # 12,000 documents: more 32-row blocks (377) than CUs (several rounds of workgroups)
    assert not np.array_equal(f.perm.numpy(), np.arange(f.M))   # the hub rows moved
    rng = np.random.default_rng(3)
    W1 = torch.from_numpy(rng.standard_normal((g["nfeat"], F)).astype(np.float32)).to(DEV)
    W2 = torch.from_numpy(rng.standard_normal((F, P)).astype(np.float32)).to(DEV)
    b1 = torch.from_numpy(rng.standard_normal(F).astype(np.float32)).to(DEV)
    a = g["adj"].coalesce()
    Ad = ssp.csr_matrix((a.values().double().numpy(), a.indices().numpy()), shape=tuple(a.shape))
    x = g["features"].coalesce()
    Xd = ssp.csr_matrix((x.values().double().numpy(), x.indices().numpy()), shape=tuple(x.shape))
    Z = Ad @ (Xd @ W1.cpu().double().numpy())
    lib = _lib.load()

    S_T = f.hub_times(W1).contiguous()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def launch(epi, store_h1=True):
        """gcnk_hubfactor_gc1_f32 right after an LDS poison launch (as ops.hubfactor_gc1 calls it)."""
        H1 = torch.empty((f.M, F), device=DEV) if store_h1 else None
        S2 = torch.empty((f.M, P), device=DEV)
        _lib.check(lib.gcnk_debug_poison_lds(0xFFFFFFFF, stream), "gcnk_debug_poison_lds")
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        _lib.check(lib.gcnk_hubfactor_gc1_f32(
            f.M, F, f.Kc, f.H, P, p(f.U), f.U.stride(0), p(W1), F, f.k0, p(S_T), F, p(f.rec),
            f.rec_words, p(b1), epi, None, 0, 1.0, 1.0, 0, 0, None, p(W2), P, p(H1), F, p(S2), P, stream),
            "gcnk_hubfactor_gc1_f32")
        return H1, S2
    for epi in (_lib.EPI_NONE, _lib.EPI_BIAS, _lib.EPI_BIAS_RELU):
        H1, S2 = launch(epi)
        assert bool(torch.isfinite(H1).all()) and bool(torch.isfinite(S2).all())
        want = Z if epi == _lib.EPI_NONE else Z + b1.cpu().double().numpy()
        if epi == _lib.EPI_BIAS_RELU:
            want = np.maximum(want, 0.0)
        _close(H1, want, atol=2e-5 * max(1.0, np.abs(want).max()))
        _close(S2, H1.cpu().double().numpy() @ W2.cpu().double().numpy(), atol=2e-5 * max(1.0, np.abs(want).max()))
    H1b, S2b = launch(_lib.EPI_BIAS_RELU, store_h1=False)
    assert H1b is None and torch.equal(S2b, S2)
    H1c, S2c = ops.hubfactor_gc1(f, W1, b1, W2, epilogue=_lib.EPI_BIAS_RELU)   # (the op wrapper: same bits)
    assert torch.equal(H1c, H1) and torch.equal(S2c, S2)


@pytest.mark.parametrize("mode", ["eval", "train_hash"])
def test_factored_forward_hub_rows_first_ragged(mode):
    """The factored forward on a synthetic doc-topic graph renumbered so the
    topic (hub) rows come FIRST, with M = 1,038 (not a multiple of the 32-row
    block) and the gensim-shaped dense X (its hub rows through the dense GEMM):
    logits and gradients against the SpMM path (ops.FACTOR_GC1 = False)."""
    from graph_convolutional_networks_for_text_classification_amd import factor, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    g = datasets.doc_topic_graph(1001, 37, 5, seed=11)
    n, ndoc = g["nodes"], 1001
    order = np.concatenate([np.arange(ndoc, n), np.arange(ndoc)])     # new position -> old node
    inv = np.empty(n, np.int64)
    inv[order] = np.arange(n)
    a = g["adj"].coalesce()
    idx = torch.from_numpy(inv)[a.indices()]
    A = torch.sparse_coo_tensor(idx, a.values(), (n, n)).coalesce().to(DEV)
    X = datasets.dense_to_coo(g["features_dense"][order]).to(DEV)
    xop = ops.Operand(X)
    f = factor.get(as_csr(A), xop)
    assert f is not None and f.hubs.cpu().tolist() == list(range(37)) and f.M % 32 != 0
    outs = {}
    for fac in (True, False):
        saved, saved_ax = ops.FACTOR_GC1, ops.DENSE_AX
        ops.FACTOR_GC1, ops.DENSE_AX = fac, False    # (the dense X would otherwise take the dense-AX gc1)
        try:
            torch.manual_seed(5)
            m = GCN(nfeat=g["nfeat"], nhid=200, nclass=g["nclass"], dropout=0.5,
                    dropout_rng="device").to(DEV)
            m.train(mode != "eval")
            lg = m(X, A)
            lg.square().sum().backward()
            outs[fac] = (lg.detach().cpu().numpy(), {k: p.grad.cpu().numpy() for k, p in m.named_parameters()})
        finally:
            ops.FACTOR_GC1, ops.DENSE_AX = saved, saved_ax
    (la, ga), (lb, gb) = outs[True], outs[False]
    scale = max(1.0, float(np.abs(lb).max()))
    assert np.abs(la - lb).max() <= 1e-5 * scale, float(np.abs(la - lb).max())
    for k in ga:
        _grads_close(ga[k], gb[k], k)


# ------------------------------------------------------------------------------ narrow-feature gc1 (A-hat X cached)

def _gensim_r8_x(r8):
    """The gensim-shaped 100-d R8 X: documents' LDA
    theta in columns 0-49, topics N(0,1) 100-d, rows L2-normalised."""
    ndoc, ntopic = r8["ndoc"], r8["ntopic"]
    X = np.zeros((r8["nodes"], 100), np.float32)
    X[:ndoc, :ntopic] = r8["features_dense"][:ndoc, :ntopic]
    X[ndoc:] = np.random.default_rng(0).standard_normal((ntopic, 100))
    X /= np.maximum(np.linalg.norm(X, axis=1, keepdims=True), 1e-12)
    return X


@pytest.mark.parametrize("K,F,P,M", [(100, 200, 20, 18916), (100, 200, 8, 7724), (7, 8, 3, 1000),
                                     (50, 52, 32, 777), (128, 256, 17, 2049), (64, 100, 16, 33), (13, 200, 1, 16),
                                     (30, 180, 18, 500), (100, 208, 20, 1000), (97, 196, 19, 300), (100, 240, 20, 600)])
def test_dense_gc1_kernel_against_float64(K, F, P, M):
    """gcnk_dense_gc1_f32 alone: H1 = relu(AX W1 + b1) and S2 = H1 W2 against
    float64 for K of 1-32 k-steps (K not a multiple of 4 included), F not a
    multiple of 16, both column layouts (three n-tiles a wave with the rotating
    tail n-tile for F in 193..208 -- 196, 200, 208 -- and without it; four past
    208), P of one and two MFMA n-tiles and of one tile + 1-4 VALU columns
    (17-20), M ragged (a partial last
    16-row tile) and below / above the CU count in tiles; H1 stored or not
    (S2 bitwise the same); the dropout-mask epilogue against the same mask in
    float64; the launch bitwise reproducible."""
    import ctypes
    rng = np.random.default_rng(K * 1000 + F + P)
    AX = rng.standard_normal((M, (K + 3) // 4 * 4)).astype(np.float32)
    AX[:, K:] = 0.0
    W1 = rng.standard_normal((K, F)).astype(np.float32)
    W2 = rng.standard_normal((F, P)).astype(np.float32)
    b1 = rng.standard_normal(F).astype(np.float32)
    mask = (rng.random((M, F)) < 0.5).astype(np.uint8)
    t = {k: torch.from_numpy(v).to(DEV) for k, v in dict(AX=AX, W1=W1, W2=W2, b1=b1, mask=mask).items()}
    lib = _lib.load()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda x: ctypes.c_void_p(x.data_ptr()) if x is not None else None

    def launch(epi, store_h1=True, m=None, scale=1.0):
        H1 = torch.full((M, F), float("nan"), device=DEV) if store_h1 else None
        S2 = torch.full((M, P), float("nan"), device=DEV)
        _lib.check(lib.gcnk_dense_gc1_f32(M, K, F, P, p(t["AX"]), t["AX"].stride(0), p(t["W1"]), F, p(t["b1"]), epi,
                                          p(m), F if m is not None else 0, scale, 0.5, 0, 0, None, p(t["W2"]), P,
                                          p(H1), F, p(S2), P, stream), "gcnk_dense_gc1_f32")
        return H1, S2
    Z = AX[:, :K].astype(np.float64) @ W1.astype(np.float64) + b1
    want = np.maximum(Z, 0.0)
    H1, S2 = launch(_lib.EPI_BIAS_RELU)
    tol = 2e-5 * max(1.0, np.abs(want).max())
    _close(H1, want, atol=tol)
    _close(S2, H1.cpu().double().numpy() @ W2.astype(np.float64), atol=tol * max(1.0, np.abs(W2).sum(0).max()))
    H1b, S2b = launch(_lib.EPI_BIAS_RELU, store_h1=False)
    assert H1b is None and torch.equal(S2b, S2)
    H1c, S2c = launch(_lib.EPI_BIAS_RELU)
    assert torch.equal(H1c, H1) and torch.equal(S2c, S2)
    Hd, Sd = launch(_lib.EPI_BIAS_RELU_DROP, m=t["mask"], scale=2.0)
    _close(Hd, want * mask * 2.0, atol=2 * tol)
    _close(Sd, Hd.cpu().double().numpy() @ W2.astype(np.float64), atol=2 * tol * max(1.0, np.abs(W2).sum(0).max()))
    with pytest.raises(RuntimeError):   # an epilogue without the ReLU is not gc1's
        launch(_lib.EPI_BIAS)


@pytest.mark.parametrize("mode", ["eval", "train_mask", "train_hash"])
@pytest.mark.parametrize("graph", ["r8_gensim", "ragged"])
def test_dense_ax_forward_backward_matches_spmm_path(r8, mode, graph, monkeypatch):
    """GCN.forward / backward through the narrow-feature gc1 (the cached
    A-hat X, gcnk_dense_gc1_f32; backward gW1 = (A-hat X)^T gZ1) against the
    SpMM path (X W1, then A-hat S1, layer.py:102,106) with the same weights and
    dropout masks: logits within fp32 reassociation error, every gradient to
    1e-4; the eval logits also against the oracle (reference ATen calls) to
    1e-4.  On R8 with the gensim-shaped X and on a ragged synthetic doc-topic
    graph (M = 1,038) whose X is dense."""
    from graph_convolutional_networks_for_text_classification_amd import ops, record
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    if graph == "r8_gensim":
        Xn, A_cpu, nclass = _gensim_r8_x(r8), r8["adj"], r8["nclass"]
    else:
        g = datasets.doc_topic_graph(1001, 37, 5, seed=11)
        Xn, A_cpu, nclass = g["features_dense"], g["adj"], g["nclass"]
    Xs = datasets.dense_to_coo(Xn)
    X, A = Xs.to(DEV), A_cpu.to(DEV)
    assert ops.dense_ax_for(as_csr(A), ops.Operand(X), 200, nclass) is not None
    outs = {}
    for dax in (True, False):
        monkeypatch.setattr(ops, "DENSE_AX", dax)
        monkeypatch.setattr(ops, "FACTOR_GC1", False)
        torch.manual_seed(123)
        m = GCN(nfeat=Xn.shape[1], nhid=200, nclass=nclass, dropout=0.5,
                dropout_rng="device" if mode == "train_hash" else "cpu").to(DEV)
        m.train(mode != "eval")
        torch.manual_seed(9)
        lg = m(X, A)
        if dax:
            kinds = {r[2].kind for r in as_csr(A)._records.values() if isinstance(r[2], record.ForwardRecord)}
            assert record.DENSE_AX in kinds, kinds
        if mode == "eval":
            assert torch.equal(lg, m(X, A))
            ref = gcn_ref.RefGCN(nfeat=Xn.shape[1], nhid=200, nclass=nclass, dropout=0.5).eval()
            ref.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
            with torch.no_grad():
                want = ref(Xs, A_cpu).numpy()
            assert np.abs(lg.detach().cpu().numpy() - want).max() <= LOGIT_TOL
        lg.square().sum().backward()
        outs[dax] = (lg.detach().cpu().numpy(), {k: p.grad.cpu().numpy() for k, p in m.named_parameters()})
    (la, ga), (lb, gb) = outs[True], outs[False]
    scale = max(1.0, float(np.abs(lb).max()))
    assert np.abs(la - lb).max() <= 1e-5 * scale, float(np.abs(la - lb).max())
    for k in ga:
        _grads_close(ga[k], gb[k], k)


def test_dense_ax_misaligned_weight_falls_back_to_the_spmm_path(r8):
    """gcnk_dense_gc1_f32 refuses W1 rows that are not 16-B aligned (GCNK_EUNSUP);
    the module then takes the SpMM path (the record is skipped, ops.dense_gc1
    returns None) instead of raising: a gc1 weight living 4 bytes
    into its storage still gives the oracle's logits."""
    Xn = _gensim_r8_x(r8)
    Xs = datasets.dense_to_coo(Xn)
    X, A = Xs.to(DEV), r8["adj"].to(DEV)
    torch.manual_seed(123)
    m = GCN(nfeat=Xn.shape[1], nhid=200, nclass=r8["nclass"], dropout=0.5).to(DEV).eval()
    w = m.gc1.weight.detach()
    buf = torch.empty(w.numel() + 1, device=DEV)
    shifted = buf[1:].view_as(w)
    shifted.copy_(w)
    assert shifted.data_ptr() % 16 != 0
    m.gc1.weight.data = shifted
    with torch.no_grad():
        lg = m(X, A)
    ref = gcn_ref.RefGCN(nfeat=Xn.shape[1], nhid=200, nclass=r8["nclass"], dropout=0.5).eval()
    ref.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    with torch.no_grad():
        want = ref(Xs, r8["adj"]).numpy()
    assert np.abs(lg.cpu().numpy() - want).max() <= LOGIT_TOL


# ------------------------------------------------------------------------------ whole-forward launch record

@pytest.mark.parametrize("path", ["factored", "spmm_proj", "spmm_gemm", "dense_factored", "dense_spmm", "dense_ax"])
@pytest.mark.parametrize("mode", ["eval", "train_mask", "train_hash"])
def test_forward_record_is_bitwise_the_per_op_path(r8, path, mode, monkeypatch):
    """gcnk_gcn_forward_f32 / gcnk_gcn_backward_f32 (record.py: the whole
    forward, the whole backward from one C call each) issue the per-op path's
    launches with the same arguments: logits and every gradient bitwise equal
    to ops.USE_RECORD = False, for each record kind
    (factored / fused projection / SpMM + GEMM, sparse and dense X), in eval
    (inference fast path, no autograd node) and in both dropout modes."""
    from graph_convolutional_networks_for_text_classification_amd import ops, record
    monkeypatch.setattr(ops, "FACTOR_GC1", path in ("factored", "dense_factored"))
    monkeypatch.setattr(ops, "FUSE_PROJECTION", path != "spmm_gemm")
    monkeypatch.setattr(ops, "DENSE_AX", path == "dense_ax")
    A = r8["adj"].to(DEV)
    if path.startswith("dense"):       # the gensim-shaped 100-d X (dense copy, MFMA GEMM)
        ndoc, ntopic = r8["ndoc"], r8["ntopic"]
        Xd = np.zeros((r8["nodes"], 100), np.float32)
        Xd[:ndoc, :ntopic] = r8["features_dense"][:ndoc, :ntopic]
        Xd[ndoc:] = np.random.default_rng(0).standard_normal((ntopic, 100))
        X, nfeat = datasets.dense_to_coo(Xd).to(DEV), 100
    else:
        X, nfeat = r8["features"].to(DEV), r8["nfeat"]
    outs = {}
    for use in (True, False):
        monkeypatch.setattr(ops, "USE_RECORD", use)
        torch.manual_seed(77)
        m = GCN(nfeat=nfeat, nhid=200, nclass=r8["nclass"], dropout=0.5,
                dropout_rng="device" if mode == "train_hash" else "cpu").to(DEV)
        m.train(mode != "eval")
        torch.manual_seed(3)
        if mode == "eval":
            with torch.no_grad():
                lg = m(X, A)
                assert torch.equal(lg, m(X, A))        # memoised operands, same record
            outs[use] = (lg.cpu(), {})
        else:
            lg = m(X, A)
            lg.square().sum().backward()
            outs[use] = (lg.detach().cpu(), {k: p.grad.cpu() for k, p in m.named_parameters()})
    assert torch.equal(outs[True][0], outs[False][0])
    for k in outs[True][1]:
        assert torch.equal(outs[True][1][k], outs[False][1][k]), k
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    recs = [r[2] for r in getattr(as_csr(A), "_records", {}).values()]
    kinds = {r.kind for r in recs if isinstance(r, record.ForwardRecord)}
    # the training modes' backward went through gcnk_gcn_backward_f32
    assert (mode != "eval") == any(isinstance(r, record.BackwardRecord) for r in recs)
    want = {"factored": record.FACTORED, "dense_factored": record.FACTORED, "spmm_proj": record.SPMM_PROJ,
            "spmm_gemm": record.SPMM_GEMM, "dense_ax": record.DENSE_AX}.get(path)
    if want is not None:
        assert want in kinds, kinds


def test_forward_record_follows_in_place_feature_updates(r8):
    """The inference fast path memoises (x, adj); an in-place change of x's
    values must reach the output (new CSR, factor and record), matching a
    fresh model on a copy."""
    A = r8["adj"].to(DEV)
    X = r8["features"].to(DEV).coalesce()
    torch.manual_seed(1)
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(DEV).eval()
    with torch.no_grad():
        a = m(X, A)
        X._values().mul_(2.0)
        b = m(X, A)
        ref = m(torch.sparse_coo_tensor(X._indices(), X._values().clone(), X.shape).coalesce(), A)
    assert not torch.equal(a, b)
    assert torch.equal(b, ref)


# ------------------------------------------------------------------------------ device factor build

@pytest.mark.parametrize("case", ["r8", "doc_topic_tt", "hubs_first_dense", "20ng"])
def test_device_factor_build_is_bitwise_the_host_build(r8, case):
    """factor.build (csrc/factor_build.hip: U as fixed-order float64 sums over
    each row's CSR items, the A_H block records by ballot compaction) against
    the host float64 restatement oracle/factor_host.py: the structure (hubs,
    k0, Kc, row order), U bit for bit after the one fp32 rounding, the records
    word for word and X's hub rows -- on R8, a doc-topic graph with
    topic-topic edges, a renumbered graph with the hubs first, a ragged M and
    dense X, and the 20ng-shaped graph (70 hubs, BASELINE config 3)."""
    from graph_convolutional_networks_for_text_classification_amd import factor, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    from oracle import factor_host
    if case == "r8":
        A, X = r8["adj"], r8["features"]
    elif case == "doc_topic_tt":
        g = datasets.doc_topic_graph(2000, 40, 5, seed=4, tt_prob=0.3)
        A, X = g["adj"], g["features"]
    elif case == "hubs_first_dense":
        g = datasets.doc_topic_graph(1001, 37, 5, seed=11)
        n = g["nodes"]
        order = np.concatenate([np.arange(1001, n), np.arange(1001)])
        inv = np.empty(n, np.int64)
        inv[order] = np.arange(n)
        a = g["adj"].coalesce()
        A = torch.sparse_coo_tensor(torch.from_numpy(inv)[a.indices()], a.values(), (n, n)).coalesce()
        X = torch.from_numpy(np.ascontiguousarray(g["features_dense"][order]))
    else:
        g = datasets.doc_topic_graph(18846, 70, 20, seed=0)
        A, X = g["adj"], g["features"]
    a = as_csr(A.to(DEV))
    xop = ops.Operand(X.to(DEV))
    Xd = X.to_dense() if X.is_sparse else X      # (a dense-enough sparse X becomes a dense operand)
    d = factor.build(a, xop)
    torch.cuda.synchronize()
    h = factor_host.build(a, xop)
    assert d is not None and h is not None
    assert (d.M, d.H, d.k0, d.Kc, d.nblk, d.rec_words) == (h.M, h.H, h.k0, h.Kc, h.nblk, h.rec_words)
    assert np.array_equal(d.hubs.cpu().numpy(), h.hubs) and np.array_equal(d.perm.numpy(), h.perm)
    Ud = d.U.cpu().numpy()
    assert Ud.shape == h.U.shape
    bad = np.flatnonzero((Ud.view(np.int32) != h.U.view(np.int32)).any(1))
    assert bad.size == 0, f"U differs on {bad.size} rows, first at position {bad[:4]}"
    assert np.array_equal(d.rec.cpu().numpy(), h.rec)
    if xop.csr is not None:
        assert np.array_equal(d.x_hub.rowptr.cpu().numpy(), h.x_hub_rowptr)
        assert np.array_equal(d.x_hub.colind.cpu().numpy(), h.x_hub_colind)
        assert np.array_equal(d.x_hub.val.cpu().numpy().view(np.int32), h.x_hub_val.view(np.int32))
    else:
        assert torch.equal(d.x_hub_dense.cpu(), Xd[torch.from_numpy(h.hubs)])
