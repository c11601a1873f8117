"""Hub factorisation of the first GCN layer (csrc/factor.hip).

The reference's gc1 computes ``th.spmm(adj, th.spmm(X, W1)) + b1``
(layer.py:102,106,110).  On its doc-topic graph (trainer.py:98-148,
utils.py:185-213) A-hat's rows split into a few hub rows (the topics) and
light rows (the documents) whose nonzeros are hub columns plus their own
diagonal, and X's document rows are supported on a small column range (the
topic-weight columns, trainer.py:226-238).  Then

    A X W1 = U W1[k0:k0+Kc] + A_H (X_hubs W1)

with U [M x Kc] dense (rows in the block order ``perm``) -- row d (light): A_dd X[d, Kc]; row t (hub):
sum over light d of A_td X[d, Kc] -- and A_H = A-hat restricted to hub columns.
U and A_H depend only on (A-hat, X), so they are built here ONCE per operand
pair (on the device: csrc/factor_build.hip, float64 sums in a fixed order,
rounded to fp32 once) and cached on the adjacency; every
forward then runs X_hubs W1 (the tile GEMM over X's dense hub rows) and one
launch of gcnk_hubfactor_gc1_f32 (U W1[Kc] on MFMA + A_H S_T + bias + ReLU +
dropout + the gc2 projection H1 W2), and the hub rows' 600-term gather sums
of the SpMM never run.  The association differs from A (X W1) only in fp32
rounding (checked against the reference's goldens to 1e-4, tests/).
"""
import os
import threading

import numpy as np
import torch

from .sparse import CSR

MAX_HUBS = 128    # hub rows staged in LDS (S_T [hubs x F]; the kernel checks the LDS budget)
# X[hubs] W1 (R8: 50 dense hub rows x 7463): the SpMM tile plan on their CSR
# plus its slab reduce (9.8 us per call; 6.8 + 4.9 us in the forward's trace);
# dense X's hub rows: the MFMA GEMM (gcnk_gemm_f32, small-M split-K).  A dense
# copy of R8's sparse hub rows through round 6's in-workgroup K-split GEMM
# (30 slabs instead of 117): 7.16 + 4.86 us against the tile plan's 6.79 + 4.89
# in one trace (profiles/r06_xhub_ab_*), yet the eval forward 25.20 / 25.26 us
# against 25.56 / 25.48 interleaved (profiles/r06_xhub_forward_ab.json); in the
# training step, where W1 arrives fresh from Adam, the tile plan is the faster
# one (profiles/r06_xhub_train_ab.log), so training forwards keep it
# (XHUB_TRAIN_TILE).  Measured
# and removed (DESIGN.md keeps the numbers): a dense copy of the sparse hub rows
# through the small-M split-K GEMM (10.4 us per call, profiles/r04_smallm_*), a
# one-launch split-K kernel with two levels of last-arriver slab sums (12.1 us,
# round 4), <= 4 K-slabs summed by the factored gc1 while it stages S_T (slab
# GEMM 11.9 us + factored gc1 9.9 -> 13.2 us, profiles/r05_fwdtrace_r8_slabs_*;
# kslab.hip, ABI 11) and a one-launch small-M GEMM whose tiles' last workgroups
# sum the partials (12.2 us, ~4 of it the coherent hand-off,
# profiles/r05_smallm_*; smallm.hip, ABI 11).
# X's hub rows at least XHUB_DENSE_FILL full run X_hubs W1 as a dense small-M
# GEMM; GCNK_XHUB_DENSE=0 keeps the tile SpMM on their CSR (A/B timing)
XHUB_DENSE = os.environ.get("GCNK_XHUB_DENSE", "1") != "0"
XHUB_DENSE_FILL = 0.5
XHUB_TRAIN_TILE = os.environ.get("GCNK_XHUB_TRAIN_TILE", "1") != "0"
MAX_KC = 128      # X's light-row column range (U's width)
ROWS_PER_BLOCK = 32   # csrc/factor.hip kRB
# record words before the items: 33 row offsets | 3 pad | 32 row ids (-1 past
# M) -- csrc/factor.hip kRecHead.  A block's rows are a slice of the row order
# `perm` (hub rows spread evenly between the light rows, so no block carries
# more than one or two hub rows' long item lists: the item loop is LDS-bound per
# workgroup, and R8's contiguous topic rows made three blocks the kernel's tail).
REC_HEAD = 68
REC_ROW = 36

_lock = threading.Lock()


class HubFactor:
    """The (A-hat, X)-fixed operands of the factored gc1, resident on the device."""

    __slots__ = ("M", "H", "K", "hubs", "k0", "Kc", "U", "perm", "rec", "rec_words", "nblk", "x_hub",
                 "x_hub_dense", "_src")

    def hub_operand(self, train=False):
        """'csr' or 'dense': which form of X[hubs] the product S_T = X[hubs] W1
        takes (a training forward keeps the tile plan where both exist)."""
        if self.x_hub_dense is None or (train and XHUB_TRAIN_TILE and self.x_hub is not None):
            return "csr"
        return "dense"

    def hub_times(self, W, train=False):
        """S_T = X[hubs] @ W  (the hub rows of reference layer.py:102)."""
        from .ops import gemm, spmm
        if self.hub_operand(train) == "csr":
            return spmm(self.x_hub, W)
        return gemm(self.x_hub_dense, W)


def _perm(hubs, M):
    """Row order: the light rows in order, hub j inserted near (j + 1/2) M / H."""
    H = len(hubs)
    light = np.ones(M, bool)
    light[hubs] = False
    lights = np.flatnonzero(light)
    pos = ((np.arange(H) + 0.5) * M / H).astype(np.int64)
    perm = np.insert(lights, np.minimum(pos - np.arange(H), len(lights)), hubs)
    assert len(perm) == M
    return perm


def build(adj, xop):
    """HubFactor for (adj, X) on adj's device, or None when the operands lack
    the structure.  The structure test (hub rows, light rows touching only hub
    columns and themselves, X's light-row column range, per-row hub-item
    counts) is one device pass read back once (gcnk_factor_analyze); X's light
    rows (Xl), U, the A_H records and X's hub rows are library kernels
    (csrc/factor_build.hip: fixed-order float64 sums, bitwise the host
    restatement oracle/factor_host.py).  No torch kernel runs here: their
    first-use module loads were ~120 ms of the first forward (round 5)."""
    import ctypes

    from . import _lib
    M, K = adj.shape
    if M != K or xop.shape[0] != M:
        return None
    dev = adj.device
    lib = _lib.load()
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    nnz = adj.nnz
    hmin = max(64, 8 * ((nnz + M - 1) // M))
    x = xop.csr
    info = np.zeros(8, np.int32)
    found = np.zeros(MAX_HUBS + 1, np.int32)
    cnt = np.zeros(M, np.int32)
    wsb = int(lib.gcnk_factor_analyze_workspace_bytes(M, MAX_HUBS + 1))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    if x is not None:
        xa = (x.rowptr.data_ptr(), x.colind.data_ptr(), x.val.data_ptr(), None, 0, x.shape[1])
    else:
        if xop.dense.stride(1) != 1:
            raise RuntimeError("factor.build: dense features need unit column stride")
        xa = (None, None, None, xop.dense.data_ptr(), xop.dense.stride(0), xop.shape[1])
    with torch.cuda.device(dev):
        _lib.check(lib.gcnk_factor_analyze(adj.rowptr.data_ptr(), adj.colind.data_ptr(), M, hmin, *xa, MAX_HUBS + 1,
                                           info.ctypes.data, found.ctypes.data, cnt.ctypes.data, ws.data_ptr(), wsb,
                                           stream), "gcnk_factor_analyze")
    H, bad, k0, k1, xtot = (int(t) for t in info[:5])
    if H == 0 or H > MAX_HUBS or H >= M or bad:
        return None
    hubs_h = np.sort(found[:H])
    if k1 >= 0:
        k1 += 1
    else:
        k0, k1 = 0, 1
    Kc = k1 - k0
    if Kc > MAX_KC:
        return None
    Kcp = (Kc + 3) // 4 * 4
    perm = _perm(hubs_h, M)
    hub_index_h = np.full(M, -1, np.int32)
    hub_index_h[hubs_h] = np.arange(H, dtype=np.int32)
    # (host -> device copies only: no kernel launches)
    perm_d = torch.from_numpy(perm.astype(np.int32)).to(dev)
    hub_index = torch.from_numpy(hub_index_h).to(dev)
    hubs_d = torch.from_numpy(hubs_h.astype(np.int32)).to(dev)
    nblk = (M + ROWS_PER_BLOCK - 1) // ROWS_PER_BLOCK
    pc = np.zeros(nblk * ROWS_PER_BLOCK, np.int64)
    pc[:M] = cnt[perm]
    rec_words = (REC_HEAD + 2 * int(pc.reshape(nblk, ROWS_PER_BLOCK).sum(1).max()) + 3) // 4 * 4
    U = torch.empty((M, Kcp), dtype=torch.float32, device=dev)
    rec = torch.empty((nblk, rec_words), dtype=torch.int32, device=dev)
    overflow = torch.empty(1, dtype=torch.int32, device=dev)
    rp, ci, v = adj.rowptr, adj.colind, adj.val
    with torch.cuda.device(dev):
        # X's light rows, columns [k0, k1), dense (hub rows never read)
        if x is not None:
            Xl = torch.empty((M, Kcp), dtype=torch.float32, device=dev)
            _lib.check(lib.gcnk_factor_xl_f32(x.rowptr.data_ptr(), x.colind.data_ptr(), x.val.data_ptr(), M,
                                              hub_index.data_ptr(), k0, Kc, Xl.data_ptr(), Kcp, Kcp, stream),
                       "gcnk_factor_xl_f32")
            xl_ptr, ldxl = Xl.data_ptr(), Kcp
        else:
            xl_ptr, ldxl = xop.dense.data_ptr() + 4 * k0, xop.dense.stride(0)
        _lib.check(lib.gcnk_factor_u_f32(rp.data_ptr(), ci.data_ptr(), v.data_ptr(), M, hub_index.data_ptr(),
                                         perm_d.data_ptr(), xl_ptr, ldxl, Kc, U.data_ptr(), Kcp, Kcp, stream),
                   "gcnk_factor_u_f32")
        # A_H records: each block's hub items, sized from the per-row counts in block order
        _lib.check(lib.gcnk_factor_records(rp.data_ptr(), ci.data_ptr(), v.data_ptr(), M, hub_index.data_ptr(),
                                           perm_d.data_ptr(), rec.data_ptr(), rec_words, overflow.data_ptr(), stream),
                   "gcnk_factor_records")
        f = HubFactor()
        if x is not None:
            # X's hub rows as a CSR (rows in hub order)
            hrp = torch.empty(H + 1, dtype=torch.int32, device=dev)
            hci = torch.empty(max(xtot, 1), dtype=torch.int32, device=dev)
            hv = torch.empty(max(xtot, 1), dtype=torch.float32, device=dev)
            _lib.check(lib.gcnk_csr_gather_rows(x.rowptr.data_ptr(), x.colind.data_ptr(), x.val.data_ptr(),
                                                hubs_d.data_ptr(), H, hrp.data_ptr(), hci.data_ptr(), hv.data_ptr(),
                                                stream), "gcnk_csr_gather_rows")
            f.x_hub = CSR(hrp, hci[:xtot], hv[:xtot], (H, x.shape[1]))
            f.x_hub_dense = None
            kx = x.shape[1]
            if XHUB_DENSE and H <= 64 and xtot >= XHUB_DENSE_FILL * H * kx and H * kx * 4 <= 64 << 20:
                # dense hub rows (R8's topic rows: all 7,463 columns): X_hubs W1 on the
                # small-M GEMM (gcnk_gemm_f32's in-workgroup K split) instead of the
                # tile plan + its slab reduce
                d = torch.empty((H, (kx + 3) // 4 * 4), dtype=torch.float32, device=dev)
                _lib.check(lib.gcnk_csr_to_dense(hrp.data_ptr(), hci.data_ptr(), hv.data_ptr(), H, kx, d.data_ptr(),
                                                 d.stride(0), stream), "gcnk_csr_to_dense")
                f.x_hub_dense = d[:, :kx]
        else:
            f.x_hub = None
            kx = xop.shape[1]
            d = torch.empty((H, (kx + 3) // 4 * 4), dtype=torch.float32, device=dev)   # rows padded to 4 floats
            _lib.check(lib.gcnk_dense_gather_rows_f32(xop.dense.data_ptr(), xop.dense.stride(0), kx,
                                                      hubs_d.data_ptr(), H, d.data_ptr(), d.stride(0), stream),
                       "gcnk_dense_gather_rows_f32")
            f.x_hub_dense = d[:, :kx]
    f.nblk = nblk
    f.M, f.H, f.k0, f.Kc = M, H, k0, Kc
    f.K = xop.shape[1]
    f.hubs = torch.from_numpy(hubs_h.astype(np.int64))            # host: tests and tools
    f.perm = torch.from_numpy(perm.astype(np.int64))              # host: tests and tools
    f.U, f.rec, f.rec_words = U, rec, rec_words
    if int(overflow.item()) != 0:   # (a device -> host copy, no kernel)
        raise RuntimeError("factor.build: A_H records overflowed their sized length (internal error)")
    return f


_cus = {}


def pays(f, device):
    """Whether the factored gc1 is the faster forward for factor ``f``.  Its
    workgroups (one per 32-row block, one per CU at R8's / 20ng's LDS) each
    restage W1[Kc], S_T and W2, so it pays while the blocks fit one round over
    the CUs: R8 (242 blocks on 256 CUs) 25.0-25.2 us per forward against
    28.7-28.9 on the SpMM path; the 20ng shape (592 blocks) 47.4 against 47.2
    (50.9 against 49.0 before this round's GEMM changes;
    profiles/r04_fwd_path_*.log, record forward, hipGraph)."""
    idx = torch.device(device).index or 0
    n = _cus.get(idx)
    if n is None:
        n = _cus[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return f.nblk <= n


def get(adj, xop):
    """The cached HubFactor of (adj, X), built on first use; None when the
    operands do not factor (the caller runs the generic SpMM path)."""
    src = xop.csr if xop.csr is not None else xop.dense
    # U and A_H bake in A-hat's values too: an in-place change of either
    # operand's values is a new key
    key = (id(src), src.data_ptr() if isinstance(src, torch.Tensor) else src.rowptr.data_ptr(),
           src._version if isinstance(src, torch.Tensor) else src.val._version,
           adj.val.data_ptr(), adj.val._version)
    cache = getattr(adj, "_factors", None)
    if cache is None:
        with _lock:
            cache = getattr(adj, "_factors", None)
            if cache is None:
                cache = adj._factors = {}
    hit = cache.get(key)
    if hit is not None:
        return hit[1]
    with _lock:
        hit = cache.get(key)
        if hit is not None:
            return hit[1]
        f = build(adj, xop)
        if f is not None:
            f._src = src
        while len(cache) >= 4:
            cache.pop(next(iter(cache)))
        cache[key] = (src, f)   # the entry holds the operand: its id cannot be recycled while cached
        return f
