"""Whole-forward and whole-backward launch records (gcnk_gcn_forward_f32,
gcnk_gcn_backward_f32, include/gcnk.h).

The reference's trainer calls ``model.forward(features, adj)`` eagerly every
epoch (trainer.py:357 train, trainer.py:382 eval).  Issued op by op, the
forward's 4-5 launches each paid Python + ctypes marshalling, plan and
workspace lookups and device guards: 76-92 us per forward for ~26 us of
kernels (profiles/r03_eager_forward_host_profile.log).  A ForwardRecord holds,
per (adjacency, features, widths, stream), every pointer that does not change
between calls -- plans and their host headers, workspaces, counter regions,
the factored operands and the intermediates S1 / S2 -- in a C struct, and one
ctypes call issues the whole forward.  The launches, their arguments and their
order are those of ops.GCNFn's per-op path, so results are bitwise the same.
"""
import ctypes
import threading

import torch

from . import _lib, factor, ops
from .sparse import DENSE_THRESHOLD

_c = ctypes


class PlanRef(_c.Structure):
    """gcnk_plan_ref (include/gcnk.h)."""
    _fields_ = [("plan", _c.c_void_p), ("hdr", _c.c_int32 * 16), ("workspace", _c.c_void_p),
                ("workspace_bytes", _c.c_int64), ("counters", _c.c_void_p), ("counter_bytes", _c.c_int64),
                ("lanes_hint", _c.c_int32), ("pad_", _c.c_int32)]


class GcnFwd(_c.Structure):
    """gcnk_gcn_fwd (include/gcnk.h)."""
    _fields_ = [("kind", _c.c_int32), ("M", _c.c_int32), ("F", _c.c_int32), ("P", _c.c_int32),
                ("x_rows", _c.c_int32), ("x_cols", _c.c_int32), ("x", PlanRef),
                ("x_dense", _c.c_void_p), ("ldx", _c.c_int64), ("x_split_k", _c.c_int32), ("pad0_", _c.c_int32),
                ("gemm_ws", _c.c_void_p), ("gemm_ws_bytes", _c.c_int64), ("s1", _c.c_void_p), ("lds1", _c.c_int64),
                ("Kc", _c.c_int32), ("nhub", _c.c_int32), ("k0", _c.c_int32), ("rec_words", _c.c_int32),
                ("U", _c.c_void_p), ("ldu", _c.c_int64), ("rec", _c.c_void_p),
                ("aF", PlanRef), ("aP", PlanRef), ("s2", _c.c_void_p), ("lds2", _c.c_int64),
                ("h1_tmp", _c.c_void_p), ("ld_h1_tmp", _c.c_int64)]


class GcnBwd(_c.Structure):
    """gcnk_gcn_bwd (include/gcnk.h)."""
    _fields_ = [("M", _c.c_int32), ("F", _c.c_int32), ("P", _c.c_int32), ("x_rows", _c.c_int32),
                ("x_cols", _c.c_int32), ("x_split_k", _c.c_int32), ("flags", _c.c_int32), ("pad1_", _c.c_int32),
                ("aTP", PlanRef), ("aTF", PlanRef),
                ("xT", PlanRef), ("x_dense", _c.c_void_p), ("ldx", _c.c_int64), ("gemm_ws", _c.c_void_p),
                ("gemm_ws_bytes", _c.c_int64), ("gS2", _c.c_void_p), ("gZ1", _c.c_void_p), ("gS1", _c.c_void_p),
                ("bwd2_ws", _c.c_void_p), ("bwd2_ws_bytes", _c.c_int64)]


FACTORED, SPMM_PROJ, SPMM_GEMM, DENSE_AX = 1, 2, 3, 4
KIND_NAMES = {FACTORED: "factored", SPMM_PROJ: "spmm+proj", SPMM_GEMM: "spmm+gemm", DENSE_AX: "dense-ax"}
BWD_AX_DIRECT = 1


def layout_ok():
    """The ctypes mirrors match the library's struct layout (gcnk_gcn_fwd_layout)."""
    buf = (_c.c_int64 * 16)()
    n = _lib.load().gcnk_gcn_fwd_layout(buf, 16)
    want = [_c.sizeof(PlanRef), _c.sizeof(GcnFwd), GcnFwd.x.offset, GcnFwd.U.offset, GcnFwd.aF.offset,
            GcnFwd.aP.offset, GcnFwd.ld_h1_tmp.offset, PlanRef.lanes_hint.offset, _c.sizeof(GcnBwd),
            GcnBwd.xT.offset, GcnBwd.bwd2_ws_bytes.offset]
    return n == len(want) and list(buf)[:n] == want


def _fill_plan(ref, plan, F, lanes, device, keep):
    """PlanRef for `plan` at width F: its header, a workspace and the counter
    region torch's current stream uses (Plan.counters)."""
    ref.plan = plan.buf.data_ptr()
    for i in range(16):
        ref.hdr[i] = plan.hdr[i]
    wsb = plan.workspace_bytes(F)
    if wsb > 0:
        ws = torch.empty((wsb + 3) // 4, dtype=torch.float32, device=device)
        keep.append(ws)
        ref.workspace, ref.workspace_bytes = ws.data_ptr(), wsb
    cnt = plan.counters(device)
    if cnt is not None:
        keep.append(cnt)
        ref.counters, ref.counter_bytes = cnt.data_ptr(), 4 * cnt.numel()
    ref.lanes_hint = int(lanes)


class ForwardRecord:
    """One filled gcnk_gcn_fwd plus the tensors and plans it points into."""

    __slots__ = ("s", "keep", "kind", "M", "F", "P", "src", "pinned", "__weakref__")

    def __init__(self, adj, xop, F, P, device, train=False):
        lib = _lib.load()
        M = adj.shape[0]
        s = GcnFwd()
        keep = []
        s.M, s.F, s.P = M, F, P
        dax = ops.dense_ax_for(adj, xop, F, P)
        fac = ops.factor_for(adj, xop) if dax is None else None
        kind = None
        if dax is not None:
            # gc1 from the cached A-hat X: no first product, no F-wide plan
            kind = DENSE_AX
            s.Kc, s.U, s.ldu = dax.K, dax.AX.data_ptr(), dax.AX.stride(0)
            keep.append(dax.AX)
            s2 = torch.empty((M, P), dtype=torch.float32, device=device)
            keep.append(s2)
            s.s2, s.lds2 = s2.data_ptr(), P
            aP = adj.plan(ops.default_ipc(adj, P, 0), int(lib.gcnk_spmm_groups(P, 0)), DENSE_THRESHOLD)
            _fill_plan(s.aP, aP, P, 0, device, keep)
            keep.append(aP)
            s.kind = kind
            self.s, self.keep, self.kind, self.M, self.F, self.P = s, keep, kind, M, F, P
            self.src = (adj, xop.dense)
            return
        if fac is not None and P <= 32 and F % 4 == 0 and F <= 256 and \
                int(lib.gcnk_hubfactor_lds_bytes(F, fac.Kc, fac.H, fac.rec_words, P)) <= 160 * 1024:
            kind = FACTORED
            s.Kc, s.nhub, s.k0, s.rec_words = fac.Kc, fac.H, fac.k0, fac.rec_words
            s.U, s.ldu, s.rec = fac.U.data_ptr(), fac.U.stride(0), fac.rec.data_ptr()
            keep += [fac.U, fac.rec]
            if fac.hub_operand(train) == "csr":
                x_csr, x_dense = fac.x_hub, None
            else:
                x_csr, x_dense = None, fac.x_hub_dense
        else:
            x_csr, x_dense = xop.csr, xop.dense
            plan = None
            if ops.FUSE_PROJECTION and P <= ops.FUSE_MAX_P and F % 4 == 0 and F <= 256:
                lanes = 64
                plan = adj.plan(ops.default_ipc(adj, F, lanes), int(lib.gcnk_spmm_groups(F, lanes)), DENSE_THRESHOLD)
                # the fused projection runs on plans without dense tile blocks
                kind = SPMM_PROJ if int(plan.hdr[8]) == 0 else None
            if kind is None:
                lanes = 0
                plan = adj.plan(ops.default_ipc(adj, F, lanes), int(lib.gcnk_spmm_groups(F, lanes)), DENSE_THRESHOLD)
                kind = SPMM_GEMM
            # H1 scratch for an eval forward: the unfused path's intermediate, and
            # the fused path's fallback where the library refuses the fusion (an
            # operand it cannot take as float4, gcnk_gcn_forward_f32)
            h = torch.empty((M, F), dtype=torch.float32, device=device)
            keep.append(h)
            s.h1_tmp, s.ld_h1_tmp = h.data_ptr(), F
            _fill_plan(s.aF, plan, F, lanes, device, keep)
            keep.append(plan)
        # the first product S1 = X W1 (factored: S_T = X_hubs W1)
        if x_csr is not None:
            rows, cols = x_csr.shape
            xp = x_csr.plan(ops.default_ipc(x_csr, F, 0), int(lib.gcnk_spmm_groups(F, 0)), DENSE_THRESHOLD)
            _fill_plan(s.x, xp, F, 0, device, keep)
            keep.append(xp)
        else:
            rows, cols = x_dense.shape
            s.x_dense, s.ldx = x_dense.data_ptr(), x_dense.stride(0)
            keep.append(x_dense)
            s.x_split_k = ops.default_split_k(rows, F, cols)
        s.x_rows, s.x_cols = rows, cols
        # GEMM workspace: split-K slabs of X W1 (dense X); H1 W2 runs unsplit
        gws = 0
        if x_dense is not None:
            gws = int(lib.gcnk_gemm_workspace_bytes(rows, F, cols, s.x_split_k))
        if gws > 0:
            g = torch.empty((gws + 3) // 4, dtype=torch.float32, device=device)
            keep.append(g)
            s.gemm_ws, s.gemm_ws_bytes = g.data_ptr(), gws
        s1 = torch.empty((rows, F), dtype=torch.float32, device=device)
        s2 = torch.empty((M, P), dtype=torch.float32, device=device)
        keep += [s1, s2]
        s.s1, s.lds1, s.s2, s.lds2 = s1.data_ptr(), F, s2.data_ptr(), P
        # gc2's aggregation A S2 + b2 (ops.spmm, lanes 0)
        aP = adj.plan(ops.default_ipc(adj, P, 0), int(lib.gcnk_spmm_groups(P, 0)), DENSE_THRESHOLD)
        _fill_plan(s.aP, aP, P, 0, device, keep)
        keep.append(aP)
        s.kind = kind
        self.s, self.keep, self.kind, self.M, self.F, self.P = s, keep, kind, M, F, P
        self.src = (adj, xop.csr if xop.csr is not None else xop.dense)

    def run(self, W1, b1, W2, b2, epi, mask, scale, keep_prob, seed, offset, rng_base, store_h1, stream):
        """(out, H1) of one forward; H1 is None unless store_h1."""
        dev = W1.device
        out = torch.empty((self.M, self.P), dtype=torch.float32, device=dev)
        H1 = torch.empty((self.M, self.F), dtype=torch.float32, device=dev) if store_h1 else None
        rc = _lib.load().gcnk_gcn_forward_f32(
            _c.byref(self.s), W1.data_ptr(), b1.data_ptr() if b1 is not None else None, W2.data_ptr(),
            b2.data_ptr() if b2 is not None else None, out.data_ptr(), self.P,
            H1.data_ptr() if H1 is not None else None, self.F, epi,
            mask.data_ptr() if mask is not None else None, mask.stride(0) if mask is not None else 0, scale,
            keep_prob, seed & (2**64 - 1), offset & (2**64 - 1),
            rng_base.data_ptr() if rng_base is not None else None, stream)
        _lib.check(rc, "gcnk_gcn_forward_f32")
        return out, H1


class BackwardRecord:
    """One filled gcnk_gcn_bwd: ops.GCNFn.backward's launches (A-hat^T G, the
    fused gcn_bwd2, A-hat^T gZ1, X^T gS1) with their plans, workspaces and
    scratch, issued by one ctypes call (bitwise the per-op backward)."""

    __slots__ = ("s", "keep", "M", "F", "P", "x_cols", "src", "pinned", "__weakref__")

    def __init__(self, adj, xop, F, P, device):
        lib = _lib.load()
        M = adj.shape[0]
        s = GcnBwd()
        keep = []
        s.M, s.F, s.P = M, F, P
        adjT = adj.t()
        keep.append(adjT)
        dax = ops.dense_ax_for(adj, xop, F, P)
        for ref, width in ((s.aTP, P), (s.aTF, F)) if dax is None else ((s.aTP, P),):
            pl = adjT.plan(ops.default_ipc(adjT, width, 0), int(lib.gcnk_spmm_groups(width, 0)), DENSE_THRESHOLD)
            _fill_plan(ref, pl, width, 0, device, keep)
            keep.append(pl)
        rows, cols = xop.shape
        s.x_rows, s.x_cols = rows, cols
        if dax is not None:        # gW1 = (A-hat X)^T gZ1 (the DENSE_AX forward's association)
            s.flags = BWD_AX_DIRECT
            s.x_dense, s.ldx = dax.AX.data_ptr(), dax.AX.stride(0)
            s.x_rows, s.x_cols = M, dax.K
            s.x_split_k = ops.default_split_k(dax.K, F, M, trans=True)
            keep.append(dax.AX)
            gws = int(lib.gcnk_gemm_workspace_bytes(dax.K, F, M, s.x_split_k))
            if gws > 0:
                g = torch.empty((gws + 3) // 4, dtype=torch.float32, device=device)
                keep.append(g)
                s.gemm_ws, s.gemm_ws_bytes = g.data_ptr(), gws
        elif xop.csr is not None:    # X^T gS1 = spmm(X^T, gS1)  (ops.XOperand.t_times)
            xT = xop.csr.t()
            pl = xT.plan(ops.default_ipc(xT, F, 0), int(lib.gcnk_spmm_groups(F, 0)), DENSE_THRESHOLD)
            _fill_plan(s.xT, pl, F, 0, device, keep)
            keep += [xT, pl]
        else:                      # gemm(X, gS1, transA=True)
            x = xop.dense
            s.x_dense, s.ldx = x.data_ptr(), x.stride(0)
            s.x_split_k = ops.default_split_k(cols, F, rows, trans=True)
            keep.append(x)
            gws = int(lib.gcnk_gemm_workspace_bytes(cols, F, rows, s.x_split_k))
            if gws > 0:
                g = torch.empty((gws + 3) // 4, dtype=torch.float32, device=device)
                keep.append(g)
                s.gemm_ws, s.gemm_ws_bytes = g.data_ptr(), gws
        gS2 = torch.empty((M, P), dtype=torch.float32, device=device)
        gZ1 = torch.empty((M, F), dtype=torch.float32, device=device)
        keep += [gS2, gZ1]
        s.gS2, s.gZ1 = gS2.data_ptr(), gZ1.data_ptr()
        if dax is None:
            gS1 = torch.empty((rows, F), dtype=torch.float32, device=device)
            keep.append(gS1)
            s.gS1 = gS1.data_ptr()
        wsb = int(lib.gcnk_gcn_bwd2_workspace_bytes(M, F, P))
        if wsb > 0:
            w = torch.empty((wsb + 3) // 4, dtype=torch.float32, device=device)
            keep.append(w)
            s.bwd2_ws, s.bwd2_ws_bytes = w.data_ptr(), wsb
        self.s, self.keep, self.M, self.F, self.P, self.x_cols = s, keep, M, F, P, cols
        self.src = (adj, xop.csr if xop.csr is not None else xop.dense)

    def run(self, G, H1, W2, scale, want_gw1, want_gb1, want_gw2, want_gb2, stream):
        """(gW1, gb1, gW2, gb2), each None unless wanted."""
        dev = G.device
        gW1 = torch.empty((self.x_cols, self.F), dtype=torch.float32, device=dev) if want_gw1 else None
        gb1 = torch.empty(self.F, dtype=torch.float32, device=dev) if want_gb1 else None
        gW2 = torch.empty((self.F, self.P), dtype=torch.float32, device=dev) if want_gw2 else None
        gb2 = torch.empty(self.P, dtype=torch.float32, device=dev) if want_gb2 else None
        rc = _lib.load().gcnk_gcn_backward_f32(
            _c.byref(self.s), G.data_ptr(), H1.data_ptr(), H1.stride(0), W2.data_ptr(), scale,
            gW1.data_ptr() if gW1 is not None else None, gb1.data_ptr() if gb1 is not None else None,
            gW2.data_ptr() if gW2 is not None else None, gb2.data_ptr() if gb2 is not None else None, stream)
        _lib.check(rc, "gcnk_gcn_backward_f32")
        return gW1, gb1, gW2, gb2


_lock = threading.Lock()


def get_backward(adj, xop, F, P, device):
    """(record, stream): the BackwardRecord of (adj, X, F, P) for torch's
    current stream, built on first use, and that stream."""
    return _get(adj, xop, F, P, device, BackwardRecord, "bwd")


def get(adj, xop, F, P, device, train=False):
    """(record, stream): the ForwardRecord of (adj, X, F, P) for torch's current
    stream, built on first use, and that stream.  ``train``: a forward whose H1
    the backward keeps (its X_hubs W1 may take another form, factor.hub_operand)."""
    return _get(adj, xop, F, P, device, ForwardRecord, "fwd", train)


def _get(adj, xop, F, P, device, cls, tag, train=False):
    """A record's launches bake in raw pointers to its scratch buffers, so a
    record is rebuilt when either operand's values change in place (the
    factored operands and plans are derived from them) and a record that was
    used while a hipGraph was being captured is never evicted: the graph keeps
    replaying into its buffers.  A record's scratch (S1, S2, H1) is shared by
    every launch on its stream; a graph captured on that stream replays into
    it, so two graphs of the same record must not replay concurrently."""
    stream = torch.cuda.current_stream(device).cuda_stream
    src = xop.csr if xop.csr is not None else xop.dense
    key = (tag, id(src), F, P, stream, ops.FACTOR_GC1, ops.FUSE_PROJECTION, ops.DENSE_AX, factor.XHUB_DENSE,
           bool(train) and factor.XHUB_TRAIN_TILE)
    recs = getattr(adj, "_records", None)
    if recs is None:
        with _lock:
            recs = getattr(adj, "_records", None)
            if recs is None:
                recs = adj._records = {}
    capturing = torch.cuda.is_current_stream_capturing()
    ver = (_version(src), _version(adj))
    hit = recs.get(key)
    if hit is not None and hit[0] is src and ver == hit[1]:
        if capturing:
            hit[2].pinned = True
        return hit[2], stream
    with _lock:
        rec = cls(adj, xop, F, P, device, train) if cls is ForwardRecord else cls(adj, xop, F, P, device)
        rec.pinned = capturing
        old = recs.get(key)
        if old is not None and old[2].pinned:
            _PINNED.append(old[2])   # replaced (operands changed) but still referenced by a graph
        while len(recs) >= 8:
            victim = next((k for k, v in recs.items() if not v[2].pinned), None)
            if victim is None:
                break
            recs.pop(victim)
        recs[key] = (src, ver, rec)
        return rec, stream


# records displaced from a cache while a captured graph still points into them:
# kept alive (a replay writes into their buffers through raw pointers, which
# no reference count sees), so this list grows by one record each time the
# operands of a captured forward change in place; release_pinned() drops them
# once the caller's graphs are gone
_PINNED = []


def release_pinned():
    """Drop the records kept alive for hipGraphs captured before their operands
    changed (call after those graphs are destroyed; replaying one afterwards
    writes into freed memory).  Returns how many were dropped."""
    with _lock:
        n = len(_PINNED)
        _PINNED.clear()
    return n


def _version(src):
    return src._version if isinstance(src, torch.Tensor) else (src.val._version, src.val.data_ptr())
