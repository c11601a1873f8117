"""North-star op probe: R8 A-hat x S (F = 200, bias + ReLU) and F = 8 on the
row plan (and the streaming floor "copy"), warm (same buffers back to back)
and cold (rotating > 256 MB of distinct B / C sets, so no launch finds its
operands in the Infinity Cache), with parity against the float64 oracle.  One
JSON line per variant.

  python scripts/hub_probe.py [--reps 200] [--variants row,copy]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gcn_amd  # noqa: E402,F401
from graph_convolutional_networks_for_text_classification_amd import _lib, datasets, ops  # noqa: E402
from graph_convolutional_networks_for_text_classification_amd.sparse import from_torch  # noqa: E402
from oracle import csr_ref  # noqa: E402

# "light" / "topic": the same plan kind over the row subsets of A-hat (the
# other rows emptied, their outputs bias + ReLU only): the document rows alone
# and the topic (hub) rows alone, to split the launch's time
VARIANTS = {"row": {}, "light": {}, "topic": {}}


def row_subset(a, keep_heavy):
    """CSR of A-hat with only its heavy (degree >= max(64, 8 x mean)) or only
    its light rows' nonzeros."""
    from graph_convolutional_networks_for_text_classification_amd.sparse import from_arrays
    rp, ci, v = (t.cpu().numpy() for t in (a.rowptr, a.colind, a.val))
    M = a.shape[0]
    deg = np.diff(rp)
    heavy = deg >= max(64, 8 * -(-a.nnz // M))
    keep = heavy if keep_heavy else ~heavy
    rows = np.repeat(np.arange(M), deg)
    m = keep[rows]
    nrp = np.concatenate([[0], np.cumsum(np.where(keep, deg, 0))]).astype(np.int32)
    return from_arrays(nrp, ci[m].astype(np.int32), v[m].astype(np.float32), a.shape, a.device)


def spmm_bytes(M, K, nnz, F):
    return 4 * (M + 1) + 8 * nnz + 4 * K * F + 4 * M * F


def time_graph(fns, reps_per_fn):
    """Average us per call of a hipGraph replaying fns round-robin."""
    for f in fns:
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    n = 0
    with torch.cuda.graph(g):
        for _ in range(reps_per_fn):
            for f in fns:
                f()
                n += 1
    g.replay()
    torch.cuda.synchronize()
    best = None
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        best = us if best is None else min(best, us)
    del g
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--variants", default="row,copy")
    ap.add_argument("--widths", default="200,8")
    ap.add_argument("--graph", default="r8", choices=["r8", "20ng"])
    ap.add_argument("--ipc", default="", help="comma list of light-row limits to sweep (default: the library's)")
    ap.add_argument("--lanes", default="0", help="comma list of lanes-per-row hints to sweep (0: the library's)")
    ap.add_argument("--mode", default="both", choices=["warm", "cold", "both"],
                    help="which timing graphs to run (one mode alone for a rocprofv3 kernel average)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    if args.graph == "r8":
        g = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    else:
        g = datasets.doc_topic_graph(18846, 70, 20, seed=0)
    a = from_torch(g["adj"].to(dev))
    M = a.shape[0]
    rp, ci, v = (t.cpu().numpy() for t in (a.rowptr, a.colind, a.val))
    for F in (int(x) for x in args.widths.split(",")):
        Bh = np.random.default_rng(F).standard_normal((M, F)).astype(np.float32)
        bias = torch.from_numpy(np.random.default_rng(F + 1).standard_normal(F).astype(np.float32)).to(dev)
        ref = csr_ref.spmm_epilogue(csr_ref.spmm_csr(rp, ci, v, Bh), bias.cpu().numpy(), relu=True)
        nbytes = spmm_bytes(M, M, a.nnz, F)
        nsets = max(2, int(np.ceil(300e6 / (2 * 4 * M * F))))
        Bs = [torch.from_numpy(Bh).to(dev) for _ in range(nsets)]
        Cs = [torch.empty(M, F, device=dev) for _ in range(nsets)]
        ipcs = [int(v) for v in args.ipc.split(",")] if args.ipc else [None]
        lanes_l = [int(v) for v in args.lanes.split(",")]
        for name, ipc, lanes in ((n, i, ln) for n in args.variants.split(",")
                                 for i in (ipcs if n != "copy" else [None])
                                 for ln in (lanes_l if n != "copy" else [0])):
            if name == "copy":
                # the streaming floor of the same bytes: one float4 copy C = B
                # (reads B once, writes C once: the op's compulsory traffic minus the CSR)
                lib = _lib.load()

                def copy(i):
                    _lib.check(lib.gcnk_stream_copy_f32(Bs[i].data_ptr(), Cs[i].data_ptr(), Bs[i].numel(),
                                                        torch.cuda.current_stream().cuda_stream), "copy")
                fns = [(lambda i=i: copy(i)) for i in range(nsets)]
                cold = time_graph(fns, max(1, args.reps // nsets)) if args.mode in ("cold", "both") else float("nan")
                warm = time_graph([lambda: copy(0)], args.reps) if args.mode in ("warm", "both") else float("nan")
                print(json.dumps({"graph": args.graph, "F": F, "variant": "copy", "bytes": 8 * M * F,
                                  "warm_us": round(warm, 3), "cold_us": round(cold, 3), "sets": nsets}), flush=True)
                continue
            assert name in VARIANTS, name
            full = a
            if name != "row":
                a = row_subset(full, name == "topic")
                srp, sci, sv = (t.cpu().numpy() for t in (a.rowptr, a.colind, a.val))
                vref = csr_ref.spmm_epilogue(csr_ref.spmm_csr(srp, sci, sv, Bh), bias.cpu().numpy(), relu=True)
            else:
                vref = ref
            out = ops.spmm(a, Bs[0], bias=bias, epilogue=_lib.EPI_BIAS_RELU, ipc=ipc, lanes=lanes)
            torch.cuda.synchronize()
            err = float(np.abs(out.cpu().numpy().astype(np.float64) - vref).max())
            again = ops.spmm(a, Bs[0], bias=bias, epilogue=_lib.EPI_BIAS_RELU, ipc=ipc, lanes=lanes)
            det = bool(torch.equal(out, again))
            plan = list(a._plans.values())[-1]
            warm = cold = float("nan")
            if args.mode in ("warm", "both"):
                warm = time_graph([lambda: ops.spmm(a, Bs[0], bias=bias, epilogue=_lib.EPI_BIAS_RELU, out=Cs[0],
                                                    ipc=ipc, lanes=lanes)], args.reps)
            fns = [(lambda i=i: ops.spmm(a, Bs[i], bias=bias, epilogue=_lib.EPI_BIAS_RELU, out=Cs[i], ipc=ipc,
                                         lanes=lanes))
                   for i in range(nsets)]
            if args.mode in ("cold", "both"):
                cold = time_graph(fns, max(1, args.reps // nsets))
            vbytes = spmm_bytes(M, M, a.nnz, F)
            print(json.dumps({"graph": args.graph, "F": F, "variant": name, "ipc": ipc, "lanes": lanes, "nnz": a.nnz,
                              "hdr": plan.header, "max_err": err, "deterministic": det,
                              "warm_us": round(warm, 3), "cold_us": round(cold, 3),
                              "warm_frac": vbytes / (warm * 1e-6) / 8e12, "cold_frac": vbytes / (cold * 1e-6) / 8e12,
                              "frac_of_full_bytes_cold": nbytes / (cold * 1e-6) / 8e12, "sets": nsets}), flush=True)
            a = full


if __name__ == "__main__":
    main()
