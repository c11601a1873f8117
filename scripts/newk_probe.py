"""Round-5 kernels alone (warm, hipGraph of back-to-back launches): the
one-launch small-M GEMM X_hubs W1 (R8 shape [50 x 7463] x [7463 x 200]) and
gcnk_dense_gc1_f32 on the 20ng shape (M 18,916, K 100, F 200, P 20) and the
gensim R8 shape (7,724, 100, 200, 8), eval epilogue, H1 not stored.  One JSON
line per op.  Run it under GCNK_LIB=<variant .so> to compare kernel builds
(the GCNK_SMALLM_EXP / GCNK_DG_EXP experiment knobs).

  python scripts/newk_probe.py [--reps 200]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--ops", default="smallm,dense20,dense8", help="subset of smallm,dense20,dense8,densem (M sweep at K 100, F 200, P 20)")
    args = ap.parse_args()
    import torch
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import _lib, ops
    from hub_probe import time_graph
    dev = torch.device("cuda", 0)
    tag = os.path.basename(os.environ.get("GCNK_LIB", "libgcnk.so"))
    lib = _lib.load()
    g = torch.Generator().manual_seed(0)

    def line(op, us, **kw):
        print(json.dumps({"lib": tag, "op": op, "us": round(us, 3), **kw}), flush=True)

    ops_sel = set(args.ops.split(","))
    # X_hubs W1
    if "smallm" in ops_sel:
        smallm(torch, ops, time_graph, g, dev, line, args.reps)
    dense(torch, _lib, lib, time_graph, g, dev, line, args.reps, ops_sel)


def smallm(torch, ops, time_graph, g, dev, line, reps):
    A = torch.zeros((50, 7464)).normal_(generator=g).to(dev)
    B = torch.zeros((7463, 200)).normal_(generator=g).to(dev)
    Av = A[:, :7463]
    C = ops.gemm_smallm(Av, B)
    err = float((C.cpu().double() - Av.cpu().double() @ B.cpu().double()).abs().max())
    line("gemm_smallm 50x200x7463", time_graph([lambda: ops.gemm_smallm(Av, B, out=C)], reps), max_err=err)
    # the library GEMMs on the same product (reference points: rocBLAS / hipBLASLt through torch.mm)
    Ac = Av.contiguous()
    C2 = torch.mm(Ac, B)
    line("torch.mm 50x200x7463 (library)", time_graph([lambda: torch.mm(Ac, B, out=C2)], reps),
         max_err=float((C2.cpu().double() - Av.cpu().double() @ B.cpu().double()).abs().max()))
    C3 = ops.gemm(Av, B)
    line("ops.gemm 50x200x7463 (tiled MFMA)", time_graph([lambda: ops.gemm(Av, B, out=C3)], reps))


def dense(torch, _lib, lib, time_graph, g, dev, line, reps, ops_sel):
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    cases = [("dense20", (18916, 100, 200, 20)), ("dense8", (7724, 100, 200, 8))]
    cases += [("densem", (m, 100, 200, 20)) for m in (8192, 16384, 16400, 18916, 24576)]
    for name, (M, K, F, P) in cases:
        if name not in ops_sel:
            continue
        AX = torch.zeros((M, K)).normal_(generator=g).to(dev)
        W1 = (torch.zeros((K, F)).normal_(generator=g) * 0.1).to(dev)
        W2 = (torch.zeros((F, P)).normal_(generator=g) * 0.1).to(dev)
        b1 = torch.zeros(F).normal_(generator=g).to(dev)
        S2 = torch.empty((M, P), device=dev)

        def run():   # (the stream inside: a hipGraph capture runs on a side stream)
            stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            _lib.check(lib.gcnk_dense_gc1_f32(M, K, F, P, p(AX), K, p(W1), F, p(b1), _lib.EPI_BIAS_RELU, None, 0,
                                              1.0, 1.0, 0, 0, None, p(W2), P, None, 0, p(S2), P, stream),
                       "gcnk_dense_gc1_f32")
        run()
        torch.cuda.synchronize()
        want = torch.relu(AX.cpu().double() @ W1.cpu().double() + b1.cpu().double()) @ W2.cpu().double()
        err = float((S2.cpu().double() - want).abs().max())
        line(f"dense_gc1 M{M} K{K} F{F} P{P}", time_graph([run], reps), max_err=err)


if __name__ == "__main__":
    main()
