"""Benchmark of the hot path: the R8 two-layer GCN forward on MI355X.

`python bench.py --gpus N --steps K --warmup W` prints ONE JSON line (rank 0).

Workload (BASELINE.json configs[1]): the R8 doc-topic graph exactly as the
reference prepares it (tests/golden/r8_graph.npz, written by the reference's
own builder and PrepareData in the build container; 7,724 nodes, Â nnz
69,130, X nnz 756,850, nfeat 7,463), 2-layer GCN hidden 200, 8 classes,
random-init weights (torch.manual_seed(0), the reference init), eval mode.
A step = one full GCN forward (X·W1 SpMM, Â·S1 SpMM + bias + ReLU, H1·W2
MFMA GEMM, Â·S2 SpMM + bias), replayed from a hipGraph with all inputs
resident in HBM; --graph-steps forwards are captured per graph (every one a
complete forward), so exactly --steps forwards run in the timed region.

metric/value: SpMM edges/s = (2 · nnz(Â) per forward — the two graph
aggregations of layer.py:106) × steps × ranks / max-over-ranks time;
ms_per_step = GCN-forward ms.  N > 1: the R8 graph does not shard (SURVEY
§8(e)): N independent replicas, "scaling": "weak".

roofline: the north-star kernel (BASELINE.json: the R8 doc-topic SpMM Â·S1 at
hidden 200, with gc1's bias + ReLU fused) with its algorithmic bytes (CSR
SpMM: 4(M+1) + 8 nnz + 4 K F + 4 M F) over its average launch duration,
timed with HIP events on the launch stream around a hipGraph of back-to-back
launches of that op alone; "roofline_dominant" gives the same for the
slowest op of the forward.  "traffic" (PMC FETCH_SIZE + WRITE_SIZE per
launch) comes from the separate rocprofv3 --pmc passes in profiles/.

cpu_baseline: the oracle (torch-CPU restatement issuing the reference's
th.spmm calls on the same COO tensors) on this host's cores, bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
# PMC summary of the forward's kernels (scripts/pmc.sh: separate FETCH_SIZE and
# WRITE_SIZE passes, FETCH doubled per the gfx950 correction), committed per round
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")
# kernels each op of the forward launches (names as rocprofv3 / the PMC summary give them)
OP_KERNELS = {
    "spmm_XW1": ["spmm_tile_kernel<true, 7>", "spmm_tile_reduce_kernel"],
    "spmm_AS1_F200": ["spmm_row_kernel<256, 64, 4, 8, 0>"],
    "gemm_H1W2": ["gemm_skinny_ksplit_kernel<4>"],
    "spmm_AS2_F8": ["spmm_row_kernel<64, 2, 4, 8, 0>"],
}


def pmc_traffic(op):
    """HBM-side bytes per launch of `op` from the committed PMC summary, or None."""
    try:
        with open(PMC_TRAFFIC) as f:
            t = json.load(f)
        return sum(t[k]["hbm_bytes_per_launch"] for k in OP_KERNELS[op])
    except (OSError, KeyError, ValueError):
        return None


def spmm_bytes(M, K, nnz, F):
    return 4 * (M + 1) + 8 * nnz + 4 * K * F + 4 * M * F


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--graph-steps", type=int, default=10,
                    help="forwards captured per hipGraph (steps must be a multiple; amortises the per-replay floor)")
    ap.add_argument("--cpu-sample-s", type=float, default=10.0, help="seconds of CPU baseline work (0 = skip)")
    ap.add_argument("--kernel-reps", type=int, default=200, help="launches per kernel-timing graph")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr

    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    N, nfeat, nclass, nhid = r8["nodes"], r8["nfeat"], r8["nclass"], 200
    torch.manual_seed(0)
    model = GCN(nfeat=nfeat, nhid=nhid, nclass=nclass, dropout=0.5).to(dev).eval()
    adj = r8["adj"].to(dev)
    x = r8["features"].to(dev)
    a_csr, x_csr = as_csr(adj), as_csr(x)
    nnz_a, nnz_x = a_csr.nnz, x_csr.nnz

    def forward():
        with torch.no_grad():
            return model(x, adj)

    out = forward()   # builds CSR caches and schedules (one-time)
    torch.cuda.synchronize()
    if args.no_graph:
        step = forward
    else:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                forward()
        torch.cuda.current_stream().wait_stream(s)
        per = max(1, args.graph_steps)
        while args.steps % per or args.warmup % per:
            per -= 1
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(per):
                out = forward()
        step = graph.replay
    per = 1 if args.no_graph else per   # forwards per step() call

    for _ in range(args.warmup // per):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps // per):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)

    # ---- per-op durations: hipGraph of back-to-back launches of one op of the
    #      forward, HIP events on the launch stream (torch's current stream, the
    #      stream every op is enqueued on).  Each duration includes the
    #      dispatch gap between consecutive launches (~1.5 us on MI355X), so it
    #      is an upper bound of the rocprofv3 kernel duration.
    W1, b1 = model.gc1.weight.detach(), model.gc1.bias.detach()
    W2, b2 = model.gc2.weight.detach(), model.gc2.bias.detach()
    with torch.no_grad():
        S1 = ops.spmm(x_csr, W1)
        H1 = ops.spmm(a_csr, S1, bias=b1, epilogue=2)
        S2 = ops.gemm(H1, W2)
        Z = ops.spmm(a_csr, S2, bias=b2, epilogue=1)
    # the forward's ops, in order (layer.py:102, :106+110+182, gc2 :102, gc2 :106+110)
    kernels = {
        "spmm_XW1": (lambda: ops.spmm(x_csr, W1, out=S1), spmm_bytes(N, nfeat, nnz_x, nhid)),
        "spmm_AS1_F200": (lambda: ops.spmm(a_csr, S1, bias=b1, epilogue=2, out=H1), spmm_bytes(N, N, nnz_a, nhid)),
        "gemm_H1W2": (lambda: ops.gemm(H1, W2, out=S2), 4 * (N * nhid + nhid * nclass + N * nclass)),
        "spmm_AS2_F8": (lambda: ops.spmm(a_csr, S2, bias=b2, epilogue=1, out=Z), spmm_bytes(N, N, nnz_a, nclass)),
    }
    ktimes = {}
    for name, (fn, nbytes) in kernels.items():
        reps = args.kernel_reps
        fn()
        torch.cuda.synchronize()
        kg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(kg):
            for _ in range(reps):
                fn()
        kg.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = None
        for _ in range(5):
            e0.record()
            kg.replay()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            best = us if best is None else min(best, us)
        ktimes[name] = {"us": best, "bytes": nbytes, "gbs": nbytes / (best * 1e-6) / 1e9}
        del kg
    dom = max(ktimes, key=lambda k: ktimes[k]["us"])
    north = "spmm_AS1_F200"   # BASELINE.json north_star: the R8 doc-topic SpMM at hidden 200

    # ---- CPU baseline: oracle (reference th.spmm calls) on this host, rank 0, N=1
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample_s > 0:
        from oracle import gcn_ref
        threads = int(os.environ.get("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1))))
        torch.set_num_threads(threads)
        torch.manual_seed(0)
        ref = gcn_ref.RefGCN(nfeat=nfeat, nhid=nhid, nclass=nclass, dropout=0.5).eval()
        xc, ac = r8["features"], r8["adj"]
        with torch.no_grad():
            ref(xc, ac)
            n, tc0 = 0, time.perf_counter()
            while time.perf_counter() - tc0 < args.cpu_sample_s:
                ref(xc, ac)
                n += 1
            tc = (time.perf_counter() - tc0) / n
        cpu = {"value": 2 * nnz_a / tc, "unit": "edges/s", "cores": threads, "kind": "port",
               "sample": f"{n} R8 eval forwards of the oracle (torch-CPU th.spmm on the reference COO tensors), "
                         f"{tc * 1e3:.2f} ms/forward"}

    ms = elapsed / args.steps * 1e3
    value = 2 * nnz_a * args.steps * world / elapsed
    kn, kd = ktimes[north], ktimes[dom]
    line = {
        "metric": "SpMM edges/s and GCN-forward ms on R8 doc-topic graph, 1×MI355X",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "R8 graph fixture generated in-container by the reference's own builder; random-init weights",
        "config": {"workload": "R8 GCN forward (eval), hidden 200, 8 classes, nfeat 7463",
                   "nodes": N, "adj_nnz": nnz_a, "x_nnz": nnz_x, "graph": not args.no_graph,
                   "forwards_per_graph": per,
                   "parallelism": f"replicas{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "kernel": north, "achieved": kn["gbs"], "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": kn["gbs"] / HBM_PEAK_GBS, "traffic": pmc_traffic(north),
                     "avg_launch_us": kn["us"], "algorithmic_bytes": kn["bytes"]},
        "roofline_dominant": {"kernel": dom, "achieved": kd["gbs"], "frac": kd["gbs"] / HBM_PEAK_GBS,
                              "avg_launch_us": kd["us"], "algorithmic_bytes": kd["bytes"],
                              "traffic": pmc_traffic(dom)},
        "kernels_us": {k: round(v["us"], 3) for k, v in ktimes.items()},
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
