"""Synthetic-graph SpMM benchmark: BASELINE.json configs 4 and 5.

  config 4: uniform random CSR, 1M nodes / 20M edges (coalesced: 19,999,805
            nonzeros), F = 256, one GPU;
  config 5: the same graph, F = 4096 feature columns split over the ranks
            (parallel.ColumnShardedSpMM: each rank computes its [M, F/P] block
            with no exchange, then one RCCL all-gather of the blocks, handed over
            in place as parallel.GatheredColumns: no re-layout copy).

One JSON line per case (rank 0).  Launched alone it runs on one GPU (config 5
then means its whole F = 4096 on that GPU, or one rank's F = 512 shard with
--shard-of 8); under torch.distributed.run with P ranks the F columns are
sharded and the all-gather is timed separately.

Per case: ms per SpMM (HIP events on the launch stream, after warm-up; B and
C far exceed the 256 MiB Infinity Cache, so every launch runs cold),
edges/s = nnz / t, GFLOP/s = 2 nnz F / t, algorithmic GB/s = (4(M+1) +
8 nnz + 4 K F + 4 M F) / t against 8 TB/s, and the gather-effective GB/s
(every nonzero reads its whole B row piece: 4(M+1) + 8 nnz + 4 nnz F + 4 M F).

usage: python scripts/bench_synthetic.py [--F 256,512] [--reps 5] [--cpu]
       python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 \\
           scripts/bench_synthetic.py --F 4096
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--F", default="256,512")
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shard-of", type=int, default=1,
                    help="single process: time one rank's shard of F split this many ways")
    ap.add_argument("--cpu", action="store_true", help="also time torch CPU sparse.mm (F = 256 only)")
    args = ap.parse_args()

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
    from graph_convolutional_networks_for_text_classification_amd import datasets, ops, parallel
    from graph_convolutional_networks_for_text_classification_amd.sparse import CSR

    t0 = time.time()
    rp, ci, v = datasets.uniform_random_csr(args.nodes, args.edges, seed=0, device=dev)
    a = CSR(rp, ci, v, (args.nodes, args.nodes))
    M, K, nnz = args.nodes, args.nodes, a.nnz
    if rank == 0:
        print(json.dumps({"graph": "uniform", "nodes": M, "nnz": nnz, "build_s": round(time.time() - t0, 1),
                          "world": world}), flush=True)

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        s = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = None
        for _ in range(reps):
            e0.record(s)
            fn()
            e1.record(s)
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return best

    for F in [int(x) for x in args.F.split(",")]:
        parts = world if world > 1 else args.shard_of
        sh = parallel.ColumnShardedSpMM(a, F) if world > 1 else None
        c0, c1 = sh.columns if sh else parallel.shard_bounds(F, parts, 0)
        Fl = c1 - c0
        g = torch.Generator(device=dev).manual_seed(1 + rank)
        B = torch.randn(K, Fl, device=dev, generator=g)
        out = torch.empty(M, sh.width if sh else Fl, device=dev)
        view = out[:, :Fl]
        ms = timed(lambda: ops.spmm(a, B, out=view), args.reps)
        if world > 1:
            t = torch.tensor([ms], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ms = float(t.item())
        alg = 4 * (M + 1) + 8 * nnz + 4 * K * Fl + 4 * M * Fl
        gat = 4 * (M + 1) + 8 * nnz + 4 * nnz * Fl + 4 * M * Fl
        rec = {"case": f"uniform_1M_20M_F{F}", "columns_per_rank": Fl, "ranks": parts, "ms_spmm": round(ms, 4),
               "edges_per_s": nnz / (ms * 1e-3), "gflops": 2 * nnz * Fl / (ms * 1e-3) / 1e9,
               "alg_GBs": alg / (ms * 1e-3) / 1e9, "alg_frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
               "gather_GBs": gat / (ms * 1e-3) / 1e9, "dtype": "f32"}
        if world > 1:
            blk = out
            msg = timed(lambda: sh.gather(blk), args.reps)
            t = torch.tensor([msg], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            msg = float(t.item())
            rec.update({"ms_allgather": round(msg, 4), "allgather_recv_GBs_per_rank":
                        (world - 1) * M * sh.width * 4 / (msg * 1e-3) / 1e9,
                        "whole_job_edges_per_s": nnz * world / ((ms + msg) * 1e-3)})
        if rank == 0:
            print(json.dumps(rec), flush=True)
        del B, out, view
        torch.cuda.empty_cache()

    if args.cpu and rank == 0:
        tc = torch.sparse_csr_tensor(rp.long().cpu(), ci.long().cpu(), v.cpu(), (M, K))
        Bc = torch.randn(K, 256)
        t1 = time.time()
        torch.sparse.mm(tc, Bc)
        s = time.time() - t1
        print(json.dumps({"case": "uniform_1M_20M_F256", "impl": "torch CPU sparse.mm (CSR)",
                          "threads": torch.get_num_threads(), "ms_spmm": round(s * 1e3, 1),
                          "edges_per_s": nnz / s}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
