"""Benchmark of the hot path: the R8 two-layer GCN forward on MI355X.

`python bench.py --gpus N --steps K --warmup W` prints ONE JSON line (rank 0).

Workload (BASELINE.json configs[1]): the R8 doc-topic graph exactly as the
reference prepares it (tests/golden/r8_graph.npz, written by the reference's
own builder and PrepareData in the build container; 7,724 nodes, Â nnz
69,130, X nnz 756,850, nfeat 7,463), 2-layer GCN hidden 200, 8 classes,
random-init weights (torch.manual_seed(0), the reference init), eval mode.
A step = one full GCN forward (X·W1, Â·S1 + bias + ReLU, H1·W2, Â·S2 + bias),
replayed from a hipGraph with all inputs resident in HBM; --graph-steps
forwards are captured per graph (every one a complete forward), so exactly
--steps forwards run in the timed region.

metric/value: SpMM edges/s = (2 · nnz(Â) per forward — the two graph
aggregations of layer.py:106) × steps × ranks / max-over-ranks time;
ms_per_step = GCN-forward ms (hipGraph replay); eager_forward_us = the same
forward issued eagerly, one call per step as trainer.py:357 does.  N > 1: the R8 graph does not shard (SURVEY
§8(e)): N independent replicas, "scaling": "weak".

roofline (the north-star op, BASELINE.json: R8 doc-topic SpMM Â·S1 at hidden
200 with gc1's bias + ReLU fused): algorithmic bytes (CSR SpMM:
4(M+1) + 8 nnz + 4 K F + 4 M F = 12.94 MB) over the kernel's average duration.
"frac" is the COLD figure: back-to-back launches that rotate
over enough distinct B / C sets (> 256 MB) that no launch finds its operands
in the Infinity Cache; "frac_warm" repeats one set.  The duration is the
kernel time of a child rocprofv3 --kernel-trace --stats run of those
rotations (scripts/hub_probe.py --mode; keep the summaries with
--rocprof-dir), so "frac" follows from the committed rocprof summary;
"hip_events" holds the same rotations timed with HIP events on the launching
stream (per call, hipGraph) -- those also hold the ~1.5-2 us dispatch gap
between launches.  Without rocprofv3 the HIP-event figure is used
("duration_source" says which).  "traffic" is measured live: two child
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; FETCH doubled per the gfx950
correction of MI355X_MICROARCH.md) over scripts/pmc_ops.py, per launch of the
op's kernels; null if rocprofv3 is unavailable.  "ops" gives the same warm /
cold figures for every op of the forward; "roofline_dominant" the slowest.

cpu_baseline: the oracle (torch-CPU restatement issuing the reference's
th.spmm calls on the same COO tensors, layer.py:102,106) on this host's
cores, bounded sample, at the job's thread share (OMP_NUM_THREADS), at 1
thread, and ("all_cores") in a child process pinned to one logical CPU per
physical core with one bound OpenMP thread each, with nproc and the CPU model; "cpu_stock_csr" is torch CSR sparse.mm (MKL) on the same host, and
"gpu_stock" stock PyTorch-ROCm torch.sparse.mm (hipSPARSE) on the device.

configs: BASELINE configs 3 (20ng-shaped doc-topic graph, hidden 200, 20
classes, gensim-shaped X) and 4 (uniform 1M nodes / 20M edges, F = 256), plus
config 4's power-law variant (R-MAT(0.57, 0.19, 0.19), 2^20 nodes, 20M edges
drawn) as extra keys: edges/s, GFLOP/s, the algorithmic
fraction, and for the 1M-node graphs the gather-rate fraction (nnz F 4 B of
row pieces over the guide's 5.5 TB/s random-row gather rate).  Each carries the
north_star's baselines beside it: "cpu_baseline" (the reference's th.spmm on
its COO layout, utils.py:196-203 -- the oracle's forward for config 3 -- at the
job's thread share and at 1 thread, >= 30 calls on config 3, 3 on config 4),
"cpu_stock_csr" (torch CSR sparse.mm, MKL) and "gpu_stock" (torch.sparse.mm on
the device, hipSPARSE).

setup_ms.first_forward_breakdown: scripts/first_forward.py in fresh child
processes -- the first forward's one-time costs step by step (library load,
first launch, COO -> CSR, hub factor, launch record, first launches).
"""
import argparse
import csv
import glob
import json
import os
import platform
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3   # dense fp32-input MFMA (= the fp32 vector rate), MI355X_MICROARCH.md
MALL_BYTES = 256 * 1024 * 1024


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
    ap.add_argument("--cpu-sample-s", type=float, default=8.0, help="seconds per CPU baseline leg (0 = skip)")
    ap.add_argument("--kernel-reps", type=int, default=200, help="launches per op-timing graph")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 --pmc traffic passes")
    ap.add_argument("--no-configs", action="store_true", help="skip BASELINE configs 3 and 4")
    ap.add_argument("--no-rmat", action="store_true", help="skip config 4's R-MAT (power-law) variant")
    ap.add_argument("--no-rmat-cpu", action="store_true", help="skip the CPU legs on the R-MAT graph (~40 s)")
    ap.add_argument("--no-train", action="store_true", help="skip the training-step and setup legs")
    ap.add_argument("--no-rocprof", action="store_true", help="skip the child rocprofv3 kernel-trace runs")
    ap.add_argument("--rocprof-dir", default=None, help="keep the child kernel-trace summaries here")
    ap.add_argument("--config5", action="store_true",
                    help="run the config-5 column-sharded leg even on one rank (it runs by default when N > 1)")
    ap.add_argument("--cpu-child", default=None, help=argparse.SUPPRESS)   # internal: the pinned CPU leg
    ap.add_argument("--dry-run", action="store_true",
                    help="print each rank's launch view (rank, world) as JSON and exit before any GPU call")
    return ap.parse_args()


def launch_ranks(args):
    """`--gpus N` (N > 1) outside a torch.distributed launcher: start the N rank
    processes as ONE child (python -m torch.distributed.run, one process per GPU,
    rendezvous on 127.0.0.1) and return its exit code.  Runs before anything
    touches the GPU; the parent never execs and never initialises HIP."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def upload_graph(graph):
    """hipGraphUpload of a captured graph's executable on torch's current
    stream, so no replay (least of all a timed one) pays the lazy upload."""
    import ctypes
    import torch
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        hip.hipGraphUpload(ctypes.c_void_p(graph.raw_cuda_graph_exec()),
                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
    except (OSError, AttributeError, RuntimeError):
        pass


def graph_us(fns, reps_per_fn):
    """Average us per call of a hipGraph replaying fns round-robin (HIP events
    on torch's current stream, the stream every op is launched on)."""
    import torch
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
    torch.cuda.synchronize()
    return best


def cpu_info():
    model = platform.processor()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "model": model}


def timed_cpu(fn, budget_s):
    fn()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s or n < 3:
        fn()
        n += 1
    return (time.perf_counter() - t0) / n, n


def timed_cpu_n(fn, n, warm=0):
    """Median seconds per call of fn over exactly n timed calls (after `warm`
    untimed ones), and every call's time: the CPU legs of the big configs,
    where one call takes seconds."""
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2], [round(t, 4) for t in ts]


# The random-row gather rate MI355X_MICROARCH.md measures for whole rows of a
# buffer far larger than the Infinity Cache, gathered into registers: 5.5-5.6
# TB/s for 1,152-B rows, 5.7-5.8 TB/s for 2,304-B rows (guide line 357).  A
# uniform-random SpMM at F = 256 gathers one 1 KB row piece of B per nonzero, so
# its bound is that rate, not the HBM peak against algorithmic bytes.
GATHER_RATE_GBS = 5550.0


def spmm_cpu_legs(rp, ci, v, shape, F, threads, iters, seed=0):
    """The synthetic configs' CPU and stock-GPU lines (BASELINE.md
    §3; north_star: "alongside the reference's scipy/torch.sparse CPU path timed on
    the same box's host cores"): C = A B for one [K x F] B of this config,
      cpu_baseline  the reference's call, th.spmm on the COO tensor laid out as
                    utils.py:196-203 hands it (column-major, uncoalesced:
                    datasets.reference_coo; layer.py:106), at the job's thread
                    share and at 1 thread;
      cpu_stock_csr torch CPU sparse.mm on a CSR tensor (MKL), same two thread counts;
    each the median of `iters` timed calls (plus one untimed call for the CSR
    leg), with the host's CPU model and nproc."""
    import torch
    from graph_convolutional_networks_for_text_classification_amd import datasets
    M, K = shape
    nnz = int(ci.numel())
    g = torch.Generator().manual_seed(seed)
    B = torch.randn(K, F, generator=g)
    coo = datasets.reference_coo(rp, ci, v, shape)
    csr = torch.sparse_csr_tensor(rp.cpu().long(), ci.cpu().long(), v.cpu(), shape)
    saved = torch.get_num_threads()
    out = {"cpu_baseline": {}, "cpu_stock_csr": {}}
    try:
        for th in sorted({threads, 1}, reverse=True):
            torch.set_num_threads(th)
            t, runs = timed_cpu_n(lambda: torch.spmm(coo, B), iters)
            out["cpu_baseline"][f"threads_{th}"] = {"s_per_spmm": round(t, 4), "runs_s": runs,
                                                     "edges_per_s": nnz / t, "gflops": 2 * nnz * F / t / 1e9}
            t, runs = timed_cpu_n(lambda: torch.sparse.mm(csr, B), iters, warm=1)
            out["cpu_stock_csr"][f"threads_{th}"] = {"s_per_spmm": round(t, 4), "runs_s": runs,
                                                      "edges_per_s": nnz / t, "gflops": 2 * nnz * F / t / 1e9}
    finally:
        torch.set_num_threads(saved)
    out["cpu_baseline"].update({"kind": "port", "unit": "edges/s", "cores": threads, "iterations": iters,
                                "value": out["cpu_baseline"][f"threads_{threads}"]["edges_per_s"],
                                "impl": "th.spmm on the reference-layout COO tensor (utils.py:196-203, "
                                        "layer.py:106), torch CPU", **cpu_info()})
    out["cpu_stock_csr"].update({"unit": "edges/s", "cores": threads, "iterations": iters,
                                 "value": out["cpu_stock_csr"][f"threads_{threads}"]["edges_per_s"],
                                 "impl": "torch CPU sparse.mm on a CSR tensor (MKL)"})
    return out


def gpu_stock_spmm(rp, ci, v, shape, B, iters=5):
    """Stock PyTorch-ROCm: torch.sparse.mm on a device CSR tensor (hipSPARSE),
    the same product; HIP events, best of `iters` after one untimed call."""
    import torch
    nnz = int(ci.numel())
    a = torch.sparse_csr_tensor(rp.long(), ci.long(), v, shape, device=B.device)
    torch.sparse.mm(a, B)
    torch.cuda.synchronize()
    best = None
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.sparse.mm(a, B)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    F = B.shape[1]
    del a
    return {"ms_spmm": round(best, 4), "edges_per_s": nnz / (best * 1e-3), "gflops": 2 * nnz * F / (best * 1e-3) / 1e9,
            "unit": "edges/s", "value": nnz / (best * 1e-3),
            "impl": "PyTorch-ROCm torch.sparse.mm on a device CSR tensor (hipSPARSE), best of %d" % iters}


def big_spmm_config(name, rp, ci, v, n, F, dev, ops, cpu_threads, cpu_iters, build_s):
    """One 1M-node synthetic config at width F on this GPU: the product path
    (ops.spmm, plan built untimed), best of 5 HIP-event timings, edges/s, GFLOP/s,
    the algorithmic-roofline fraction and the gather-rate fraction (nnz F 4 B of
    row pieces over the guide's random-row gather rate), the heaviest row, then
    the stock-GPU and CPU lines of the same product."""
    import torch
    from graph_convolutional_networks_for_text_classification_amd.sparse import CSR
    big = CSR(rp, ci, v, (n, n))
    g = torch.Generator(device=dev).manual_seed(7)
    Bb = torch.randn(n, F, device=dev, generator=g)
    Cb = torch.empty(n, F, device=dev)
    t0 = time.time()
    ops.spmm(big, Bb, out=Cb)
    torch.cuda.synchronize()
    plan_s = time.time() - t0
    best = None
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.spmm(big, Bb, out=Cb)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    nb = spmm_bytes(n, n, big.nnz, F)
    gathered = 4 * big.nnz * F
    deg = rp[1:] - rp[:-1]
    res = {"nodes": n, "nnz": big.nnz, "F": F, "max_row_nnz": int(deg.max()), "ms_spmm": round(best, 4),
           "edges_per_s": big.nnz / (best * 1e-3), "gflops": 2 * big.nnz * F / (best * 1e-3) / 1e9,
           "frac": nb / (best * 1e-3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": nb,
           "gather_bytes": gathered, "gather_gbs": gathered / (best * 1e-3) / 1e9,
           "gather_frac": gathered / (best * 1e-3) / 1e9 / GATHER_RATE_GBS,
           "gather_rate_ref": "MI355X_MICROARCH.md: 5.5-5.6 TB/s random 1,152-B rows gathered into registers "
                              "(%.0f GB/s used)" % GATHER_RATE_GBS,
           "graph_build_s": round(build_s, 1), "plan_build_s": round(plan_s, 2),
           "note": "B (%.1f GB) and C exceed the 256 MB Infinity Cache: every launch is cold" % (4 * n * F / 1e9)}
    hdr = big.plan(ops.default_ipc(big, F), int(ops._lib.load().gcnk_spmm_groups(F, 0))).header
    res["plan"] = {"ipc": hdr[4], "row_units": hdr[5], "heavy_segments": hdr[6], "multi_segment_rows": hdr[7],
                   "partial_slots": hdr[14]}
    try:
        res["gpu_stock"] = gpu_stock_spmm(rp, ci, v, (n, n), Bb)
    except RuntimeError as e:   # reported, never fatal to the bench line
        res["gpu_stock"] = {"error": str(e)[:300]}
    del big, Bb, Cb
    torch.cuda.empty_cache()
    if cpu_iters > 0:
        res.update(spmm_cpu_legs(rp.cpu(), ci.cpu(), v.cpu(), (n, n), F, cpu_threads, cpu_iters))
    return res


def first_forward_breakdown():
    """scripts/first_forward.py in a fresh child process: the first R8 forward's
    one-time costs step by step (library load, first launch, COO -> CSR, hub
    factor, launch record / plans, the first launches), and the same first
    forward as one step (--direct) in another fresh process."""
    out = {}
    for key, extra in (("steps", []), ("direct", ["--direct"])):
        try:
            r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "first_forward.py")] + extra, cwd=ROOT,
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=300)
            line = [ln for ln in r.stdout.decode(errors="replace").splitlines() if ln.startswith("{")]
            out[key] = json.loads(line[-1]) if r.returncode == 0 and line else {"error": f"rc={r.returncode}"}
        except (OSError, subprocess.SubprocessError, ValueError) as e:
            out[key] = {"error": str(e)[:200]}
    return out


def pmc_traffic(op, kernels_like, detail=None):
    """HBM-side bytes per launch of the op's kernels from child rocprofv3 --pmc
    passes, one counter each (FETCH_SIZE x 2 per the gfx950 correction +
    WRITE_SIZE), and the L1 -> L2 read requests (TCP_TCC_READ_REQ_sum, 128 B
    each on gfx950) in a third pass; `detail` (a dict) receives the per-counter
    figures."""
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not on PATH"
    tmp = tempfile.mkdtemp(prefix="gcnk_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    per = {}
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE", "TCP_TCC_READ_REQ_sum"):
            out = os.path.join(tmp, counter)
            cmd = ["timeout", "-s", "KILL", "120", exe, "--pmc", counter, "--output-format", "csv", "-d", out,
                   "-o", "run", "--", sys.executable, os.path.join(ROOT, "scripts", "pmc_ops.py"), "--op", op,
                   "--reps", "10"]
            r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=150)
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {counter} rc={r.returncode}"
            vals = {}
            for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                for row in csv.DictReader(open(f)):
                    name = row["Kernel_Name"]
                    if any(k in name for k in kernels_like):
                        vals.setdefault(name, []).append(float(row["Counter_Value"]))
            if not vals:
                return None, f"no {counter} rows for {kernels_like}"
            # per launch of the op: sum over its kernels of the mean per dispatch
            # (FETCH_SIZE / WRITE_SIZE in KiB, the request count as is)
            per[counter] = sum(sum(v) / len(v) for v in vals.values()) * (1 if counter.startswith("TCP") else 1024)
        if detail is not None:
            detail.update({"fetch_bytes_x2": 2 * per["FETCH_SIZE"], "write_bytes": per["WRITE_SIZE"],
                           "l2_read_req": per["TCP_TCC_READ_REQ_sum"],
                           "l2_read_bytes": 128 * per["TCP_TCC_READ_REQ_sum"]})
        return 2 * per["FETCH_SIZE"] + per["WRITE_SIZE"], "live rocprofv3 --pmc (FETCH_SIZE x2 + WRITE_SIZE)"
    except (OSError, subprocess.SubprocessError, KeyError, ValueError) as e:
        return None, f"pmc pass failed: {e}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def rocprof_kernel_us(mode, kernels_like, save_dir=None, variant="row"):
    """Average kernel duration (us) of the north-star op's kernels from a child
    rocprofv3 --kernel-trace --stats run of scripts/hub_probe.py (the same op,
    the same warm / cold rotation as the HIP-event figure), so the reported
    fraction can be checked against a rocprof summary of the same launches."""
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not on PATH"
    tmp = tempfile.mkdtemp(prefix="gcnk_kt_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        cmd = ["timeout", "-s", "KILL", "150", exe, "--kernel-trace", "--stats", "--output-format", "csv", "-d", tmp,
               "-o", "kt", "--", sys.executable, os.path.join(ROOT, "scripts", "hub_probe.py"), "--reps", "200",
               "--variants", variant, "--widths", "200", "--mode", mode]
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=180)
        if r.returncode != 0:
            return None, f"rocprofv3 --kernel-trace rc={r.returncode}"
        files = glob.glob(os.path.join(tmp, "**", "*kernel_stats.csv"), recursive=True)
        total, found = 0.0, False
        for f in files:
            for row in csv.DictReader(open(f)):
                if any(k in row["Name"] for k in kernels_like):
                    total += float(row["AverageNs"]) / 1e3
                    found = True
            if save_dir:
                os.makedirs(save_dir, exist_ok=True)
                tag = mode if variant != "copy" else "copyfloor"
                shutil.copy(f, os.path.join(save_dir, f"bench_rocprof_as1_{tag}_kernel_stats.csv"))
        if not found:
            return None, f"no kernel rows for {kernels_like}"
        return total, f"rocprofv3 --kernel-trace --stats, scripts/hub_probe.py --mode {mode}"
    except (OSError, subprocess.SubprocessError, KeyError, ValueError) as e:
        return None, f"kernel trace failed: {e}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _factored(a_csr, x):
    """The HubFactor the product forward uses for (A-hat, X), or None (SpMM path)."""
    from graph_convolutional_networks_for_text_classification_amd import ops
    return ops.factor_for(a_csr, ops.Operand(x))


def forward_kernels(save_dir=None, graph="r8"):
    """Per-kernel durations of the product forward (hipGraph replay) from a child
    rocprofv3 --kernel-trace run of scripts/fwd_trace.py, in launch order."""
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not on PATH"
    tmp = tempfile.mkdtemp(prefix="gcnk_fwd_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp", GCNK_TRACE_GRAPH=graph)
    try:
        cmd = ["timeout", "-s", "KILL", "150", exe, "--kernel-trace", "--stats", "--output-format", "csv", "-d", tmp,
               "-o", "fwd", "--", sys.executable, os.path.join(ROOT, "scripts", "fwd_trace.py")]
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=180)
        if r.returncode != 0:
            return None, f"rocprofv3 --kernel-trace rc={r.returncode}"
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import fwd_trace
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            res = fwd_trace.report(tmp)
        if save_dir:
            os.makedirs(save_dir, exist_ok=True)
            for f in glob.glob(os.path.join(tmp, "**", "*kernel_stats.csv"), recursive=True):
                shutil.copy(f, os.path.join(save_dir, f"bench_forward_{graph}_kernel_stats.csv"))
        return res, "rocprofv3 --kernel-trace, scripts/fwd_trace.py (hipGraph of 10 forwards, 20 replays)"
    except (OSError, subprocess.SubprocessError, KeyError, ValueError, ImportError) as e:
        return None, f"forward trace failed: {e}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def forward_path(a_csr, x, nhid, nclass):
    """The record kind the product forward takes for (A-hat, X): "dense-ax"
    (ops.dense_ax_for), "factored" (ops.factor_for), "spmm+proj" or "spmm+gemm"."""
    from graph_convolutional_networks_for_text_classification_amd import ops
    xop = ops.Operand(x)
    if ops.dense_ax_for(a_csr, xop, nhid, nclass) is not None:
        return "dense-ax"
    if ops.factor_for(a_csr, xop) is not None:
        return "factored"
    fused = ops.FUSE_PROJECTION and nclass <= ops.FUSE_MAX_P and nhid % 4 == 0 and nhid <= 256
    return "spmm+proj" if fused else "spmm+gemm"


def labelled_forward_kernels(save_dir, graph, a_csr, x, N, nfeat, nnz_a, nnz_x, nhid, nclass):
    """forward_kernels() with each launch labelled by the op it belongs to and
    that op's algorithmic bytes (SURVEY §8(d) formulas: every operand read once,
    every output written once) and fraction of the HBM peak."""
    trace, trace_src = forward_kernels(save_dir, graph)
    if trace is None or not trace.get("kernels"):
        return {"error": trace_src}
    from graph_convolutional_networks_for_text_classification_amd import ops
    dense_x = ops.Operand(x).dense is not None
    path = forward_path(a_csr, x, nhid, nclass)
    a_s2 = spmm_bytes(N, N, nnz_a, nclass)
    flops = {}   # the MFMA-bound ops' useful fp32 FLOPs (fraction of the fp32 MFMA peak beside the HBM one)
    if path == "dense-ax":
        # one launch: A-hat X [N x nfeat] (cached), W1, b1, W2 read; S2 written
        alg = {"AX W1 + H1 W2": 4 * (N * nfeat + nfeat * nhid + nhid + nhid * nclass + N * nclass), "A S2": a_s2}
        flops = {"AX W1 + H1 W2": 2 * N * (nfeat * nhid + nhid * nclass)}
    elif path == "factored":
        fac = _factored(a_csr, x)
        # X[hubs] W1 (dense hub rows on the one-pass small-M GEMM, or their CSR),
        # then one launch reading U [N x Kc], the A_H records, W1[Kc], S_T, W2, writing S2
        xw = 4 * (fac.H * nfeat + nfeat * nhid + fac.H * nhid) if fac.x_hub_dense is not None \
            else spmm_bytes(fac.H, nfeat, fac.x_hub.nnz, nhid)
        alg = {"X_hubs W1": xw,
               "A X W1 factored + H1 W2": (4 * fac.U.numel() + 4 * fac.rec.numel() + 4 * fac.Kc * nhid
                                            + 4 * fac.H * nhid + 4 * nhid * nclass + 4 * N * nclass),
               "A S2": a_s2}
        flops = {"X_hubs W1": 2 * fac.H * nfeat * nhid,
                 "A X W1 factored + H1 W2": 2 * N * (fac.Kc * nhid + nhid * nclass)
                 + 2 * nhid * (fac.rec.numel() - 68 * fac.nblk) // 2}   # (+ the A_H items: 2 words each)
    else:
        fused = path == "spmm+proj"
        alg = {   # dense X (gensim-shaped): the GEMM's operands once; sparse X: the CSR SpMM formula
            "X W1": 4 * (N * nfeat + nfeat * nhid + N * nhid) if dense_x else spmm_bytes(N, nfeat, nnz_x, nhid),
            # gc2's support fused into the gc1 aggregation: it writes S2 [N x nclass];
            # unfused it writes H1 [N x nhid] and the skinny GEMM reads it back
            "A S1": (4 * (N + 1) + 8 * nnz_a + 4 * N * nhid + 4 * N * nclass + 4 * nhid * nclass) if fused
            else spmm_bytes(N, N, nnz_a, nhid),
            "A S2": a_s2,
            "H1 W2": 4 * (N * nhid + nhid * nclass + N * nclass)}
    ks, na = [], 0
    for k in trace["kernels"]:   # launch order: the A-hat launches are the row kernels
        name = k["kernel"]
        if path == "dense-ax":
            key = "A S2" if "spmm_row_kernel" in name else "AX W1 + H1 W2"
        elif path == "factored":
            key = ("A X W1 factored + H1 W2" if ("hubfactor" in name or "dense_gc1" in name)
                   else "A S2" if "spmm_row_kernel" in name else "X_hubs W1")
        elif "spmm_row_kernel" in name:
            key = "A S1" if na == 0 else "A S2"
            na += 1
        else:
            key = "H1 W2" if na > 0 else "X W1"   # (the skinny GEMM sits between the two aggregations)
        ks.append({"kernel": name[:120], "us": k["us"], "op": key})
    for key, nb in alg.items():   # per op: its launches' summed duration against its bytes
        us = sum(e["us"] for e in ks if e["op"] == key)
        for e in ks:
            if e["op"] == key:
                e.update({"op_us": round(us, 3), "algorithmic_bytes": nb,
                          "frac": nb / (us * 1e-6) / 1e9 / HBM_PEAK_GBS if us > 0 else None})
                if key in flops and us > 0:
                    e.update({"flops": flops[key], "tflops": flops[key] / (us * 1e-6) / 1e12,
                              "mfma_frac": flops[key] / (us * 1e-6) / 1e12 / FP32_MFMA_PEAK_TFLOPS})
    per_op = {}
    for e in ks:
        per_op.setdefault(e["op"], {"op_us": e.get("op_us"), "algorithmic_bytes": e.get("algorithmic_bytes"),
                                    "frac": e.get("frac"), "tflops": e.get("tflops"), "mfma_frac": e.get("mfma_frac"),
                                    "kernels": []})["kernels"].append(e["kernel"][:60])
    return {"source": trace_src, "path": path, "x_operand": "dense" if dense_x else "csr",
            "forward_span_us": trace["forward_span_us_median"], "kernels": ks, "ops": per_op}


def factor_build_ms(a_csr, x):
    """Fresh device builds of the hub factorisation of (A-hat, X) (factor.build,
    csrc/factor_build.hip: the one-time setup the first forward pays, like the
    CSR plans): {"first_ms", "ms"} -- the first in this process (module load
    included) and the median of three more; None when the operands do not
    factor."""
    import torch
    from graph_convolutional_networks_for_text_classification_amd import factor, ops
    xop = ops.Operand(x)
    ts = []
    for _ in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f = factor.build(a_csr, xop)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        if f is None:
            return None
    return {"first_ms": round(ts[0], 2), "ms": round(sorted(ts[1:])[1], 2)}


def train_step_legs(r8, dev, steps=30):
    """The training step of trainer.py:349-362 on R8 (model.train(), zero_grad,
    forward, cross-entropy on the training nodes, backward, Adam): eager with the
    reference's CPU dropout masks (the default: a seeded run trains on the
    reference's own masks), eager with the in-kernel hash masks, and the latter
    captured once in a hipGraph and replayed (capturable Adam; the hash offset
    lives on the device, so every replay draws a fresh mask -- checked)."""
    import torch
    from graph_convolutional_networks_for_text_classification_amd import GCN
    x, adj = r8["features"].to(dev), r8["adj"].to(dev)
    tgt = torch.as_tensor(r8["target"]).long().to(dev)
    idx = torch.as_tensor(r8["train_lst"]).long().to(dev)
    crit = torch.nn.CrossEntropyLoss()
    res = {}
    for rng in ("cpu", "device"):
        torch.manual_seed(0)
        model = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5, dropout_rng=rng).to(dev)
        opt = torch.optim.Adam(model.parameters(), lr=0.02)

        def step():
            model.train()
            opt.zero_grad()
            loss = crit(model(x, adj)[idx], tgt[idx])
            loss.backward()
            opt.step()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        # host-bound: the median of 5 timed runs (one run swung 0.38 -> 0.52 ms
        # between boxes with the same build)
        runs = []
        for _ in range(5):
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            runs.append(round((time.perf_counter() - t0) / steps * 1e3, 4))
        res[f"eager_{rng}_masks_ms"] = sorted(runs)[len(runs) // 2]
        res[f"eager_{rng}_masks_runs_ms"] = runs
    torch.manual_seed(0)
    model = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5, dropout_rng="device").to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.02, capturable=True)
    model.train()

    def gstep():
        opt.zero_grad(set_to_none=False)
        loss = crit(model(x, adj)[idx], tgt[idx])
        loss.backward()
        opt.step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            gstep()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gstep()
    g.replay()
    torch.cuda.synchronize()
    base0 = int(model._rng_base.item())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        g.replay()
    e1.record()
    e1.synchronize()
    res["graph_device_masks_ms"] = round(e0.elapsed_time(e1) / steps, 4)
    res["graph_fresh_masks"] = (int(model._rng_base.item()) - base0) // (r8["nodes"] * 200) == steps
    res["steps"] = steps
    res["note"] = ("trainer.py:354-362 per step; eager = one Python step per call as the reference's loop runs it "
                   "(median of 5 runs of `steps`); "
                   "graph = the same step (hash masks) replayed from one hipGraph")
    del g
    torch.cuda.synchronize()
    return res


def setup_legs(r8, dev, nhid=200):
    """One-time cost of each forward path in this (warm) process: a fresh copy
    of the R8 tensors (no cached CSR, plans, factor or launch record), then one
    eval forward, synchronised -- COO -> CSR, the SpMM plans, the hub factor
    (factored path) and the launch record, plus the forward itself."""
    import torch
    from graph_convolutional_networks_for_text_classification_amd import GCN, ops
    out = {}
    saved = ops.FACTOR_GC1
    try:
        for path, flag in (("factored", True), ("spmm", False)):
            ops.FACTOR_GC1 = flag
            ts = []
            for _ in range(3):
                torch.manual_seed(0)
                m = GCN(nfeat=r8["nfeat"], nhid=nhid, nclass=r8["nclass"], dropout=0.5).to(dev).eval()
                x, adj = r8["features"].to(dev).clone(), r8["adj"].to(dev).clone()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                with torch.no_grad():
                    m(x, adj)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
                del m, x, adj
            out[path] = {"setup_ms": round(sorted(ts)[1], 3), "runs_ms": [round(t, 3) for t in ts]}
    finally:
        ops.FACTOR_GC1 = saved
    return out


def dense_ax_build_ms(a_csr, x, nhid, nclass):
    """Fresh builds of the narrow-feature path's one-time operand A-hat X
    (ops.dense_ax_for: gcnk_aggregate_f32, float64 row sums rounded once):
    {"first_ms", "ms"} as factor_build_ms; None where the path does not apply."""
    import torch
    from graph_convolutional_networks_for_text_classification_amd import ops
    xop = ops.Operand(x)
    ts = []
    for _ in range(4):
        if hasattr(a_csr, "_dense_ax"):
            a_csr._dense_ax.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d = ops.dense_ax_for(a_csr, xop, nhid, nclass)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        if d is None:
            return None
    return {"first_ms": round(ts[0], 3), "ms": round(sorted(ts[1:])[1], 3)}


def sharded_config5(dev, world, rank, datasets, ops, F=4096, reps=3):
    """BASELINE config 5 on this job's ranks: the replicated 1M / 20M CSR, this
    rank's F / P columns of B, the local SpMM and the all-gather of the result
    (times are the max over ranks of the per-rep medians)."""
    import torch
    import torch.distributed as dist
    from graph_convolutional_networks_for_text_classification_amd.parallel import ColumnShardedSpMM
    from graph_convolutional_networks_for_text_classification_amd.sparse import CSR
    n, nnz = 1_000_000, 20_000_000
    err = None
    try:   # setup; every rank learns whether all ranks got through before any timed collective
        rp, ci, v = datasets.uniform_random_csr(n, nnz, seed=0, device=dev)
        a = CSR(rp, ci, v, (n, n))
        cs = ColumnShardedSpMM(a, F)
        c0, c1 = cs.columns
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        Bp = torch.randn((n, c1 - c0), generator=g, device=dev)
        blk = cs.local(Bp)           # plan build, untimed
        torch.cuda.synchronize()
        del blk
    except (RuntimeError, MemoryError) as e:
        err = str(e)[:300]
    ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=dev)
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok) == 0:
        return {"error": err or "another rank failed its setup"}
    try:
        cs.gather(cs.local(Bp))      # first all-gather, untimed
        torch.cuda.synchronize()
        t_loc, t_tot = [], []
        for _ in range(reps):
            if world > 1:
                dist.barrier(device_ids=[torch.cuda.current_device()])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            blk = cs.local(Bp)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            out = cs.gather(blk)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            t_loc.append(t1 - t0)
            t_tot.append(t2 - t0)
            del blk, out
        t = torch.tensor([sorted(t_loc)[reps // 2], sorted(t_tot)[reps // 2]], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        loc, tot = float(t[0]), float(t[1])
        res = {"nodes": n, "nnz": a.nnz, "F": F, "ranks": world, "columns_per_rank": cs.width,
               "ms_local_spmm": round(loc * 1e3, 3), "ms_all_gather": round((tot - loc) * 1e3, 3),
               "ms_total": round(tot * 1e3, 3), "edges_per_s": a.nnz / tot,
               "gflops": 2 * a.nnz * F / tot / 1e9, "gathered_bytes_per_rank": 4 * n * cs.width * world,
               "scaling": "strong", "collective": "RCCL all_gather_into_tensor" if world > 1 else "none (1 rank)"}
        del a, Bp, rp, ci, v
        torch.cuda.empty_cache()
        return res
    except (RuntimeError, MemoryError) as e:   # reported, never fatal to the bench line
        return {"error": str(e)[:300]}


def physical_cores():
    """One logical CPU per physical core among the CPUs this process may run on
    (sysfs topology), so a pinned leg runs one thread per core, no SMT siblings."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = list(range(os.cpu_count() or 1))
    seen, cores = set(), []
    for c in allowed:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            key = (open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip())
        except OSError:
            key = ("?", str(c))
        if key not in seen:
            seen.add(key)
            cores.append(c)
    return cores


def cpu_child(args):
    """The pinned all-cores CPU leg (a child of bench.py; never touches the GPU):
    the oracle forward on the R8 fixture with the parent's weights, timed for
    --cpu-sample-s seconds; prints one JSON line."""
    import torch
    import gcn_amd  # noqa: F401  (the package alias; loads no GPU code)
    from graph_convolutional_networks_for_text_classification_amd import datasets
    from oracle import gcn_ref
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    sd = torch.load(args.cpu_child, weights_only=True)
    ref = gcn_ref.RefGCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).eval()
    ref.load_state_dict(sd)
    with torch.no_grad():
        t, n = timed_cpu(lambda: ref(r8["features"], r8["adj"]), args.cpu_sample_s)
    print(json.dumps({"s_per_forward": t, "forwards": n, "threads": torch.get_num_threads()}), flush=True)


def pinned_cpu_leg(state_dict, sample_s):
    """Runs cpu_child in a child process restricted (before it starts any thread)
    to one logical CPU per physical core, with one OpenMP thread per core bound
    to it; returns (seconds per forward, forwards, cores) or None."""
    import torch
    cores = physical_cores()
    tmp = tempfile.mkdtemp(prefix="gcnk_cpu_", dir="/tmp")
    try:
        path = os.path.join(tmp, "sd.pt")
        torch.save({k: v.detach().cpu() for k, v in state_dict.items()}, path)
        env = dict(os.environ, OMP_NUM_THREADS=str(len(cores)), OMP_PROC_BIND="close", OMP_PLACES="cores",
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-child", path, "--cpu-sample-s",
                            str(sample_s)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           preexec_fn=lambda: os.sched_setaffinity(0, cores), timeout=sample_s * 10 + 120)
        line = [ln for ln in r.stdout.decode(errors="replace").splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not line:
            return None
        d = json.loads(line[-1])
        return d["s_per_forward"], d["forwards"], len(cores)
    except (OSError, subprocess.SubprocessError, ValueError, KeyError):
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def config3_baselines(g20, m20, a20, x20, ac20, sample_s):
    """BASELINE config 3 (the 20ng-shaped doc-topic graph) beside the product:
    the reference's forward on the host CPU (the oracle issuing layer.py's
    th.spmm calls on the same COO tensors, layer.py:102,106) at the job's thread
    share and at 1 thread, the same forward through torch CPU CSR sparse.mm
    (MKL), and through stock PyTorch-ROCm torch.sparse.mm (hipSPARSE) on the
    device; plus the north-star-shaped op alone (A-hat S at F = 200) on the
    reference's COO path.  >= 30 timed calls each (bounded by sample_s)."""
    import torch
    from oracle import gcn_ref
    threads = int(os.environ.get("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1))))
    nnz = ac20.nnz
    ref = gcn_ref.RefGCN(nfeat=g20["nfeat"], nhid=200, nclass=20, dropout=0.5).eval()
    ref.load_state_dict({k: v.cpu() for k, v in m20.state_dict().items()})
    xc, adc = g20["features"], g20["adj"]
    W1, b1, W2, b2 = (p.detach() for p in (m20.gc1.weight, m20.gc1.bias, m20.gc2.weight, m20.gc2.bias))
    Wc1, bc1, Wc2, bc2 = (p.cpu() for p in (W1, b1, W2, b2))
    xs, as_ = xc.coalesce().to_sparse_csr(), adc.coalesce().to_sparse_csr()
    S = torch.randn(adc.shape[0], 200, generator=torch.Generator().manual_seed(3))
    saved = torch.get_num_threads()
    fwd, csr, op = {}, {}, {}

    def budgeted(fn):
        fn()
        n, t0, ts = 0, time.perf_counter(), []
        while n < 30 or time.perf_counter() - t0 < sample_s / 4:
            t1 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t1)
            n += 1
            if time.perf_counter() - t0 > 4 * sample_s and n >= 30:
                break
        return sorted(ts)[len(ts) // 2], n
    try:
        with torch.no_grad():
            for th in sorted({threads, 1}, reverse=True):
                torch.set_num_threads(th)
                t, n = budgeted(lambda: ref(xc, adc))
                fwd[f"threads_{th}"] = {"ms_per_forward": round(t * 1e3, 3), "forwards": n,
                                        "edges_per_s": 2 * nnz / t}

                def csr_forward():
                    h = torch.relu(torch.sparse.mm(as_, torch.sparse.mm(xs, Wc1)) + bc1)
                    return torch.sparse.mm(as_, h @ Wc2) + bc2
                t, n = budgeted(csr_forward)
                csr[f"threads_{th}"] = {"ms_per_forward": round(t * 1e3, 3), "forwards": n,
                                        "edges_per_s": 2 * nnz / t}
                t, n = budgeted(lambda: torch.spmm(adc, S))
                op[f"threads_{th}"] = {"ms": round(t * 1e3, 3), "calls": n, "edges_per_s": nnz / t,
                                       "gflops": 2 * nnz * 200 / t / 1e9}
    finally:
        torch.set_num_threads(saved)
    xg, ag = x20.coalesce().to_sparse_csr(), a20.coalesce().to_sparse_csr()

    def stock_forward():
        with torch.no_grad():
            h = torch.relu(torch.sparse.mm(ag, torch.sparse.mm(xg, W1)) + b1)
            return torch.sparse.mm(ag, h @ W2) + b2
    stock_forward()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(30):
        stock_forward()
    e1.record()
    e1.synchronize()
    tg = e0.elapsed_time(e1) / 30 * 1e-3
    return {
        "cpu_baseline": {"value": fwd[f"threads_{threads}"]["edges_per_s"], "unit": "edges/s", "cores": threads,
                         "kind": "port", "ms_per_forward": fwd[f"threads_{threads}"]["ms_per_forward"],
                         "sample": "20ng-shaped eval forwards of the oracle (torch-CPU th.spmm on the reference COO "
                                   "tensors, layer.py:102,106), median", **fwd, **cpu_info(),
                         "spmm_F200_reference_coo": op},
        "cpu_stock_csr": {"value": csr[f"threads_{threads}"]["edges_per_s"], "unit": "edges/s", "cores": threads,
                          "ms_per_forward": csr[f"threads_{threads}"]["ms_per_forward"],
                          "impl": "torch CPU sparse.mm on CSR tensors (MKL), same forward", **csr},
        "gpu_stock": {"value": 2 * nnz / tg, "unit": "edges/s", "ms_per_forward": round(tg * 1e3, 4),
                      "impl": "PyTorch-ROCm torch.sparse.mm on CSR tensors (hipSPARSE), eager, same forward"}}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.dry_run:
        print(json.dumps({"rank": rank, "local_rank": local, "world": world}), flush=True)
        return
    if args.cpu_child:
        cpu_child(args)
        return
    import numpy as np
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)   # before the process group: RCCL binds each rank to its own GPU
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")

    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, datasets, ops
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr

    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    N, nfeat, nclass, nhid = r8["nodes"], r8["nfeat"], r8["nclass"], 200
    torch.manual_seed(0)
    model = GCN(nfeat=nfeat, nhid=nhid, nclass=nclass, dropout=0.5).to(dev).eval()
    adj = r8["adj"].to(dev)
    x = r8["features"].to(dev)

    def forward():
        with torch.no_grad():
            return model(x, adj)

    # the first forward of a fresh process: module load, COO -> CSR, plans, the
    # factored operands and the launch record (one-time), then the forward
    torch.cuda.synchronize()
    tf = time.perf_counter()
    out = forward()
    torch.cuda.synchronize()
    first_forward_ms = (time.perf_counter() - tf) * 1e3
    a_csr, x_csr = as_csr(adj), as_csr(x)
    nnz_a, nnz_x = a_csr.nnz, x_csr.nnz
    fb_r8 = factor_build_ms(a_csr, x)
    if args.no_graph:
        step = forward
        per = 1
    else:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                forward()
        torch.cuda.current_stream().wait_stream(s)
        # the largest forwards-per-graph <= --graph-steps that divides --steps and
        # --warmup (every replay is `per` complete forwards, so exactly --steps run
        # timed and exactly --warmup untimed, the latter including a replay of the
        # same graph: its first launch pays one-time costs)
        per = max(1, min(args.graph_steps, args.steps))
        while args.steps % per or (args.warmup and args.warmup % per):
            per -= 1
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(per):
                out = forward()
        upload_graph(graph)
        step = graph.replay

    for _ in range(args.warmup // per):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(device_ids=[torch.cuda.current_device()])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps // per):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier(device_ids=[torch.cuda.current_device()])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)

    # ---- the forward as the reference's trainer issues it: eager calls, one
    #      model.forward per step (trainer.py:357,382), no graph -- host launch
    #      overhead included (synchronised once per 50 calls)
    for _ in range(5):
        forward()
    torch.cuda.synchronize()
    te = time.perf_counter()
    for _ in range(50):
        forward()
    torch.cuda.synchronize()
    eager_us = (time.perf_counter() - te) / 50 * 1e6

    # ---- per-op durations, warm and cold (rotating operand sets > the MALL)
    W1, b1 = model.gc1.weight.detach(), model.gc1.bias.detach()
    W2, b2 = model.gc2.weight.detach(), model.gc2.bias.detach()
    with torch.no_grad():
        S1 = ops.spmm(x_csr, W1)
        H1 = ops.spmm(a_csr, S1, bias=b1, epilogue=2)
        S2 = ops.gemm(H1, W2)
        Z = ops.spmm(a_csr, S2, bias=b2, epilogue=1)
    torch.cuda.synchronize()

    def rot(t, n):
        return [t.clone() for _ in range(n)]

    f4 = 4
    specs = {   # name: (bytes, per-set bytes, maker given the set count)
        "spmm_XW1": (spmm_bytes(N, nfeat, nnz_x, nhid), f4 * (nfeat * nhid + N * nhid),
                     lambda n: (rot(W1, n), rot(S1, n), lambda i, Ws, Ss: lambda: ops.spmm(x_csr, Ws[i], out=Ss[i]))),
        "spmm_AS1_F200": (spmm_bytes(N, N, nnz_a, nhid), f4 * 2 * N * nhid,
                          lambda n: (rot(S1, n), rot(H1, n), lambda i, Bs, Cs: lambda: ops.spmm(
                              a_csr, Bs[i], bias=b1, epilogue=2, out=Cs[i]))),
        "gemm_H1W2": (f4 * (N * nhid + nhid * nclass + N * nclass), f4 * (N * nhid + N * nclass),
                      lambda n: (rot(H1, n), rot(S2, n), lambda i, Hs, Ss: lambda: ops.gemm(Hs[i], W2, out=Ss[i]))),
        "spmm_AS2_F8": (spmm_bytes(N, N, nnz_a, nclass), f4 * 2 * N * nclass,
                        lambda n: (rot(S2, n), rot(Z, n), lambda i, Bs, Cs: lambda: ops.spmm(
                            a_csr, Bs[i], bias=b2, epilogue=1, out=Cs[i]))),
    }
    optimes = {}
    for name, (nbytes, set_bytes, maker) in specs.items():
        nsets = max(2, -(-int(1.25 * MALL_BYTES) // set_bytes))
        ins, outs, mk = maker(nsets)
        fns = [mk(i, ins, outs) for i in range(nsets)]
        warm = graph_us(fns[:1], args.kernel_reps)
        cold = graph_us(fns, max(1, args.kernel_reps // nsets))
        optimes[name] = {"warm_us": round(warm, 3), "cold_us": round(cold, 3), "sets": nsets,
                         "algorithmic_bytes": nbytes,
                         "frac_cold": nbytes / (cold * 1e-6) / 1e9 / HBM_PEAK_GBS,
                         "frac_warm": nbytes / (warm * 1e-6) / 1e9 / HBM_PEAK_GBS}
        del ins, outs, fns
        torch.cuda.empty_cache()
    north = "spmm_AS1_F200"   # BASELINE.json north_star: the R8 doc-topic SpMM at hidden 200
    dom = max(optimes, key=lambda k: optimes[k]["cold_us"])

    extras = rank == 0 and world == 1
    # ---- live HBM traffic of the north-star op (child rocprofv3 --pmc passes)
    traffic, traffic_src = (None, "skipped")
    traffic_detail = {}
    if extras and not args.no_pmc:
        traffic, traffic_src = pmc_traffic("AS1", ["spmm_row_kernel"], traffic_detail)
    # ---- the same op's kernel durations from rocprofv3 (warm and cold rotations)
    kt = {}
    if extras and not args.no_rocprof:
        for mode in ("warm", "cold"):
            kt[mode] = rocprof_kernel_us(mode, ["spmm_row_kernel"], args.rocprof_dir, "row")
        # the streaming floor at this size: one elementwise pass over the same B / C
        # rotation (reads B once, writes C once) under the same rocprofv3 timing
        kt["copy"] = rocprof_kernel_us("cold", ["stream_copy_kernel"], args.rocprof_dir, "copy")

    # ---- the product forward's own kernels (rocprofv3 trace of the graph replay),
    #      each against its algorithmic bytes; the fused north-star kernel among them
    fwd_k = None
    if extras and not args.no_rocprof:
        fwd_k = labelled_forward_kernels(args.rocprof_dir, "r8", a_csr, x, N, nfeat, nnz_a, nnz_x, nhid, nclass)

    # ---- CPU baselines (rank 0, N = 1): oracle at all cores and 1 thread, torch CSR (MKL)
    cpu = cpu_stock = gpu_stock = None
    if extras and args.cpu_sample_s > 0:
        from oracle import gcn_ref
        threads = int(os.environ.get("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1))))
        torch.manual_seed(0)
        ref = gcn_ref.RefGCN(nfeat=nfeat, nhid=nhid, nclass=nclass, dropout=0.5).eval()
        ref.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
        xc, ac = r8["features"], r8["adj"]
        legs = {}
        with torch.no_grad():
            for th in sorted({threads, 1}, reverse=True):
                torch.set_num_threads(th)
                tc, n = timed_cpu(lambda: ref(xc, ac), args.cpu_sample_s)
                legs[th] = (tc, n)
            torch.set_num_threads(threads)
            # best stock CPU: the same forward through torch CSR sparse.mm (MKL)
            xs, as_ = xc.coalesce().to_sparse_csr(), ac.coalesce().to_sparse_csr()
            Wc1, bc1, Wc2, bc2 = (p.detach().cpu() for p in (W1, b1, W2, b2))

            def csr_forward():
                h = torch.relu(torch.sparse.mm(as_, torch.sparse.mm(xs, Wc1)) + bc1)
                return torch.sparse.mm(as_, h @ Wc2) + bc2
            tm, nm = timed_cpu(csr_forward, args.cpu_sample_s / 2)
        tc, n = legs[threads]
        t1, n1 = legs[1]
        pinned = pinned_cpu_leg(model.state_dict(), args.cpu_sample_s)
        cpu = {"value": 2 * nnz_a / tc, "unit": "edges/s", "cores": threads, "kind": "port",
               "sample": f"{n} R8 eval forwards of the oracle (torch-CPU th.spmm on the reference COO tensors, "
                         f"layer.py:102,106), {tc * 1e3:.2f} ms/forward at {threads} threads",
               "ms_per_forward": tc * 1e3,
               "one_thread": {"value": 2 * nnz_a / t1, "ms_per_forward": t1 * 1e3, "forwards": n1},
               "all_cores": ({"threads": pinned[2], "pinned": "one OpenMP thread per physical core, bound",
                              "value": 2 * nnz_a / pinned[0], "ms_per_forward": pinned[0] * 1e3,
                              "forwards": pinned[1]} if pinned else None),
               **cpu_info()}
        cpu_stock = {"value": 2 * nnz_a / tm, "unit": "edges/s", "cores": threads, "ms_per_forward": tm * 1e3,
                     "impl": "torch CPU sparse.mm on CSR tensors (MKL), same forward", "forwards": nm}
        # stock GPU: PyTorch-ROCm torch.sparse.mm (hipSPARSE) for the same forward
        xg, ag = x.coalesce().to_sparse_csr(), adj.coalesce().to_sparse_csr()

        def stock_forward():
            with torch.no_grad():
                h = torch.relu(torch.sparse.mm(ag, torch.sparse.mm(xg, W1)) + b1)
                return torch.sparse.mm(ag, h @ W2) + b2
        stock_forward()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            stock_forward()
        e1.record()
        e1.synchronize()
        tg = e0.elapsed_time(e1) / 20 * 1e-3
        gpu_stock = {"value": 2 * nnz_a / tg, "unit": "edges/s", "ms_per_forward": tg * 1e3,
                     "impl": "PyTorch-ROCm torch.sparse.mm on CSR tensors (hipSPARSE), eager, same forward"}

    # ---- the training step (trainer.py:349-362) and each path's one-time setup
    train = setup = None
    if extras and not args.no_train:
        train = train_step_legs(r8, dev)
        setup = setup_legs(r8, dev)
        setup["first_forward_fresh_process_ms"] = round(first_forward_ms, 3)
        setup["first_forward_breakdown"] = first_forward_breakdown()

    # ---- BASELINE configs 3 and 4 (bounded)
    configs = None
    if extras and not args.no_configs:
        configs = {}
        g20 = datasets.doc_topic_graph(18846, 70, 20, seed=0)
        torch.manual_seed(1)
        m20 = GCN(nfeat=g20["nfeat"], nhid=200, nclass=20, dropout=0.5).to(dev).eval()
        a20, x20 = g20["adj"].to(dev), g20["features"].to(dev)
        ac20 = as_csr(a20)

        def fwd20():
            with torch.no_grad():   # inference, as the R8 line (trainer.py:382 runs eval under no_grad)
                return m20(x20, a20)
        fwd20()
        us_fwd = graph_us([fwd20], 50)
        fk20 = None if args.no_rocprof else labelled_forward_kernels(
            args.rocprof_dir, "20ng", ac20, x20, ac20.shape[0], g20["nfeat"], ac20.nnz, as_csr(x20).nnz, 200, 20)
        fb20 = factor_build_ms(ac20, x20)
        dab20 = dense_ax_build_ms(ac20, x20, 200, 20)
        # the same forward on the reference's CPU path and on stock PyTorch-ROCm
        legs20 = {}
        if args.cpu_sample_s > 0:
            legs20 = config3_baselines(g20, m20, a20, x20, ac20, args.cpu_sample_s)
        M20 = ac20.shape[0]
        bb = torch.randn(200, device=dev)
        nsets = max(2, -(-int(1.25 * MALL_BYTES) // (2 * 4 * M20 * 200)))
        Bs = [torch.randn(M20, 200, device=dev) for _ in range(nsets)]
        Cs = [torch.empty(M20, 200, device=dev) for _ in range(nsets)]
        fns = [(lambda i=i: ops.spmm(ac20, Bs[i], bias=bb, epilogue=2, out=Cs[i])) for i in range(nsets)]
        w = graph_us(fns[:1], 100)
        c = graph_us(fns, max(1, 100 // nsets))
        del Bs, Cs, fns
        nb = spmm_bytes(ac20.shape[0], ac20.shape[0], ac20.nnz, 200)
        configs["20ng_shaped"] = {
            "nodes": ac20.shape[0], "adj_nnz": ac20.nnz, "forward_us": round(us_fwd, 3),
            "edges_per_s": 2 * ac20.nnz / (us_fwd * 1e-6),
            "spmm_F200_warm_us": round(w, 3), "spmm_F200_cold_us": round(c, 3),
            "spmm_F200_frac_cold": nb / (c * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "spmm_F200_frac_warm": nb / (w * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "spmm_F200_gflops_cold": 2 * ac20.nnz * 200 / (c * 1e-6) / 1e9,
            "path": forward_path(ac20, x20, 200, 20), "factor_build_ms": fb20, "dense_ax_build_ms": dab20,
            "forward_kernels": fk20, **legs20}
        del m20, a20, x20, ac20
        torch.cuda.empty_cache()
        threads = int(os.environ.get("OMP_NUM_THREADS", str(min(16, os.cpu_count() or 1))))
        cpu_iters = 3 if args.cpu_sample_s > 0 else 0
        tb = time.time()
        rp, ci, v = datasets.uniform_random_csr(1_000_000, 20_000_000, seed=0, device=dev)
        configs["uniform_1M_20M_F256"] = big_spmm_config("uniform", rp, ci, v, 1_000_000, 256, dev, ops, threads,
                                                         cpu_iters, time.time() - tb)
        del rp, ci, v
        torch.cuda.empty_cache()
        if not args.no_rmat:
            # SURVEY §8(d) row 4's power-law variant, reported separately: R-MAT(0.57,
            # 0.19, 0.19), 2^20 nodes, 20M edges drawn (rows of up to ~45k nonzeros)
            tb = time.time()
            rp, ci, v = datasets.rmat_csr(20, 20_000_000, seed=0, device=dev)
            configs["rmat_1M_20M_F256"] = big_spmm_config("rmat", rp, ci, v, 1 << 20, 256, dev, ops, threads,
                                                          0 if args.no_rmat_cpu else cpu_iters, time.time() - tb)
            configs["rmat_1M_20M_F256"]["generator"] = "datasets.rmat_csr(20, 20_000_000, a=0.57, b=0.19, c=0.19, seed=0)"
            del rp, ci, v
            torch.cuda.empty_cache()

    # ---- BASELINE config 5 (N > 1): 1M nodes / 20M edges, F = 4096 feature
    #      columns sharded over the ranks (parallel.ColumnShardedSpMM: local
    #      SpMM, then one RCCL all-gather of the [M, F/P] blocks over xGMI);
    #      total work fixed ("strong"), max over ranks
    config5 = None
    if (world > 1 or args.config5) and not args.no_configs:
        config5 = sharded_config5(dev, world, rank, datasets, ops)

    ms = elapsed / args.steps * 1e3
    value = 2 * nnz_a * args.steps * world / elapsed
    kn, kd = optimes[north], optimes[dom]
    # the slowest op of the product forward as it runs (its own launches in the
    # rocprofv3 trace, against that op's algorithmic bytes); the unfused per-op
    # timings above only when no trace is available
    dominant = {"op": dom, "frac": kd["frac_cold"], "frac_warm": kd["frac_warm"], "avg_launch_us": kd["cold_us"],
                "algorithmic_bytes": kd["algorithmic_bytes"], "source": "ops (unfused per-op timing, cold)"}
    if fwd_k and fwd_k.get("ops"):
        op, d = max(fwd_k["ops"].items(), key=lambda kv: kv[1]["op_us"] or 0.0)
        dominant = {"op": op, "kernels": d["kernels"], "frac": d["frac"], "avg_launch_us": d["op_us"],
                    "algorithmic_bytes": d["algorithmic_bytes"], "path": fwd_k.get("path"),
                    "source": "forward_kernels: the product forward's own launches (rocprofv3 trace)"}
    # the north-star kernel's average launch duration: the cold rocprofv3 kernel
    # time of the child run (so "frac" follows from the committed rocprof
    # summary); the HIP-event per-call figure, which also holds the dispatch gap
    # between back-to-back launches (~1.5-2 us), beside it
    nb = kn["algorithmic_bytes"]
    kcold, kwarm = kt.get("cold", (None, "")), kt.get("warm", (None, ""))
    dur, dur_w, src = kn["cold_us"], kn["warm_us"], "HIP events per call (hipGraph of back-to-back launches)"
    if kcold[0] is not None and kwarm[0] is not None:
        dur, dur_w, src = kcold[0], kwarm[0], kcold[1]
    roof = {"bound": "hbm", "kernel": north, "plan": "row",
            "achieved": nb / (dur * 1e-6) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": nb / (dur * 1e-6) / 1e9 / HBM_PEAK_GBS, "frac_warm": nb / (dur_w * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "traffic": traffic, "traffic_source": traffic_src, "traffic_detail": traffic_detail or None,
            "avg_launch_us": round(dur, 3), "avg_launch_us_warm": round(dur_w, 3), "duration_source": src,
            "hip_events": {"avg_call_us": kn["cold_us"], "avg_call_us_warm": kn["warm_us"],
                           "frac": kn["frac_cold"], "frac_warm": kn["frac_warm"]},
            "algorithmic_bytes": nb}
    line = {
        "metric": "SpMM edges/s and GCN-forward ms on R8 doc-topic graph, 1×MI355X",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "eager_forward_us": round(eager_us, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "R8 graph fixture generated in-container by the reference's own builder; random-init weights",
        "config": {"workload": "R8 GCN forward (eval), hidden 200, 8 classes, nfeat 7463",
                   "nodes": N, "adj_nnz": nnz_a, "x_nnz": nnz_x, "graph": not args.no_graph,
                   "forwards_per_graph": per,
                   "path": forward_path(a_csr, x, nhid, nclass),
                   "factor_build_ms": fb_r8,
                   "parallelism": f"replicas{world}" if world > 1 else "single"},
        "roofline": roof,
        # the same op under rocprofv3: kernel time without the dispatch gap that the
        # per-call HIP-event figure above includes
        "roofline_rocprof": {m: ({"kernel_us": round(v[0], 3),
                                  "frac": kn["algorithmic_bytes"] / (v[0] * 1e-6) / 1e9 / HBM_PEAK_GBS,
                                  "source": v[1],
                                  **({"note": "streaming floor: one float4 copy C = B (gcnk_stream_copy_f32) over "
                                              "the same cold B / C rotation (no CSR, no gathers); frac = the op's "
                                              "bytes at that duration, the ceiling of any single launch at this size"}
                                     if m == "copy" else {})} if v[0] is not None else {"error": v[1]})
                             for m, v in kt.items()},
        "roofline_dominant": dominant,
        "forward_kernels": fwd_k,
        "train_step_ms": train,
        "setup_ms": setup,
        "ops": optimes,
        "cpu_baseline": cpu,
        "cpu_stock_csr": cpu_stock,
        "gpu_stock": gpu_stock,
        "configs": configs,
        "config5_column_sharded": config5,
    }
    if rank == 0:
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
