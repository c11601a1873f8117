"""Where the first R8 forward of a fresh process spends its time (bench.py runs
this as a child process and puts the JSON line it prints into setup_ms).

Runs, in a new process, the steps the module's first eval forward takes
(trainer.py:341-347 moves the COO tensors to the device, trainer.py:382 calls
the forward) one at a time, synchronising after each, so each one-time cost is
measured by itself:

  import_torch_ms / import_package_ms   Python imports (CPU)
  cuda_init_ms        torch's HIP context (first device tensor)
  model_h2d_ms        GCN(...).to(dev) and the COO tensors to the device
  lib_load_ms         dlopen of libgcnk.so + ctypes binding (_lib.load)
  first_launch_ms     the library's first kernel launch (a 4-float copy)
  coo_to_csr_adj_ms   A-hat COO -> CSR (gcnk_coo_to_csr, first use: its module)
  coo_to_csr_x_ms     X COO -> CSR (+ the dense-operand check)
  factor_build_ms     the hub factor's U and A_H records (factor.get)
  record_ms           the launch record: SpMM plans (host build + upload), scratch
  forward_ms          the first forward's launches (first use of their kernels)
  second_forward_ms   the next forward (steady-state eager call)

`--direct` instead times only the first forward as one step (what
bench.py's first_forward_fresh_process_ms measures) after the same imports,
context and transfers, for the sum check."""
import time

T0 = time.perf_counter()
import argparse  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import sys  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--direct", action="store_true")
    args = ap.parse_args()
    out = {}
    t = time.perf_counter()
    import torch
    out["import_torch_ms"] = (time.perf_counter() - t) * 1e3

    def step(name, fn):
        if name != "cuda_init_ms":   # (the context does not exist before that step)
            torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        out[name] = round((time.perf_counter() - t) * 1e3, 3)
        return r

    t = time.perf_counter()
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import GCN, _lib, datasets, factor, ops, record
    from graph_convolutional_networks_for_text_classification_amd.sparse import as_csr
    out["import_package_ms"] = round((time.perf_counter() - t) * 1e3, 3)
    r8 = datasets.load_r8_fixture(os.path.join(ROOT, "tests", "golden", "r8_graph.npz"))
    dev = torch.device("cuda", 0)
    step("cuda_init_ms", lambda: torch.zeros(1, device=dev))

    def h2d():
        torch.manual_seed(0)
        m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5).to(dev).eval()
        return m, r8["features"].to(dev), r8["adj"].to(dev)
    m, x, adj = step("model_h2d_ms", h2d)
    if args.direct:
        with torch.no_grad():
            step("first_forward_ms", lambda: m(x, adj))
        out["total_since_start_ms"] = round((time.perf_counter() - T0) * 1e3, 3)
        print(json.dumps(out), flush=True)
        return
    lib = step("lib_load_ms", _lib.load)
    src = torch.zeros(4, device=dev)
    dst = torch.empty(4, device=dev)
    step("first_launch_ms", lambda: _lib.check(lib.gcnk_stream_copy_f32(
        src.data_ptr(), dst.data_ptr(), 4, torch.cuda.current_stream().cuda_stream), "gcnk_stream_copy_f32"))
    a_csr = step("coo_to_csr_adj_ms", lambda: as_csr(adj))
    xop = step("coo_to_csr_x_ms", lambda: ops.Operand(x))
    step("factor_build_ms", lambda: ops.factor_for(a_csr, xop))
    W1 = m.gc1.weight
    step("record_ms", lambda: record.get(a_csr, xop, W1.shape[1], m.gc2.weight.shape[1], dev))
    with torch.no_grad():
        step("forward_ms", lambda: m(x, adj))
        step("second_forward_ms", lambda: m(x, adj))
    out["path"] = record.KIND_NAMES.get(record.get(a_csr, xop, W1.shape[1], m.gc2.weight.shape[1], dev)[0].kind)
    out["factored"] = factor.get(a_csr, xop) is not None
    out["library_bytes"] = os.path.getsize(_lib.LIB_PATH)
    out["total_since_start_ms"] = round((time.perf_counter() - T0) * 1e3, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
