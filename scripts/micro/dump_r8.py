"""Dump R8 A-hat (the reference-built fixture tests/golden/r8_graph.npz) as a
sorted int32 CSR binary for the standalone HIP microbenchmarks:
int32 M, int32 nnz, int32 rowptr[M + 1], int32 colind[nnz], float32 val[nnz]."""
import sys

import numpy as np


def main(out):
    z = np.load("tests/golden/r8_graph.npz")
    r, c, v = z["adj_row"].astype(np.int64), z["adj_col"].astype(np.int64), z["adj_val"]
    M = int(z["shape"][0])
    order = np.lexsort((c, r))
    r, c, v = r[order], c[order], v[order]
    rp = np.zeros(M + 1, np.int32)
    np.add.at(rp, r + 1, 1)
    rp = np.cumsum(rp).astype(np.int32)
    with open(out, "wb") as f:
        np.array([M, len(c)], np.int32).tofile(f)
        rp.tofile(f)
        c.astype(np.int32).tofile(f)
        v.astype(np.float32).tofile(f)
    print(f"wrote {out}: M={M} nnz={len(c)}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/r8_adj.bin")
