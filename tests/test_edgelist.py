"""CPU tests of the native edge-list loader (gcnk_edgelist_*): the reference's
graph file (build_graph.py:199, nx.write_weighted_edgelist) -> the symmetric
float32 adjacency trainer.py:98-148 builds with networkx.  Host code only: no
GPU needed.  networkx (the reference's own loader) is the checker where it is
importable."""
import numpy as np
import pytest

import gcn_amd  # noqa: F401
from graph_convolutional_networks_for_text_classification_amd import _lib, datasets
from oracle import csr_ref


def _write(path, lines):
    path.write_text("\n".join(lines) + "\n")
    return str(path)


def _dense(rp, ci, v, n):
    out = np.zeros((n, n), np.float32)
    for r in range(n):
        out[r, ci[rp[r]:rp[r + 1]]] = v[rp[r]:rp[r + 1]]
    return out


def test_small_file_semantics(tmp_path):
    p = _write(tmp_path / "g.txt", [
        "# comment", "0 1 0.5", "", "1 2 0.25", "2 0 1e-3",
        "1 0 0.75",            # same undirected edge: the last weight wins
        "3 3 2.0",             # self loop, stored once
        "   2 3 0.1"])
    rp, ci, v = datasets.load_edgelist(p)
    want = np.zeros((4, 4), np.float32)
    for u, w_, x in [(0, 1, 0.75), (1, 2, 0.25), (2, 0, 1e-3), (3, 3, 2.0), (2, 3, 0.1)]:
        want[u, w_] = want[w_, u] = np.float32(x)
    np.testing.assert_array_equal(_dense(rp, ci, v, 4), want)
    assert all(np.all(np.diff(ci[rp[r]:rp[r + 1]]) > 0) for r in range(4)), "sorted, duplicate-free rows"


def test_matches_networkx_adjacency(tmp_path):
    nx = pytest.importorskip("networkx")
    rng = np.random.default_rng(3)
    n = 300
    lines = [f"{u} {w} {rng.random()!r}" for u, w in zip(rng.integers(0, n, 2000), rng.integers(0, n, 2000))]
    lines += [f"{i} {(i + 1) % n} 0.5" for i in range(n)]      # every id present
    p = _write(tmp_path / "g.txt", lines)
    rp, ci, v = datasets.load_edgelist(p)
    G = nx.read_weighted_edgelist(p, nodetype=int)
    A = nx.adjacency_matrix(G, nodelist=list(range(G.number_of_nodes())), weight="weight", dtype=np.float32)
    A = A.tocsr()
    A.sort_indices()
    assert np.array_equal(rp, A.indptr) and np.array_equal(ci, A.indices)
    assert np.array_equal(v.view(np.uint32), A.data.astype(np.float32).view(np.uint32))


def test_r8_adjacency_round_trip(tmp_path, r8):
    """R8's raw adjacency written the way build_graph.py:199 writes it (each
    undirected edge once) loads back bit for bit."""
    rows, cols, vals = r8["a_rows"], r8["a_cols"], np.asarray(r8["a_vals"], np.float32)
    up = rows < cols
    p = _write(tmp_path / "R8_topic.txt",
               [f"{u} {w} {float(x)!r}" for u, w, x in zip(rows[up], cols[up], vals[up])])
    rp, ci, v = datasets.load_edgelist(p)
    wrp, wci, wv = csr_ref.coo_to_csr(rows, cols, vals, (r8["nodes"], r8["nodes"]))
    assert np.array_equal(rp, wrp) and np.array_equal(ci, wci)
    assert np.array_equal(v, wv.astype(np.float32))


def test_errors(tmp_path):
    with pytest.raises(_lib.GcnkError, match="not contiguous"):
        datasets.load_edgelist(_write(tmp_path / "a.txt", ["0 2 1.0"]))
    with pytest.raises(_lib.GcnkError, match="expected"):
        datasets.load_edgelist(_write(tmp_path / "b.txt", ["0 1 1.0", "0 x 2"]))
    with pytest.raises(_lib.GcnkError, match="cannot open"):
        datasets.load_edgelist(str(tmp_path / "missing.txt"))
    # a huge node id is refused before anything is sized by it
    with pytest.raises(_lib.GcnkError, match="too large"):
        datasets.load_edgelist(_write(tmp_path / "c.txt", ["0 1 1.0", "1 1000000000000 1.0"]))
