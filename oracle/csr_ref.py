"""ORACLE (test infrastructure only): float64 numpy restatement from the math.

Kernel-level checkers for arbitrary inputs (any graph, any F), written from
the operations the reference calls:
  spmm_csr        C = A @ B          (th.spmm(adj, support), layer.py:106)
  spmm_epilogue   + bias, relu, dropout multiply  (layer.py:110,182,185)
  coo_to_csr      sum duplicates, row-major order (what th.spmm sees after coalescing)
  csr_transpose   A^T (stable), operand of the autograd of layer.py:102/106
  gemm / colsum   dense products and bias gradients
Results are float64; tests compare the fp32 HIP outputs against them with an
explicit tolerance.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")


def coo_to_csr(rows, cols, vals, shape):
    M, K = shape
    rows = np.asarray(rows, np.int64)
    cols = np.asarray(cols, np.int64)
    vals = np.asarray(vals, np.float64)
    key = rows * K + cols
    order = np.argsort(key, kind="stable")
    key, vals = key[order], vals[order]
    uniq, start = np.unique(key, return_index=True)
    summed = np.add.reduceat(vals, start) if len(vals) else vals
    r = uniq // K
    c = uniq % K
    rowptr = np.zeros(M + 1, np.int64)
    np.add.at(rowptr, r + 1, 1)
    return np.cumsum(rowptr), c.astype(np.int64), summed


def csr_transpose(rowptr, colind, val, shape):
    M, K = shape
    rows = np.repeat(np.arange(M), np.diff(rowptr))
    order = np.lexsort((rows, colind))  # by column, then source row
    rp = np.zeros(K + 1, np.int64)
    np.add.at(rp, np.asarray(colind)[order] + 1, 1)
    return np.cumsum(rp), rows[order], np.asarray(val)[order]


def spmm_csr(rowptr, colind, val, B, M=None):
    """float64 C = A @ B for CSR A.  Uses the C oracle when built, else numpy."""
    rowptr = np.asarray(rowptr, np.int64)
    M = len(rowptr) - 1 if M is None else M
    B = np.ascontiguousarray(B, np.float64)
    lib = _load_c()
    if lib is not None:
        F = B.shape[1]
        out = np.zeros((M, F), np.float64)
        rp = np.ascontiguousarray(rowptr, np.int64)
        ci = np.ascontiguousarray(colind, np.int64)
        v = np.ascontiguousarray(val, np.float64)
        lib.oracle_spmm_csr_f64(rp.ctypes.data, ci.ctypes.data, v.ctypes.data, M, B.ctypes.data, F,
                                out.ctypes.data)
        return out
    rows = np.repeat(np.arange(M), np.diff(rowptr))
    out = np.zeros((M, B.shape[1]), np.float64)
    np.add.at(out, rows, np.asarray(val, np.float64)[:, None] * B[np.asarray(colind)])
    return out


def spmm_epilogue(acc, bias=None, relu=False, mask=None, scale=1.0):
    out = np.array(acc, np.float64)
    if bias is not None:
        out = out + np.asarray(bias, np.float64)[None, :]
    if relu:
        out = np.maximum(out, 0.0)
    if mask is not None:
        out = np.where(np.asarray(mask) != 0, out * scale, 0.0)
    return out


def gemm(A, B, transA=False, transB=False):
    A = np.asarray(A, np.float64)
    B = np.asarray(B, np.float64)
    return (A.T if transA else A) @ (B.T if transB else B)


def colsum(X):
    return np.asarray(X, np.float64).sum(0)


_lib = None


def _load_c():
    global _lib
    if _lib is None and os.path.exists(LIB_PATH):
        lib = ctypes.CDLL(LIB_PATH)
        lib.oracle_spmm_csr_f64.restype = None
        lib.oracle_spmm_csr_f64.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                            ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        lib.oracle_spmm_csr_f32.restype = None
        lib.oracle_spmm_csr_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                            ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        _lib = lib
    return _lib


def spmm_csr_f32_seq(rowptr, colind, val, B):
    """fp32 sequential-accumulation CSR SpMM in C (a scalar CPU 'port' of the
    SpMM, used as a CPU baseline timing leg and for fp32 error bounds)."""
    lib = _load_c()
    if lib is None:
        raise RuntimeError("oracle/liboracle.so not built (run __graft_entry__.build())")
    rp = np.ascontiguousarray(rowptr, np.int64)
    ci = np.ascontiguousarray(colind, np.int64)
    v = np.ascontiguousarray(val, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    M = len(rp) - 1
    out = np.zeros((M, B.shape[1]), np.float32)
    lib.oracle_spmm_csr_f32(rp.ctypes.data, ci.ctypes.data, v.ctypes.data, M, B.ctypes.data, B.shape[1],
                            out.ctypes.data)
    return out
