"""CPU checks of the C-ABI boundary: the library loads, exports every symbol
include/gcnk.h declares, and validates arguments (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

import gcn_amd  # noqa: F401
from graph_convolutional_networks_for_text_classification_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "gcnk.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gcnk_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    declared = _declared_symbols()
    assert len(declared) >= 14
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_lib.SIGNATURES), "ctypes signatures out of sync with include/gcnk.h"


MAGIC = 0x474E4B35  # plan header word 0 ("GNK5")


def _hdr(M=10, K=10, groups=1, ipc=32, nslots=0, nslabs=0):
    # magic M K groups ipc nunits nhunits nheavy ntile nred nslabs ntblk has_diag nnz nslots 0
    h = (ctypes.c_int32 * 16)(MAGIC, M, K, groups, ipc, 0, 0, 0, 0, 0, nslabs, 0, 0, 0, nslots, 0)
    return ctypes.cast(h, ctypes.c_void_p), h


def test_abi_version_and_error_text():
    lib = _lib.load()
    assert lib.gcnk_abi_version() == _lib.ABI_VERSION == 12
    rc = lib.gcnk_spmm_csr_f32(None, None, None, 0, 8, None, 0, None, 0, None, 0,
                               1.0, 1.0, 0, 0, None, None, 0, None, 0, 0, None)
    assert rc == _lib.EARG
    assert b"bad argument" in lib.gcnk_last_error()
    with pytest.raises(_lib.GcnkError):
        _lib.check(rc, "spmm")


def test_argument_validation_without_gpu():
    lib = _lib.load()
    # leading dimension too small
    rc = lib.gcnk_gemm_f32(0, 0, 4, 4, 4, ctypes.c_void_p(16), 2, ctypes.c_void_p(16), 4, ctypes.c_void_p(16), 4,
                           None, 0, None, 0, 1.0, 1, None, 0, None)
    assert rc == _lib.EARG
    # split-K without workspace
    rc = lib.gcnk_gemm_f32(0, 0, 4, 4, 4096, ctypes.c_void_p(16), 4096, ctypes.c_void_p(16), 4,
                           ctypes.c_void_p(16), 4, None, 0, None, 0, 1.0, 8, None, 0, None)
    assert rc == _lib.EARG
    # plan build without operands
    rc = lib.gcnk_spmm_plan_build(ctypes.c_void_p(16), None, None, 10, 10, 100, 8, 4, 0.25, ctypes.c_void_p(16),
                                  4, None)
    assert rc == _lib.EARG
    # a header that is not a plan's is refused
    bad = (ctypes.c_int32 * 16)()
    rc = lib.gcnk_spmm_csr_f32(ctypes.c_void_p(16), ctypes.cast(bad, ctypes.c_void_p), ctypes.c_void_p(16), 8, 8,
                               ctypes.c_void_p(16), 8, None, 0, None, 0, 1.0, 1.0, 0, 0, None, None, 0, None, 0, 0, None)
    assert rc == _lib.EARG and b"not a gcnk plan" in lib.gcnk_last_error()
    # plan/groups mismatch is refused before any launch (F=200 uses 1 lane group per wave)
    h, _keep = _hdr(groups=7)
    rc = lib.gcnk_spmm_csr_f32(ctypes.c_void_p(16), h, ctypes.c_void_p(16), 200, 200,
                               ctypes.c_void_p(16), 200, None, 0, None, 0, 1.0, 1.0, 0, 0, None, None, 0, None, 0, 0, None)
    assert rc == _lib.EARG and b"groups" in lib.gcnk_last_error()
    # workspace too small for the plan's partial slots
    h, _keep = _hdr(groups=1, nslots=3)
    rc = lib.gcnk_spmm_csr_f32(ctypes.c_void_p(16), h, ctypes.c_void_p(16), 200, 200,
                               ctypes.c_void_p(16), 200, None, 0, None, 0, 1.0, 1.0, 0, 0, None, None, 0, None, 0, 0, None)
    assert rc == _lib.EARG and b"workspace" in lib.gcnk_last_error()
    # empty problems are no-ops that succeed without touching the device
    h, _keep = _hdr(M=0)
    assert lib.gcnk_spmm_csr_f32(ctypes.c_void_p(16), h, None, 8, 8, None, 8, None,
                                 0, None, 0, 1.0, 1.0, 0, 0, None, None, 0, None, 0, 0, None) == _lib.OK
    assert lib.gcnk_gemm_f32(0, 0, 0, 5, 5, None, 5, None, 5, None, 5, None, 0, None, 0, 1.0, 1, None, 0,
                             None) == _lib.OK


def test_plan_and_workspace_sizes():
    lib = _lib.load()
    # lane groups per wavefront = 64 / lanes per row group
    assert lib.gcnk_spmm_groups(200, 0) == 1 and lib.gcnk_spmm_groups(8, 0) == 32 and lib.gcnk_spmm_groups(64, 0) == 4
    assert lib.gcnk_spmm_groups(7, 0) == 8 and lib.gcnk_spmm_groups(200, 16) == 4 and lib.gcnk_spmm_groups(200, 32) == 2
    h, _keep = _hdr(nslots=10, nslabs=3)
    assert lib.gcnk_spmm_workspace_bytes(h, 198) == 8192 + 3 * 64 * 208 * 4
    assert lib.gcnk_gemm_workspace_bytes(200, 8, 7724, 4) == 4 * 200 * 8 * 4
    assert lib.gcnk_colsum_workspace_bytes(7724, 200) == ((7724 + 63) // 64) * 200 * 4
    # heavy-segment size follows the operand at 64 lanes (R8 12, 20ng-shaped 32); narrow groups:
    # 16 with workgroup-wide heavy segments (2+ lanes, round 5), 8 for 1-lane groups
    assert lib.gcnk_spmm_default_ipc(7724, 69130, 200, 0) == 12
    assert lib.gcnk_spmm_default_ipc(18916, 174674, 200, 0) == 32
    assert lib.gcnk_spmm_default_ipc(1000000, 19999805, 256, 0) == 32
    assert lib.gcnk_spmm_default_ipc(7724, 69130, 8, 0) == 16
    assert lib.gcnk_spmm_default_ipc(7724, 69130, 4, 0) == 8


def test_product_path_refuses_cpu_tensors(r8):
    """No silent CPU fallback: CPU inputs raise instead of computing."""
    import torch
    from graph_convolutional_networks_for_text_classification_amd import GCN
    torch.manual_seed(0)
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        m(r8["features"], r8["adj"])


def test_forward_record_layout_and_validation():
    """gcnk_gcn_forward_f32's record: the ctypes mirror matches the C layout, and
    incomplete records are refused before any launch (no GPU needed)."""
    from graph_convolutional_networks_for_text_classification_amd import record
    lib = _lib.load()
    assert record.layout_ok()
    p = ctypes.c_void_p(16)
    args = (p, None, p, None, p, 8, None, 0, _lib.EPI_BIAS_RELU, None, 0, 1.0, 1.0, 0, 0, None, None)
    assert lib.gcnk_gcn_forward_f32(None, *args) == _lib.EARG
    r = record.GcnFwd()
    r.kind, r.M, r.F, r.P = record.FACTORED, 10, 16, 8
    r.s1, r.s2, r.aP.plan, r.x_dense = 16, 16, 16, 16
    assert lib.gcnk_gcn_forward_f32(ctypes.byref(r), *args) == _lib.EARG   # factored without U / records
    assert b"missing an operand" in lib.gcnk_last_error()
    r.kind = record.SPMM_PROJ                                                # no F-wide plan
    assert lib.gcnk_gcn_forward_f32(ctypes.byref(r), *args) == _lib.EARG
    r.kind = 9
    r.aF.plan = 16
    assert lib.gcnk_gcn_forward_f32(ctypes.byref(r), *args) == _lib.EARG
    assert b"unknown record kind" in lib.gcnk_last_error()


def test_backward_record_validation():
    """gcnk_gcn_backward_f32 refuses a null or incomplete record before any
    launch (no GPU needed)."""
    from graph_convolutional_networks_for_text_classification_amd import record
    lib = _lib.load()
    p = ctypes.c_void_p(16)
    args = (p, p, 200, p, 1.0, p, None, None, None, None)
    assert lib.gcnk_gcn_backward_f32(None, *args) == _lib.EARG
    r = record.GcnBwd()
    r.M, r.F, r.P = 10, 200, 8
    r.aTP.plan, r.gS2, r.gZ1 = 16, 16, 16
    assert lib.gcnk_gcn_backward_f32(ctypes.byref(r), *args) == _lib.EARG   # gW1 wanted, no A^T / X^T plan
    assert b"incomplete record" in lib.gcnk_last_error()
    r.aTF.plan, r.gS1 = 16, 16
    assert lib.gcnk_gcn_backward_f32(ctypes.byref(r), *args) == _lib.EARG   # neither X^T plan nor dense X
    r.M = 0
    assert lib.gcnk_gcn_backward_f32(ctypes.byref(r), p, p, 200, p, 1.0, None, None, p, None, None) == _lib.EARG
