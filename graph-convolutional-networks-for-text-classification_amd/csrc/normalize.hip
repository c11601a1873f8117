// Device-side adjacency preparation:
//   Â = D^-1/2 (A + I) D^-1/2,   D = rowsum(A + I)
// Replaces the reference's host-side preprocess_adj / normalize_adj
// (utils.py:185-213, scipy) for graphs that live on the GPU.  Arithmetic is
// the reference's, so the result is bit-for-bit its fp32 COO values:
//   * A + I in float64 (sp.eye is float64, utils.py:188): an existing
//     diagonal entry gets + 1, a missing one is inserted at its sorted place;
//   * rowsum in float64, summed in column order (scipy's CSR row sum);
//     d = rowsum^-0.5 with inf -> 0 (utils.py:209-210);
//   * value(r, c) = (d[r] * a) * d[c] in float64 -- what
//     adj.dot(D).transpose().dot(D) evaluates for a symmetric A
//     (utils.py:212) -- rounded to fp32 once (utils.py:198).
// Input: a SYMMETRIC A as CSR with sorted, duplicate-free columns per row
// (what sparse.from_torch produces from the reference's COO).  The kernels do
// not check either property (that would need a host sync per call):
// sparse.preprocess_adj validates both once and raises, since an unsorted row
// misplaces the inserted diagonal and a non-symmetric A gets D A D where the
// reference computes D A^T D.  Output: CSR of Â, capacity nnz + n; its row
// pointer's last word is the output nnz.
#include "gcnk_common.h"

#include <hipcub/hipcub.hpp>

namespace gcnk {
namespace {

// One thread per row: output count (deg + 1 unless the diagonal exists) and d[r].
__global__ void norm_rows_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colind,
                                 const float* __restrict__ val, int32_t n, int32_t* __restrict__ counts,
                                 double* __restrict__ d) {
  const int32_t r = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r > n) return;
  if (r == n) {  // the scan's last element: 0, so rowptr_out[n] = total
    counts[n] = 0;
    return;
  }
  const int32_t b = rowptr[r], e = rowptr[r + 1];
  double s = 0.0;
  bool placed = false;  // the identity's 1 is in the sum
  bool has = false;     // A has a diagonal entry
  for (int32_t k = b; k < e; ++k) {
    const int32_t c = colind[k];
    if (!placed && c > r) {  // the identity's entry sits before the first larger column
      s += 1.0;
      placed = true;
    }
    double a = (double)val[k];
    if (c == r) {
      a += 1.0;
      placed = has = true;
    }
    s += a;
  }
  if (!placed) s += 1.0;
  counts[r] = (e - b) + (has ? 0 : 1);
  const double p = pow(s, -0.5);
  d[r] = isinf(p) ? 0.0 : p;
}

// One thread per row: entries in column order with the diagonal inserted.
__global__ void norm_fill_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colind,
                                 const float* __restrict__ val, int32_t n, const int32_t* __restrict__ rowptr_out,
                                 const double* __restrict__ d, int32_t* __restrict__ colind_out,
                                 float* __restrict__ val_out) {
  const int32_t r = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r >= n) return;
  const int32_t b = rowptr[r], e = rowptr[r + 1];
  int32_t o = rowptr_out[r];
  const double dr = d[r];
  bool placed = false;
  for (int32_t k = b; k < e; ++k) {
    const int32_t c = colind[k];
    if (!placed && c > r) {
      colind_out[o] = r;
      val_out[o++] = (float)((dr * 1.0) * dr);
      placed = true;
    }
    double a = (double)val[k];
    if (c == r) {
      a += 1.0;
      placed = true;
    }
    colind_out[o] = c;
    val_out[o++] = (float)((dr * a) * d[c]);
  }
  if (!placed) {
    colind_out[o] = r;
    val_out[o] = (float)((dr * 1.0) * dr);
  }
}

size_t scan_temp_bytes(int32_t n) {
  size_t bytes = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr, n + 1) !=
      hipSuccess)
    return 0;
  return bytes;
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int64_t gcnk_sym_normalize_workspace_bytes(int32_t n, int64_t nnz) {
  (void)nnz;
  if (n < 0) return GCNK_EARG;
  const int64_t dbytes = (((int64_t)n * 8) + 255) & ~255LL;
  const int64_t cbytes = ((((int64_t)n + 1) * 4) + 255) & ~255LL;
  return dbytes + cbytes + (int64_t)scan_temp_bytes(n);
}

extern "C" int gcnk_sym_normalize(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t n,
                                  int64_t nnz, int32_t* rowptr_out, int32_t* colind_out, float* val_out,
                                  void* workspace, int64_t workspace_bytes, void* stream) {
  if (n < 0 || nnz < 0 || !rowptr || !rowptr_out || (nnz > 0 && (!colind || !val)) ||
      (n > 0 && (!colind_out || !val_out))) {
    set_error("gcnk_sym_normalize: bad argument (n=%d nnz=%lld)", n, (long long)nnz);
    return GCNK_EARG;
  }
  if (nnz + n >= (int64_t)INT32_MAX) {
    set_error("gcnk_sym_normalize: nnz + n = %lld exceeds int32 CSR", (long long)(nnz + n));
    return GCNK_EUNSUP;
  }
  const int64_t need = gcnk_sym_normalize_workspace_bytes(n, nnz);
  if (!workspace || workspace_bytes < need) {
    set_error("gcnk_sym_normalize: needs %lld B of workspace, got %lld", (long long)need, (long long)workspace_bytes);
    return GCNK_EARG;
  }
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  double* d = (double*)ws;
  const int64_t dbytes = (((int64_t)n * 8) + 255) & ~255LL;
  int32_t* counts = (int32_t*)(ws + dbytes);
  const int64_t cbytes = ((((int64_t)n + 1) * 4) + 255) & ~255LL;
  void* tmp = ws + dbytes + cbytes;
  size_t tmp_bytes = scan_temp_bytes(n);
  hipLaunchKernelGGL(norm_rows_kernel, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, s, rowptr, colind, val, n,
                     counts, d);
  int rc = launch_check("norm_rows_kernel");
  if (rc) return rc;
  rc = hip_check(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, counts, rowptr_out, n + 1, s), "norm scan");
  if (rc || n == 0) return rc;
  hipLaunchKernelGGL(norm_fill_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rowptr, colind, val, n,
                     rowptr_out, d, colind_out, val_out);
  return launch_check("norm_fill_kernel");
}
