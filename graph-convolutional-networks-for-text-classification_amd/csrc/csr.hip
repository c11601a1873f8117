// Sparse-format helpers: CSR transpose (stable), used once per graph to build
// the A^T / X^T operands of the autograd products (reference: the backward of
// th.spmm(adj, support) / th.spmm(X, W) at layer.py:102,106 needs sparse^T g).
//
// Stable counting layout via an LSD radix sort of (column, source index)
// pairs: within each transposed row the entries keep ascending source-row
// order, so the result is a pure function of the input (no atomics decide
// placement).
#include "gcnk_common.h"

#include <hipcub/hipcub.hpp>

namespace gcnk {
namespace {

__global__ void iota_kernel(int32_t* __restrict__ v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (int32_t)i;
}

// rowptr_t[c] = first position whose sorted key >= c  (sorted keys are columns)
__global__ void bounds_kernel(const int32_t* __restrict__ keys, int64_t nnz, int32_t K,
                              int32_t* __restrict__ rowptr_t) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c > K) return;
  int64_t lo = 0, hi = nnz;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < c) lo = mid + 1;
    else hi = mid;
  }
  rowptr_t[c] = (int32_t)lo;
}

// source row of nonzero perm[i] (binary search in rowptr), and its value
__global__ void gather_kernel(const int32_t* __restrict__ rowptr, int32_t M, const float* __restrict__ val,
                              const int32_t* __restrict__ perm, int64_t nnz, int32_t* __restrict__ colind_t,
                              float* __restrict__ val_t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const int32_t k = perm[i];
  int32_t lo = 0, hi = M;  // rowptr[lo] <= k < rowptr[hi]
  while (hi - lo > 1) {
    const int32_t mid = (lo + hi) >> 1;
    if (rowptr[mid] <= k) lo = mid;
    else hi = mid;
  }
  colind_t[i] = lo;
  val_t[i] = val[k];
}

inline int bits_for(int32_t K) {
  int b = 1;
  while (b < 31 && ((int64_t)1 << b) < (int64_t)K) ++b;
  return b;
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

static size_t cub_temp_bytes(int64_t nnz, int32_t K) {
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const int32_t*)nullptr, (int32_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, (int)nnz, 0, bits_for(K));
  return (tmp + 255) & ~(size_t)255;
}

extern "C" int64_t gcnk_csr_transpose_workspace_bytes(int32_t M, int32_t K, int64_t nnz) {
  (void)M;
  const int64_t arr = ((nnz * 4 + 255) & ~255LL);
  return 3 * arr + (int64_t)cub_temp_bytes(nnz, K);
}

extern "C" int gcnk_csr_transpose(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                                  int32_t K, int64_t nnz, int32_t* rowptr_t, int32_t* colind_t, float* val_t,
                                  void* workspace, int64_t workspace_bytes, void* stream) {
  if (M < 0 || K < 0 || nnz < 0 || nnz >= INT32_MAX) {
    set_error("gcnk_csr_transpose: bad shape");
    return GCNK_EARG;
  }
  if (!rowptr || !rowptr_t || (nnz > 0 && (!colind || !val || !colind_t || !val_t))) {
    set_error("gcnk_csr_transpose: null pointer");
    return GCNK_EARG;
  }
  hipStream_t s = (hipStream_t)stream;
  if (nnz == 0) return hip_check(hipMemsetAsync(rowptr_t, 0, ((size_t)K + 1) * 4, s), "transpose memset");
  if (!workspace || workspace_bytes < gcnk_csr_transpose_workspace_bytes(M, K, nnz)) {
    set_error("gcnk_csr_transpose: workspace too small");
    return GCNK_EARG;
  }
  const int64_t arr = ((nnz * 4 + 255) & ~255LL);
  char* w = (char*)workspace;
  int32_t* keys_out = (int32_t*)(w);
  int32_t* idx_in = (int32_t*)(w + arr);
  int32_t* idx_out = (int32_t*)(w + 2 * arr);
  void* tmp = w + 3 * arr;
  size_t tmp_bytes = cub_temp_bytes(nnz, K);
  const unsigned nb = (unsigned)((nnz + 255) / 256);
  hipLaunchKernelGGL(iota_kernel, dim3(nb), dim3(256), 0, s, idx_in, nnz);
  int rc = launch_check("iota_kernel");
  if (rc) return rc;
  rc = hip_check(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, colind, keys_out, idx_in, idx_out, (int)nnz, 0,
                                                    bits_for(K), s),
                 "radix sort");
  if (rc) return rc;
  hipLaunchKernelGGL(bounds_kernel, dim3((unsigned)(((int64_t)K + 1 + 255) / 256)), dim3(256), 0, s, keys_out, nnz,
                     K, rowptr_t);
  if ((rc = launch_check("bounds_kernel"))) return rc;
  hipLaunchKernelGGL(gather_kernel, dim3(nb), dim3(256), 0, s, rowptr, M, val, idx_out, nnz, colind_t, val_t);
  return launch_check("gather_kernel");
}
