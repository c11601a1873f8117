// Sparse-format helpers, used once per graph:
//  * COO -> CSR (gcnk_coo_to_csr): the reference hands th.spmm torch sparse COO
//    tensors -- A-hat column-major and uncoalesced (utils.py:196-203), X
//    row-major (trainer.py:226-238) -- which ATen re-coalesces on every call;
//    here they are converted once: stable radix sort of (row * K + col), runs
//    of equal keys summed in input order (what ATen's coalesce computes), row
//    pointers as the lower bounds of each row in the sorted output;
//  * CSR transpose (stable), for the A^T / X^T operands of the autograd
//    products (the backward of th.spmm(adj, support) / th.spmm(X, W) at
//    layer.py:102,106 needs sparse^T g).
//
// Stable counting layout via an LSD radix sort of (column, source index)
// pairs: within each transposed row the entries keep ascending source-row
// order, so the result is a pure function of the input (no atomics decide
// placement).
#include "gcnk_common.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>

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

// key = row * K + col; an index out of range poisons the result (rowptr[M] = -1)
__global__ void coo_keys_kernel(const int64_t* __restrict__ rows, const int64_t* __restrict__ cols, int64_t nnz,
                                int32_t M, int32_t K, uint64_t* __restrict__ keys, int32_t* __restrict__ idx,
                                int32_t* __restrict__ bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const int64_t r = rows[i], c = cols[i];
  const bool ok = r >= 0 && r < M && c >= 0 && c < K;
  if (!ok) atomicOr(bad, 1);
  keys[i] = ok ? (uint64_t)r * (uint64_t)K + (uint64_t)c : 0;
  idx[i] = (int32_t)i;
}

// head[i] = 1 where a run of equal sorted keys starts
__global__ void run_heads_kernel(const uint64_t* __restrict__ keys, int64_t nnz, int32_t* __restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nnz) head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

// at each run head: the run's values summed in input order (the sort is stable),
// written at the run's rank (pos = inclusive scan of heads), with the run's row
// in orow[rank] (the output rows are then sorted: the row pointers are their
// lower bounds, no per-nonzero counting -- round 4 counted rows with one integer
// atomic per run, 7,463 of them on each of R8 X's 50 dense topic rows: 2.2 ms)
__global__ void run_sum_kernel(const uint64_t* __restrict__ keys, const int32_t* __restrict__ idx,
                               const int32_t* __restrict__ pos, const float* __restrict__ vals, int64_t nnz,
                               int32_t K, int32_t* __restrict__ colind, float* __restrict__ val,
                               int32_t* __restrict__ orow) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz || (i > 0 && keys[i] == keys[i - 1])) return;
  const uint64_t k = keys[i];
  float v = vals[idx[i]];
  for (int64_t j = i + 1; j < nnz && keys[j] == k; ++j) v += vals[idx[j]];
  const int32_t o = pos[i] - 1;
  colind[o] = (int32_t)(k % (uint64_t)K);
  val[o] = v;
  orow[o] = (int32_t)(k / (uint64_t)K);
}

// rowptr[r] = first output position whose row >= r, over the n = pos[nnz - 1]
// unique entries (orow sorted ascending)
__global__ void row_bounds_kernel(const int32_t* __restrict__ orow, const int32_t* __restrict__ pos, int64_t nnz,
                                  int32_t M, int32_t* __restrict__ rowptr) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > M) return;
  int64_t lo = 0, hi = pos[nnz - 1];
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (orow[mid] < r) lo = mid + 1;
    else hi = mid;
  }
  rowptr[r] = (int32_t)lo;
}

__global__ void poison_kernel(const int32_t* __restrict__ bad, int32_t M, int32_t* __restrict__ rowptr) {
  if (*bad) rowptr[M] = -1;
}

inline int bits_for64(uint64_t n) {
  int b = 1;
  while (b < 64 && ((uint64_t)1 << b) < n) ++b;
  return b;
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

// ---------------------------------------------------------------------------
// COO -> CSR
namespace {
struct CooWs {
  int64_t keys_in, keys_out, idx_in, idx_out, head, pos, cnt, bad, tmp, total;
  size_t tmp_bytes;
  CooWs(int64_t nnz, int32_t M, int32_t K) {
    auto a = [](int64_t b) { return (b + 255) & ~255LL; };
    size_t sort_b = 0, scan_b = 0, scan2_b = 0;
    const int bits = bits_for64((uint64_t)M * (uint64_t)(K > 0 ? K : 1));
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, (int)nnz, 0, bits);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, scan_b, (const int32_t*)nullptr, (int32_t*)nullptr, (int)nnz);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan2_b, (const int32_t*)nullptr, (int32_t*)nullptr, M + 1);
    tmp_bytes = std::max(sort_b, std::max(scan_b, scan2_b));
    keys_in = 0;
    keys_out = keys_in + a(nnz * 8);
    idx_in = keys_out + a(nnz * 8);
    idx_out = idx_in + a(nnz * 4);
    head = idx_out + a(nnz * 4);
    pos = head + a(nnz * 4);
    cnt = pos + a(nnz * 4);
    bad = cnt + a(((int64_t)M + 1) * 4);
    tmp = bad + 256;
    total = tmp + a((int64_t)tmp_bytes);
  }
};
}  // namespace

extern "C" int64_t gcnk_coo_to_csr_workspace_bytes(int64_t nnz, int32_t M, int32_t K) {
  if (nnz < 0 || M < 0 || K < 0) return GCNK_EARG;
  return CooWs(nnz, M, K).total;
}

extern "C" int gcnk_coo_to_csr(const int64_t* rows, const int64_t* cols, const float* vals, int64_t nnz, int32_t M,
                               int32_t K, int32_t* rowptr, int32_t* colind, float* val, void* workspace,
                               int64_t workspace_bytes, void* stream) {
  if (nnz < 0 || nnz >= INT32_MAX || M < 0 || K < 0 || !rowptr ||
      (nnz > 0 && (!rows || !cols || !vals || !colind || !val))) {
    set_error("gcnk_coo_to_csr: bad argument (nnz=%lld M=%d K=%d)", (long long)nnz, M, K);
    return GCNK_EARG;
  }
  hipStream_t s = (hipStream_t)stream;
  if (nnz == 0) return hip_check(hipMemsetAsync(rowptr, 0, ((size_t)M + 1) * 4, s), "coo_to_csr memset");
  const CooWs L(nnz, M, K);
  if (!workspace || workspace_bytes < L.total) {
    set_error("gcnk_coo_to_csr: workspace %lld B < %lld B", (long long)workspace_bytes, (long long)L.total);
    return GCNK_EARG;
  }
  char* w = (char*)workspace;
  uint64_t* keys_in = (uint64_t*)(w + L.keys_in);
  uint64_t* keys_out = (uint64_t*)(w + L.keys_out);
  int32_t* idx_in = (int32_t*)(w + L.idx_in);
  int32_t* idx_out = (int32_t*)(w + L.idx_out);
  int32_t* head = (int32_t*)(w + L.head);
  int32_t* pos = (int32_t*)(w + L.pos);
  int32_t* cnt = (int32_t*)(w + L.cnt);
  int32_t* bad = (int32_t*)(w + L.bad);
  void* tmp = w + L.tmp;
  size_t tb = L.tmp_bytes;
  const unsigned nb = (unsigned)((nnz + 255) / 256);
  (void)cnt;
  int rc = hip_check(hipMemsetAsync(bad, 0, 4, s), "coo_to_csr flag");
  if (rc) return rc;
  hipLaunchKernelGGL(coo_keys_kernel, dim3(nb), dim3(256), 0, s, rows, cols, nnz, M, K, keys_in, idx_in, bad);
  if ((rc = launch_check("coo_keys_kernel"))) return rc;
  const int bits = bits_for64((uint64_t)M * (uint64_t)(K > 0 ? K : 1));
  rc = hip_check(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys_in, keys_out, idx_in, idx_out, (int)nnz, 0, bits, s),
                 "coo_to_csr radix sort");
  if (rc) return rc;
  hipLaunchKernelGGL(run_heads_kernel, dim3(nb), dim3(256), 0, s, keys_out, nnz, head);
  if ((rc = launch_check("run_heads_kernel"))) return rc;
  tb = L.tmp_bytes;
  rc = hip_check(hipcub::DeviceScan::InclusiveSum(tmp, tb, head, pos, (int)nnz, s), "coo_to_csr scan");
  if (rc) return rc;
  // (head is free once scanned: it receives the output rows)
  hipLaunchKernelGGL(run_sum_kernel, dim3(nb), dim3(256), 0, s, keys_out, idx_out, pos, vals, nnz, K, colind, val,
                     head);
  if ((rc = launch_check("run_sum_kernel"))) return rc;
  hipLaunchKernelGGL(row_bounds_kernel, dim3((unsigned)(((int64_t)M + 1 + 255) / 256)), dim3(256), 0, s, head, pos,
                     nnz, M, rowptr);
  if ((rc = launch_check("row_bounds_kernel"))) return rc;
  hipLaunchKernelGGL(poison_kernel, dim3(1), dim3(1), 0, s, bad, M, rowptr);
  return launch_check("poison_kernel");
}

// ---------------------------------------------------------------------------
// CSR -> dense row-major (one-time layout change of a dense-enough sparse
// operand, e.g. a gensim-shaped X: the MFMA GEMM then replaces the tile path,
// whose 64-column chunks would leave every row block split over slabs).
// One wavefront per row; lane l owns columns l, l + 64, ... and writes each
// of them once: the sum of the row's entries in that column, in CSR order
// (no lane reads what another wrote).  Meant for the dense-enough operands it
// is used on (a few hundred columns, tens of nonzeros per row).
namespace gcnk {
namespace {
__global__ void __launch_bounds__(256) csr_to_dense_kernel(const int32_t* __restrict__ rowptr,
                                                           const int32_t* __restrict__ colind,
                                                           const float* __restrict__ val, int32_t M, int32_t K,
                                                           float* __restrict__ out, int64_t ld) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= M) return;
  const int32_t b = rowptr[r], e = rowptr[r + 1];
  float* row = out + r * ld;
  // strictly increasing columns (every CSR from_torch builds): zero the row,
  // then one plain store per nonzero -- O(K + nnz) per row
  bool sorted = true;
  for (int32_t k = b + 1 + lane; k < e; k += 64) sorted &= colind[k] > colind[k - 1];
  sorted = __all(sorted);
  if (sorted) {
    for (int32_t c = lane; c < K; c += 64) row[c] = 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zeros land before any lane's value
    for (int32_t k = b + lane; k < e; k += 64) row[colind[k]] = val[k];
    return;
  }
  // otherwise (repeated or unordered columns): each output element sums its
  // entries in CSR order -- O(K x nnz / 64) per row
  for (int32_t c = lane; c < K; c += 64) {
    float v = 0.f;
    for (int32_t k = b; k < e; ++k)
      if (colind[k] == c) v += val[k];
    row[c] = v;
  }
}
}  // namespace
}  // namespace gcnk

extern "C" int gcnk_csr_to_dense(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                                 int32_t K, float* out, int64_t ld, void* stream) {
  if (M < 0 || K < 0 || ld < K || (M > 0 && (!rowptr || !out))) {
    set_error("gcnk_csr_to_dense: bad argument (M=%d K=%d ld=%lld)", M, K, (long long)ld);
    return GCNK_EARG;
  }
  if (M == 0) return GCNK_OK;
  hipLaunchKernelGGL(csr_to_dense_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, (hipStream_t)stream, rowptr,
                     colind, val, M, K, out, ld);
  return launch_check("csr_to_dense_kernel");
}
