// The (A-hat, X)-fixed operands of the factored gc1 (factor.py), built on the
// device once per operand pair.
//
//   gc1 = A-hat (X W1) + b1        (reference layer.py:102,106,110)
//       = U W1[k0:k0+Kc] + A_H (X_hubs W1) + b1
//
// U [M x Kcp] (rows in the block order `perm`): row r's sum over its items
// (r, d) with d a light row of A-hat_rd X[d, k0 + c] -- for a light row only
// its diagonal item contributes, for a hub row every light neighbour does.
// The sum runs in float64 in the row's CSR item order and is rounded to fp32
// once: the order the host restatement's sparse product uses (scipy csr_matmat
// accumulates over A's row items in order), and the fp32 x fp32 products are
// exact in float64, so device U equals the host float64 U bit for bit
// (tests/test_gpu_parity.py pins it).
//
// A_H is stored as one record per 32-row block of `perm` (csrc/factor.hip):
// 33 block-relative item offsets, 3 pad words, 32 row ids (-1 past M), then
// the block's rows' hub-column items {hub index, value bits} in CSR order.
//
// Both kernels are one-time setup: latency-bound gathers over ~M rows, a few
// hundred microseconds for R8 against ~80 ms for the host build they replace.
//
// Round 6: the structure analysis in front of them (which rows are hubs, do
// the light rows touch only hub columns and themselves, X's light-row column
// range, per-row hub-item counts), X's light rows as the dense Xl and X's hub
// rows are built here too (gcnk_factor_analyze, gcnk_factor_xl_f32,
// gcnk_*_gather_rows) -- the torch element-wise / nonzero / repeat_interleave /
// index kernels factor.py used for them cost ~120 ms of first-use module loads
// in a fresh process (the first forward's largest piece, scripts/first_forward.py).
#include "gcnk_common.h"

#include <climits>

namespace gcnk {
namespace {

constexpr int kBuildRows = 4;      // rows (one wave each) per 256-thread workgroup
constexpr int kRecRows = 32;       // csrc/factor.hip kRB
constexpr int kRecHeadW = 68;      // csrc/factor.hip kRecHead
constexpr int kRecRowIds = 36;

// One wave per output position p: row r = perm[p]; lane c owns columns c and
// c + 64 (Kcp <= 128).  Items are read in CSR order; loads of four items are
// issued before their adds, which still run in item order.
__global__ void __launch_bounds__(256) factor_u_kernel(const int32_t* __restrict__ rowptr,
                                                       const int32_t* __restrict__ colind,
                                                       const float* __restrict__ val, int32_t M,
                                                       const int32_t* __restrict__ hub_index,
                                                       const int32_t* __restrict__ perm, const float* __restrict__ Xl,
                                                       int64_t ldxl, int32_t Kc, float* __restrict__ U, int64_t ldu,
                                                       int32_t Kcp) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * kBuildRows + (threadIdx.x >> 6);
  if (p >= M) return;
  const int r = perm ? perm[p] : (int)p;
  const int c0 = lane, c1 = lane + 64;
  const bool in0 = c0 < Kc, in1 = c1 < Kc;
  double acc0 = 0.0, acc1 = 0.0;
  const int beg = rowptr[r], end = rowptr[r + 1];
  int j = beg;
  for (; j + 4 <= end; j += 4) {
    int d[4];
    double a[4];
    float x0[4], x1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      d[u] = colind[j + u];
      a[u] = (double)val[j + u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool light = !hub_index || hub_index[d[u]] < 0;
      const float* xr = Xl + (int64_t)d[u] * ldxl;
      x0[u] = light && in0 ? xr[c0] : 0.f;
      x1[u] = light && in1 ? xr[c1] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {   // item order (a product of two fp32 values is exact in float64)
      acc0 += a[u] * (double)x0[u];
      acc1 += a[u] * (double)x1[u];
    }
  }
  for (; j < end; ++j) {
    const int d = colind[j];
    if (hub_index && hub_index[d] >= 0) continue;
    const double a = (double)val[j];
    const float* xr = Xl + (int64_t)d * ldxl;
    acc0 += a * (double)(in0 ? xr[c0] : 0.f);
    acc1 += a * (double)(in1 ? xr[c1] : 0.f);
  }
  float* ur = U + p * ldu;
  if (c0 < Kcp) ur[c0] = (float)acc0;
  if (c1 < Kcp) ur[c1] = (float)acc1;
}

// One wave per 32-row block: lane i < 32 counts row perm[32b + i]'s hub items,
// an exclusive scan gives the block-relative offsets, then the wave walks the
// block's rows in order and compacts each row's hub items (ballot + popcount
// keeps CSR order) into the record.  `rec` is zeroed first (by the entry point); items past
// rec_words are dropped and counted in *overflow (the caller sized rec_words
// from the same counts, so it stays 0).
__global__ void __launch_bounds__(64) factor_rec_kernel(const int32_t* __restrict__ rowptr,
                                                        const int32_t* __restrict__ colind,
                                                        const float* __restrict__ val, int32_t M,
                                                        const int32_t* __restrict__ hub_index,
                                                        const int32_t* __restrict__ perm, int32_t* __restrict__ rec,
                                                        int32_t rec_words, int32_t* __restrict__ overflow) {
  __shared__ int s_off[kRecRows + 1];
  __shared__ int s_row[kRecRows];
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  int32_t* rb = rec + b * rec_words;
  const int64_t p = b * kRecRows + lane;
  int r = -1, cnt = 0;
  if (lane < kRecRows && p < M) {
    r = perm[p];
    for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) cnt += hub_index[colind[j]] >= 0;
  }
  // inclusive scan over the wave (lanes >= 32 hold 0)
  int incl = cnt;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const int o = __shfl_up(incl, s, 64);
    if (lane >= s) incl += o;
  }
  if (lane < kRecRows) {
    s_off[lane] = incl - cnt;
    s_row[lane] = r;
  }
  if (lane == kRecRows - 1) s_off[kRecRows] = incl;
  __syncthreads();
  if (lane <= kRecRows) rb[lane] = s_off[lane];
  if (lane < kRecRows) rb[kRecRowIds + lane] = s_row[lane];
  int dropped = 0;
  for (int i = 0; i < kRecRows; ++i) {
    const int ri = s_row[i];
    if (ri < 0) break;
    int base = kRecHeadW + 2 * s_off[i];
    const int e = rowptr[ri + 1];
    for (int j0 = rowptr[ri]; j0 < e; j0 += 64) {
      const int j = j0 + lane;
      int h = -1;
      float v = 0.f;
      if (j < e) {
        h = hub_index[colind[j]];
        v = val[j];
      }
      const uint64_t m = __ballot(h >= 0);
      const int before = __popcll(m & ((1ull << lane) - 1ull));
      if (h >= 0) {
        const int w = base + 2 * before;
        if (w + 1 < rec_words) {
          rb[w] = h;
          rb[w + 1] = __float_as_int(v);
        } else {
          dropped = 1;
        }
      }
      base += 2 * __popcll(m);
    }
  }
  if (dropped) atomicAdd(overflow, 1);
}

// ---- structure analysis (gcnk_factor_analyze).  Workspace words:
//   flag[M] | cnt[M] | info[8] {H, bad, k0, k1, xtot} | list[max_hubs]
constexpr int kInfoH = 0, kInfoBad = 1, kInfoK0 = 2, kInfoK1 = 3, kInfoXTot = 4;

__global__ void factor_info_init_kernel(int32_t* __restrict__ info) {
  if (threadIdx.x == 0) {
    info[kInfoH] = 0;
    info[kInfoBad] = 0;
    info[kInfoK0] = INT_MAX;
    info[kInfoK1] = -1;
    info[kInfoXTot] = 0;
  }
}

// thread per row: hub iff at least hmin nonzeros; hubs appended (order fixed on the host)
__global__ void __launch_bounds__(256) factor_hub_kernel(const int32_t* __restrict__ rowptr, int32_t M, int32_t hmin,
                                                         int32_t* __restrict__ flag, int32_t* __restrict__ info,
                                                         int32_t* __restrict__ list, int32_t max_hubs) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= M) return;
  const bool hub = rowptr[r + 1] - rowptr[r] >= hmin;
  flag[r] = hub ? 1 : 0;
  if (hub) {
    const int32_t pos = atomicAdd(info + kInfoH, 1);
    if (pos < max_hubs) list[pos] = (int32_t)r;
  }
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// wave per row r: its hub-item count; a light row with a column that is
// neither a hub nor r breaks the structure; X's light rows give the column
// range of their nonzero entries (CSR X, or dense X when x_rowptr is null),
// X's hub rows their total length
__global__ void __launch_bounds__(256) factor_scan_kernel(const int32_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ colind, int32_t M,
                                                          const int32_t* __restrict__ x_rowptr,
                                                          const int32_t* __restrict__ x_colind,
                                                          const float* __restrict__ x_val,
                                                          const float* __restrict__ x_dense, int64_t ldx, int32_t K,
                                                          const int32_t* __restrict__ flag, int32_t* __restrict__ cnt,
                                                          int32_t* __restrict__ info) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * kBuildRows + (threadIdx.x >> 6);
  if (r >= M) return;
  const bool hub = flag[r] != 0;
  int c_hub = 0, viol = 0;
  for (int j = rowptr[r] + lane; j < rowptr[r + 1]; j += 64) {
    const int c = colind[j];
    const bool ch = flag[c] != 0;
    c_hub += ch;
    viol |= !hub && !ch && c != r;
  }
  c_hub = wave_sum(c_hub);
  viol = wave_sum(viol);
  int lo = INT_MAX, hi = -1, xlen = 0;
  if (x_rowptr) {
    const int b = x_rowptr[r], e = x_rowptr[r + 1];
    if (hub) {
      xlen = e - b;
    } else {
      for (int j = b + lane; j < e; j += 64)
        if (x_val[j] != 0.f) {
          lo = min(lo, x_colind[j]);
          hi = max(hi, x_colind[j]);
        }
    }
  } else if (!hub) {
    const float* xr = x_dense + r * ldx;
    for (int c = lane; c < K; c += 64)
      if (xr[c] != 0.f) {
        lo = min(lo, c);
        hi = max(hi, c);
      }
  }
  lo = wave_min(lo);
  hi = wave_max(hi);
  if (lane == 0) {
    cnt[r] = c_hub;
    if (viol) atomicOr(info + kInfoBad, 1);
    if (hi >= 0) {
      atomicMin(info + kInfoK0, lo);
      atomicMax(info + kInfoK1, hi);
    }
    if (xlen) atomicAdd(info + kInfoXTot, xlen);
  }
}

// wave per row: Xl[r, c] = X[r, k0 + c] for c < Kc (light rows; 0 elsewhere and
// for hub rows, which the U kernel never reads), columns Kc .. Kcp - 1 zero
__global__ void __launch_bounds__(256) factor_xl_kernel(const int32_t* __restrict__ x_rowptr,
                                                        const int32_t* __restrict__ x_colind,
                                                        const float* __restrict__ x_val, int32_t M,
                                                        const int32_t* __restrict__ hub_index, int32_t k0, int32_t Kc,
                                                        float* __restrict__ Xl, int64_t ldxl, int32_t Kcp) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * kBuildRows + (threadIdx.x >> 6);
  if (r >= M) return;
  float* row = Xl + r * ldxl;
  for (int c = lane; c < Kcp; c += 64) row[c] = 0.f;
  if (hub_index[r] >= 0) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zeros land before any value (one lane per column)
  for (int j = x_rowptr[r] + lane; j < x_rowptr[r + 1]; j += 64) {
    const int c = x_colind[j] - k0;
    if (c >= 0 && c < Kc) row[c] = x_val[j];
  }
}

// workgroup per selected row i: out row i = in row rows[i] (CSR: at the offset
// of the lengths of rows[0 .. i), summed in order; block 0 also writes the end)
__global__ void __launch_bounds__(256) csr_gather_rows_kernel(const int32_t* __restrict__ rowptr,
                                                              const int32_t* __restrict__ colind,
                                                              const float* __restrict__ val,
                                                              const int32_t* __restrict__ rows, int32_t nrows,
                                                              int32_t* __restrict__ out_rowptr,
                                                              int32_t* __restrict__ out_colind,
                                                              float* __restrict__ out_val) {
  const int i = blockIdx.x;
  int off = 0;
  for (int k = 0; k < i; ++k) off += rowptr[rows[k] + 1] - rowptr[rows[k]];
  const int b = rowptr[rows[i]], e = rowptr[rows[i] + 1];
  if (threadIdx.x == 0) {
    out_rowptr[i] = off;
    if (i == nrows - 1) out_rowptr[nrows] = off + (e - b);
  }
  for (int j = b + (int)threadIdx.x; j < e; j += 256) {
    out_colind[off + j - b] = colind[j];
    out_val[off + j - b] = val[j];
  }
}

__global__ void __launch_bounds__(256) dense_gather_rows_kernel(const float* __restrict__ X, int64_t ldx, int32_t K,
                                                                const int32_t* __restrict__ rows,
                                                                float* __restrict__ out, int64_t ldo) {
  const float* src = X + (int64_t)rows[blockIdx.x] * ldx;
  float* dst = out + (int64_t)blockIdx.x * ldo;
  for (int c = threadIdx.x; c < ldo; c += 256) dst[c] = c < K ? src[c] : 0.f;
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int64_t gcnk_factor_analyze_workspace_bytes(int32_t M, int32_t max_hubs) {
  if (M < 0 || max_hubs < 0) return GCNK_EARG;
  return 4 * (2 * (int64_t)M + 8 + max_hubs);
}

extern "C" int gcnk_factor_analyze(const int32_t* rowptr, const int32_t* colind, int32_t M, int32_t hmin,
                                   const int32_t* x_rowptr, const int32_t* x_colind, const float* x_val,
                                   const float* x_dense, int64_t ldx, int32_t K, int32_t max_hubs, int32_t* info,
                                   int32_t* hubs, int32_t* cnt, void* workspace, int64_t workspace_bytes,
                                   void* stream) {
  if (M <= 0 || max_hubs <= 0 || hmin < 1 || !rowptr || !colind || !info || !hubs || !cnt || !workspace ||
      (!x_rowptr && (!x_dense || ldx < K || K <= 0)) || (x_rowptr && (!x_colind || !x_val))) {
    set_error("gcnk_factor_analyze: bad sizes or null operand (M=%d K=%d)", M, K);
    return GCNK_EARG;
  }
  if (workspace_bytes < gcnk_factor_analyze_workspace_bytes(M, max_hubs)) {
    set_error("gcnk_factor_analyze: workspace too small");
    return GCNK_EARG;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int32_t* flag = static_cast<int32_t*>(workspace);
  int32_t* dcnt = flag + M;
  int32_t* dinfo = dcnt + M;
  int32_t* list = dinfo + 8;
  hipLaunchKernelGGL(factor_info_init_kernel, dim3(1), dim3(64), 0, s, dinfo);
  int rc = launch_check("factor_info_init_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(factor_hub_kernel, dim3((unsigned)(((int64_t)M + 255) / 256)), dim3(256), 0, s, rowptr, M, hmin,
                     flag, dinfo, list, max_hubs);
  if ((rc = launch_check("factor_hub_kernel"))) return rc;
  hipLaunchKernelGGL(factor_scan_kernel, dim3((unsigned)(((int64_t)M + kBuildRows - 1) / kBuildRows)),
                     dim3(64 * kBuildRows), 0, s, rowptr, colind, M, x_rowptr, x_colind, x_val, x_dense, ldx, K, flag,
                     dcnt, dinfo);
  if ((rc = launch_check("factor_scan_kernel"))) return rc;
  if ((rc = hip_check(hipMemcpyAsync(info, dinfo, 8 * 4, hipMemcpyDeviceToHost, s), "analyze info copy"))) return rc;
  if ((rc = hip_check(hipMemcpyAsync(hubs, list, (size_t)max_hubs * 4, hipMemcpyDeviceToHost, s), "hub list copy")))
    return rc;
  if ((rc = hip_check(hipMemcpyAsync(cnt, dcnt, (size_t)M * 4, hipMemcpyDeviceToHost, s), "count copy"))) return rc;
  return hip_check(hipStreamSynchronize(s), "analyze sync");
}

extern "C" int gcnk_factor_xl_f32(const int32_t* x_rowptr, const int32_t* x_colind, const float* x_val, int32_t M,
                                  const int32_t* hub_index, int32_t k0, int32_t Kc, float* Xl, int64_t ldxl,
                                  int32_t Kcp, void* stream) {
  if (M <= 0 || Kc <= 0 || Kcp < Kc || ldxl < Kcp || k0 < 0 || !x_rowptr || !x_colind || !x_val || !hub_index ||
      !Xl) {
    set_error("gcnk_factor_xl_f32: bad sizes or null operand (M=%d Kc=%d Kcp=%d)", M, Kc, Kcp);
    return GCNK_EARG;
  }
  hipLaunchKernelGGL(factor_xl_kernel, dim3((unsigned)(((int64_t)M + kBuildRows - 1) / kBuildRows)),
                     dim3(64 * kBuildRows), 0, reinterpret_cast<hipStream_t>(stream), x_rowptr, x_colind, x_val, M,
                     hub_index, k0, Kc, Xl, ldxl, Kcp);
  return launch_check("factor_xl_kernel");
}

extern "C" int gcnk_csr_gather_rows(const int32_t* rowptr, const int32_t* colind, const float* val,
                                    const int32_t* rows, int32_t nrows, int32_t* out_rowptr, int32_t* out_colind,
                                    float* out_val, void* stream) {
  if (nrows <= 0 || !rowptr || !colind || !val || !rows || !out_rowptr || !out_colind || !out_val) {
    set_error("gcnk_csr_gather_rows: bad sizes or null operand (nrows=%d)", nrows);
    return GCNK_EARG;
  }
  hipLaunchKernelGGL(csr_gather_rows_kernel, dim3((unsigned)nrows), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     rowptr, colind, val, rows, nrows, out_rowptr, out_colind, out_val);
  return launch_check("csr_gather_rows_kernel");
}

extern "C" int gcnk_dense_gather_rows_f32(const float* X, int64_t ldx, int32_t K, const int32_t* rows, int32_t nrows,
                                          float* out, int64_t ldo, void* stream) {
  if (nrows <= 0 || K <= 0 || ldx < K || ldo < K || !X || !rows || !out) {
    set_error("gcnk_dense_gather_rows_f32: bad sizes or null operand (nrows=%d K=%d)", nrows, K);
    return GCNK_EARG;
  }
  hipLaunchKernelGGL(dense_gather_rows_kernel, dim3((unsigned)nrows), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), X, ldx, K, rows, out, ldo);
  return launch_check("dense_gather_rows_kernel");
}

extern "C" int gcnk_factor_u_f32(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                                 const int32_t* hub_index, const int32_t* perm, const float* Xl, int64_t ldxl,
                                 int32_t Kc, float* U, int64_t ldu, int32_t Kcp, void* stream) {
  if (M <= 0 || Kc <= 0 || Kcp < Kc || Kcp > 128 || ldu < Kcp || ldxl < Kc || !rowptr || !colind || !val ||
      !hub_index || !perm || !Xl || !U) {
    set_error("gcnk_factor_u_f32: bad sizes or null operand (M=%d Kc=%d Kcp=%d)", M, Kc, Kcp);
    return GCNK_EARG;
  }
  const unsigned grid = (unsigned)(((int64_t)M + kBuildRows - 1) / kBuildRows);
  hipLaunchKernelGGL(factor_u_kernel, dim3(grid), dim3(64 * kBuildRows), 0, reinterpret_cast<hipStream_t>(stream),
                     rowptr, colind, val, M, hub_index, perm, Xl, ldxl, Kc, U, ldu, Kcp);
  return launch_check("factor_u_kernel");
}

// A-hat X for the narrow-feature gc1 (csrc/dense_gc1.hip): every item of every
// row, rows in order -- factor_u_kernel with no hub index and no permutation.
extern "C" int gcnk_aggregate_f32(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                                  const float* X, int64_t ldx, int32_t K, float* out, int64_t ldo, int32_t Kp,
                                  void* stream) {
  if (M <= 0 || K <= 0 || Kp < K || Kp > 128 || ldo < Kp || ldx < K || !rowptr || !colind || !val || !X || !out) {
    set_error("gcnk_aggregate_f32: bad sizes or null operand (M=%d K=%d Kp=%d)", M, K, Kp);
    return GCNK_EARG;
  }
  const unsigned grid = (unsigned)(((int64_t)M + kBuildRows - 1) / kBuildRows);
  hipLaunchKernelGGL(factor_u_kernel, dim3(grid), dim3(64 * kBuildRows), 0, reinterpret_cast<hipStream_t>(stream),
                     rowptr, colind, val, M, nullptr, nullptr, X, ldx, K, out, ldo, Kp);
  return launch_check("factor_u_kernel");
}

extern "C" int gcnk_factor_records(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                                   const int32_t* hub_index, const int32_t* perm, int32_t* rec, int32_t rec_words,
                                   int32_t* overflow, void* stream) {
  if (M <= 0 || rec_words < kRecHeadW || rec_words % 4 || !rowptr || !colind || !val || !hub_index || !perm ||
      !rec || !overflow) {
    set_error("gcnk_factor_records: bad sizes or null operand (M=%d rec_words=%d)", M, rec_words);
    return GCNK_EARG;
  }
  const unsigned nblk = (unsigned)(((int64_t)M + kRecRows - 1) / kRecRows);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int rc = hip_check(hipMemsetAsync(rec, 0, (size_t)nblk * rec_words * 4, s), "records memset");
  if (!rc) rc = hip_check(hipMemsetAsync(overflow, 0, 4, s), "overflow memset");
  if (rc) return rc;
  hipLaunchKernelGGL(factor_rec_kernel, dim3(nblk), dim3(64), 0, s, rowptr,
                     colind, val, M, hub_index, perm, rec, rec_words, overflow);
  return launch_check("factor_rec_kernel");
}
