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
#include "gcnk_common.h"

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
// keeps CSR order) into the record.  `rec` is zeroed by the caller; items past
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

}  // namespace
}  // namespace gcnk

using namespace gcnk;

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
  hipLaunchKernelGGL(factor_rec_kernel, dim3(nblk), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), rowptr,
                     colind, val, M, hub_index, perm, rec, rec_words, overflow);
  return launch_check("factor_rec_kernel");
}
