// Small-M, long-K GEMM into a FEW K-slabs, no reduction (gfx950):
//   C_s = A[:, K_s] B[K_s, :],  s < nslab (<= 4)
// for S_T = X[hubs] W1 of the factored gc1 (reference layer.py:102 on the topic
// rows; R8: [50 x 7463] x [7463 x 200]).  The consumer, the hub-factored gc1
// (csrc/factor.hip), sums the slabs in slab order while it stages S_T, so the
// split-K reduction costs no launch and no hand-off: round 4's tile kernel +
// slab-reduce launch took 6.6 + 4.9 us, round 5's one-launch last-arriver form
// (csrc/smallm.hip) 12 us, of which ~4 us was the coherent hand-off.
//
// K is cut into 16-deep chunks; slab s owns the chunks [s cps, (s + 1) cps),
// cps = ceil(chunks / nslab).  One workgroup (8 waves) per (16-row tile,
// 16-column tile, slab): wave w takes CPW consecutive chunks of the slab's
// range, every A and B fragment of them loaded at once (A: one 16-B piece per
// chunk, k order permuted alike for A and B -- lane quadrant q, step j
// multiplies k = 16 ch + 4 q + j; B: four 4-B loads per chunk), four
// accumulator chains (one per step j), then the 8 waves' 16 x 16 partials summed
// in wave order through LDS and stored.  Fixed order throughout: bitwise
// reproducible.
#include "gcnk_common.h"

#include <algorithm>

namespace gcnk {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kMaxSlabs = 64;   // (gcnk_hubfactor_gc1_slabs_f32 sums at most 4 of them)

template <int CPW>
__global__ void __launch_bounds__(kThreads)
gemm_kslab_kernel(int32_t M, int32_t N, int32_t K, const float* __restrict__ A, int64_t lda,
                  const float* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc, int64_t slab_stride,
                  int32_t nrt, int32_t nct, int32_t cps) {
  __shared__ __attribute__((aligned(16))) float s_red[kWaves][256];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int b = (int)blockIdx.x;
  const int rt = b % nrt, ct = (b / nrt) % nct, s = b / (nrt * nct);
  const int nchunk = (K + 15) / 16;
  const int ch_end = min(nchunk, (s + 1) * cps);
  const int ch0 = s * cps + w * CPW;
  const int64_t row = (int64_t)rt * 16 + c, col = (int64_t)ct * 16 + c;
  const bool rok = row < M, cok = col < N;
  const float* ap = A + (rok ? row : 0) * lda;
  // ---- every fragment of the wave's chunks in flight at once
  float4 af[CPW];
  float bf[CPW][4];
#pragma unroll
  for (int i = 0; i < CPW; ++i) {
    const int ch = ch0 + i;
    const int64_t k = 16 * (int64_t)ch + 4 * q;
    const bool ok = ch < ch_end && rok && k < K;   // lda % 4 == 0: the 16-B piece lies in the row's padding
    af[i] = ok ? *reinterpret_cast<const float4*>(ap + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok && k + 3 >= K) {                        // zero the columns past K
      if (k + 1 >= K) af[i].y = 0.f;
      if (k + 2 >= K) af[i].z = 0.f;
      if (k + 3 >= K) af[i].w = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bf[i][j] = (ch < ch_end && cok && k + j < K) ? B[(k + j) * ldb + col] : 0.f;
  }
  // ---- four independent MFMA chains (one per step j), summed in a fixed order
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < CPW; ++i) {
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i].x, bf[i][0], acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i].y, bf[i][1], acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i].z, bf[i][2], acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i].w, bf[i][3], acc[3], 0, 0, 0);
  }
  const f32x4 pv = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  // ---- the 8 waves' partials (C/D map: reg r -> row 4 q + r, column c) summed
  //      in wave order; thread e < 256 owns element (row e / 16, column e % 16)
  *reinterpret_cast<f32x4*>(&s_red[w][4 * lane]) = pv;
  __syncthreads();
  if (tid < 256) {
    const int er = tid >> 4, ec = tid & 15;
    const int idx = 4 * (16 * (er >> 2) + ec) + (er & 3);
    float sum = s_red[0][idx];
#pragma unroll
    for (int v = 1; v < kWaves; ++v) sum += s_red[v][idx];
    const int64_t orow = (int64_t)rt * 16 + er, ocol = (int64_t)ct * 16 + ec;
    if (orow < M && ocol < N) C[s * slab_stride + orow * ldc + ocol] = sum;
  }
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int gcnk_gemm_kslabs_f32(int32_t M, int32_t N, int32_t K, const float* A, int64_t lda, const float* B,
                                    int64_t ldb, int32_t nslab, float* C, int64_t ldc, int64_t slab_stride,
                                    void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !A || !B || !C || lda < K || ldb < N || ldc < N || nslab < 1 ||
      nslab > kMaxSlabs || (nslab > 1 && slab_stride < (int64_t)M * ldc)) {
    set_error("gcnk_gemm_kslabs_f32: bad sizes or null operand (M=%d N=%d K=%d nslab=%d)", M, N, K, nslab);
    return GCNK_EARG;
  }
  if (lda % 4 || !aligned16(A)) {
    set_error("gcnk_gemm_kslabs_f32: A needs 16-B aligned rows (lda %% 4 == 0)");
    return GCNK_EUNSUP;
  }
  const int nchunk = (K + 15) / 16;
  const int cps = (nchunk + nslab - 1) / nslab;
  const int need = (cps + kWaves - 1) / kWaves;   // chunks per wave
  const int nrt = (M + 15) / 16, nct = (N + 15) / 16;
  const dim3 grid((unsigned)(nrt * nct * nslab));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define GCNK_KSLAB(CPW_)                                                                                          \
  hipLaunchKernelGGL((gemm_kslab_kernel<CPW_>), grid, dim3(kThreads), 0, s, M, N, K, A, lda, B, ldb, C, ldc, \
                     slab_stride, nrt, nct, cps)
  if (need <= 4) GCNK_KSLAB(4);
  else if (need <= 8) GCNK_KSLAB(8);
  else if (need <= 12) GCNK_KSLAB(12);
  else if (need <= 16) GCNK_KSLAB(16);
  else if (need <= 24) GCNK_KSLAB(24);
  else {
    set_error("gcnk_gemm_kslabs_f32: K=%d too deep for %d slabs (<= %d)", K, nslab, 16 * 24 * kWaves * nslab);
    return GCNK_EUNSUP;
  }
#undef GCNK_KSLAB
  return launch_check("gemm_kslab_kernel");
}
