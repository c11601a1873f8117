// gc1 of a narrow-feature GCN from a cached aggregated operand (gfx950).
//
// Reference (layer.py:102,106,110,182,185 inside GCN.forward, layer.py:164-190,
// and gc2's support layer.py:102):
//   H1 = dropout(relu(A-hat (X W1) + b1)),   S2 = H1 W2
// When X is dense and narrow (nfeat <= nhid: the gensim-shaped 100-d topic
// features the README's R8 / 20ng numbers use, README.md:77,95), A-hat X is a
// fixed [M x K] operand of the (A-hat, X) pair, built once (the float64 row sums
// of csrc/factor_build.hip, rounded to fp32 once).  Then
//   Z = (A-hat X) W1
// is ONE short-K MFMA product per forward: the F-wide SpMM A-hat (X W1) and the
// X W1 GEMM in front of it never run (the association differs from the
// reference's A-hat (X W1) only in fp32 rounding, ~1e-6 relative).
//
// Persistent workgroups (two per CU, so one wave's MFMAs overlap the other's
// epilogue on each SIMD).  4 waves each; wave w owns the 64 columns 64 w .. 64 w + 63 of F as four
// MFMA n-tiles INTERLEAVED by lane: n-tile t, lane column c is physical column
// 64 w + 4 c + t, so a lane's four n-tiles are four consecutive columns and every
// W1 row piece, b1 and H1 piece it touches is one 16-B access
// (the n-tile-major mapping took 100 4-B W1 loads a wave, 4 rows x 64 B each --
// with 512 workgroups re-reading W1 that was half of the launch).  The W1 and W2
// fragments stay in registers for the whole launch.  Per 16-row tile:
//   0. the A tile [16 x K] is staged in LDS by the whole workgroup with
//      coalesced loads, one tile ahead (round 5's first version had every wave
//      load its own fragments straight from global memory -- 16 rows x 4 B per
//      instruction, four waves fetching the same tile -- and ran 4x slower);
//   1. Z_w = A_tile W1[:, cols_w] on v_mfma_f32_16x16x4_f32 (exact fp32 FMA
//      chains);
//   2. + b1, ReLU, dropout (mask or hash: the SpMM's epilogue), H1 stored only
//      when a backward needs it;
//   3. H1[:, cols_w] W2[cols_w, :] on MFMA (the tile transposed to the A layout
//      through wave-private LDS), the four waves' partials summed in LDS in a
//      fixed order and stored as S2.
// No atomics, no hand-off between workgroups: bitwise reproducible.
#include "gcnk_common.h"

#include <algorithm>

namespace gcnk {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;        // one per SIMD
constexpr int kThreads = 64 * kWaves;
constexpr int kNTQ = 4;          // n-tiles per wave: F <= 16 * 4 * kNTQ = 256
constexpr int kHP = 64 + 4;      // wave-private H1 tile row stride (floats): 16 x (64 + 4)
constexpr int kMaxP = 32;
struct DenseArgs {
  int32_t M, K, F, P;
  const float* A; int64_t lda;     // A-hat X [M x >= K]
  const float* W; int64_t ldw;     // W1 [K x F]
  const float* W2; int64_t ldw2;   // [F x P]
  float* H; int64_t ldh;           // nullable
  float* C2; int64_t ldc2;         // S2 [M x P]
  Epi epi;
  int32_t ntiles;                  // ceil(M / 16)
};

// KS k-steps of 4 (K <= 4 KS; lane quadrant q of step s multiplies k = 4 s + q),
// NP 16-column tiles of P
// A-tile row stride: >= 4 KS and = 4 (mod 64), so lane (row c, quadrant q)
// reading k = 4 s + q hits bank 4 c + q: conflict-free
constexpr int a_stride(int ks) { return 64 * ((4 * ks - 4 + 63) / 64) + 4; }

template <int KS, int NP>
__global__ void __launch_bounds__(kThreads, 2)
dense_gc1_kernel(DenseArgs a) {
  resolve_rng(a.epi);
  constexpr int KP = a_stride(KS);
  constexpr int kAPer = (16 * 4 * KS + kThreads - 1) / kThreads;   // A-tile elements per thread
  __shared__ __attribute__((aligned(16))) float s_A[2][16 * KP];
  __shared__ __attribute__((aligned(16))) float s_h[kWaves][16 * kHP];
  __shared__ __attribute__((aligned(16))) float s_red[2][kWaves][NP][64 * 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int F = a.F, K = a.K, P = a.P;
  const int col0 = 64 * w + 4 * c;   // this lane's four physical columns col0 + t (n-tile t)
  const bool cok = col0 < F;         // (F % 4 == 0, checked on the host: all four or none)

  // ---- registers for the whole launch: W1 fragments (k = 4 s + q, columns
  //      col0 + t: one 16-B load per k-step), W2 fragments of this wave's
  //      columns (local column lc = 16 t + 4 j + q of step (t, j) is physical
  //      column 64 w + lc), b1.  All in flight at once (staging them through LDS
  //      in rounds -- a barrier per 16 W1 rows -- measured 2x slower: eleven
  //      dependent memory round trips)
  stamp(a.epi, 0);
  float wf[KS][kNTQ];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 4 * s + q;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (cok && k < K) v = *reinterpret_cast<const float4*>(a.W + (int64_t)k * a.ldw + col0);
    wf[s][0] = v.x; wf[s][1] = v.y; wf[s][2] = v.z; wf[s][3] = v.w;
  }
  float w2f[kNTQ][4][NP];
#pragma unroll
  for (int t = 0; t < kNTQ; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int col = 64 * w + 16 * t + 4 * j + q, pc = 16 * p + c;
        w2f[t][j][p] = (col < F && pc < P) ? a.W2[(int64_t)col * a.ldw2 + pc] : 0.f;
      }
  float bv[kNTQ];
  {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.epi.bias && cok) v = *reinterpret_cast<const float4*>(a.epi.bias + col0);
    bv[0] = v.x; bv[1] = v.y; bv[2] = v.z; bv[3] = v.w;
  }
#ifdef GCNK_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(a.epi, 1);
#endif
  float* hw = s_h[w];
  // the A tile [16 x 4 KS] (zero past K and M): thread element e -> row e / (4 KS),
  // k e % (4 KS) -- consecutive threads, consecutive k: coalesced
  auto load_a = [&](int tile, float (&av)[kAPer]) {
#pragma unroll
    for (int i = 0; i < kAPer; ++i) {
      const int e = tid + kThreads * i, r = e / (4 * KS), k = e % (4 * KS);
      const int64_t row = (int64_t)tile * 16 + r;
      // (the address clamped into A, the value selected: no branch per load)
      const int64_t rc = row < a.M ? row : a.M - 1;
      const float v = a.A[rc * a.lda + (k < K ? k : K - 1)];
      av[i] = (e < 16 * 4 * KS && tile < a.ntiles && row < a.M && k < K) ? v : 0.f;
    }
  };
  auto put_a = [&](int buf, const float (&av)[kAPer]) {
#pragma unroll
    for (int i = 0; i < kAPer; ++i) {
      const int e = tid + kThreads * i;
      if (e < 16 * 4 * KS) s_A[buf][(e / (4 * KS)) * KP + e % (4 * KS)] = av[i];
    }
  };
  {
    float av[kAPer];
    load_a(blockIdx.x, av);
    put_a(0, av);
    __syncthreads();
  }

  // one 16-row tile from LDS buffer `buf`; the next tile's A is loaded under
  // its MFMAs and written to buffer buf ^ 1 before the barrier
  auto tile_step = [&](int tile, int buf) {
    float av[kAPer];
    load_a(tile + gridDim.x, av);
    // ---- 1. Z = A W1[:, cols_w]; lane (row c, quadrant q) reads A[c][4 s + q]
    //      All KS fragments read before the MFMAs (one LDS wait), and every
    //      wave issues kNTQ MFMAs per k-step: an absent n-tile's W1 fragments
    //      are zero (a branch per MFMA broke the back-to-back issue and put an
    //      LDS wait on every k-step)
    const float* sa = &s_A[buf][c * KP + q];
    float af[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) af[s] = sa[4 * s];
    f32x4 acc[kNTQ];
#pragma unroll
    for (int t = 0; t < kNTQ; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int t = 0; t < kNTQ; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], wf[s][t], acc[t], 0, 0, 0);
    // ---- 2. epilogue (C/D map: reg r -> row 4 q + r, column c), H1 store,
    //      tile into wave-private LDS
    const int64_t row0 = (int64_t)tile * 16;
    const bool plain = a.epi.code == GCNK_EPI_BIAS_RELU;
    //      (columns past F: acc and b1 zero, h = 0 written)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = row0 + 4 * q + r;
      float h[kNTQ];
#pragma unroll
      for (int t = 0; t < kNTQ; ++t) {
        if (plain) h[t] = fmaxf(acc[t][r] + bv[t], 0.f);
        else h[t] = (row < a.M && cok) ? apply_epi(a.epi, acc[t][r], bv[t], row, col0 + t) : 0.f;
      }
      const f32x4 h4 = {h[0], h[1], h[2], h[3]};
      if (a.H && row < a.M && cok) __builtin_nontemporal_store(h4, reinterpret_cast<f32x4*>(a.H + row * a.ldh + col0));
      *reinterpret_cast<f32x4*>(&hw[(4 * q + r) * kHP + 4 * c]) = h4;
    }
    // the wave's own LDS writes before its reads (other lanes' elements)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- 3. partial S2 = H1[:, cols_w] W2[cols_w, :]; A layout: lane (row c,
    //      quadrant q) reads local columns 16 t + 4 j + q
    f32x4 pacc[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) pacc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < kNTQ; ++t) {   // (absent n-tiles: zero H1 x zero W2, no branch)
      float ha[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) ha[j] = hw[c * kHP + 16 * t + 4 * j + q];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          pacc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[j], w2f[t][j][p], pacc[p], 0, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) *reinterpret_cast<f32x4*>(&s_red[buf][w][p][4 * lane]) = pacc[p];
    put_a(buf ^ 1, av);     // the next tile's A (its readers passed the previous barrier)
    // (double-buffered by tile parity: wave 0 reads buffer `buf` before it
    // reaches the next barrier, and buffer `buf` is written again only after it)
    __syncthreads();
    // the four waves' partials summed in wave order by the whole workgroup
    // (partial (row 4 q + r, column 16 p + c) at s_red[.][w][p][4 (16 q + c) + r])
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int e = tid + kThreads * i, tr = e / (16 * NP), col = e % (16 * NP);
      const int p = col >> 4, cc = col & 15, idx = 4 * (16 * (tr >> 2) + cc) + (tr & 3);
      float sum = s_red[buf][0][p][idx];
#pragma unroll
      for (int v = 1; v < kWaves; ++v) sum += s_red[buf][v][p][idx];
      if (row0 + tr < a.M && col < P) a.C2[(row0 + tr) * a.ldc2 + col] = sum;
    }
    // the wave-private H1 tile is rewritten next tile after these reads (in
    // order within the wave): no barrier needed
    __builtin_amdgcn_wave_barrier();
  };
  int buf = 0;
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x, buf ^= 1) {
    tile_step(tile, buf);
    if (tile == (int)blockIdx.x) stamp(a.epi, 2);
  }
  stamp(a.epi, 3);
}

template <int KS>
int launch_ks(const DenseArgs& a, int np, unsigned grid, hipStream_t s) {
  if (np == 1)
    hipLaunchKernelGGL((dense_gc1_kernel<KS, 1>), dim3(grid), dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL((dense_gc1_kernel<KS, 2>), dim3(grid), dim3(kThreads), 0, s, a);
  return launch_check("dense_gc1_kernel");
}

int cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  int n = dev < 64 ? cus[dev] : 0;
  if (n <= 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    if (dev < 64) cus[dev] = n;
  }
  return n;
}

int launch(const DenseArgs& a, hipStream_t s) {
  // persistent: 4 waves per workgroup, two workgroups per CU (<= 256 registers a wave)
  const unsigned grid = (unsigned)std::min<int64_t>(a.ntiles, 2 * cu_count());
  const int np = a.P <= 16 ? 1 : 2;
  const int ks = (a.K + 3) / 4;
  if (ks <= 8) return launch_ks<8>(a, np, grid, s);
  if (ks <= 13) return launch_ks<13>(a, np, grid, s);
  if (ks <= 16) return launch_ks<16>(a, np, grid, s);
  if (ks <= 25) return launch_ks<25>(a, np, grid, s);
  return launch_ks<32>(a, np, grid, s);
}

// the epilogue fields of the entry point
Epi make_epi(const float* bias, int32_t epilogue, const uint8_t* mask, int64_t ldm, int32_t F, float scale, float keep,
             uint64_t seed, uint64_t offset, const uint64_t* rng_base) {
  Epi e;
  e.bias = bias;
  e.mask = mask;
  e.ldm = epilogue == GCNK_EPI_BIAS_RELU_HASH ? (ldm > 0 ? ldm : F) : ldm;
  e.scale = scale;
  e.keep_prob = keep;
  e.seed_lo = (uint32_t)seed;
  e.seed_hi = (uint32_t)(seed >> 32);
  e.offset = offset;
  e.rng_base = rng_base;
  e.code = epilogue;
  e.stamps = debug_stamps();
  return e;
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int gcnk_dense_gc1_f32(int32_t M, int32_t K, int32_t F, int32_t P, const float* AX, int64_t ldax,
                                  const float* W1, int64_t ldw1, const float* bias, int32_t epilogue,
                                  const uint8_t* drop_mask, int64_t ldm, float drop_scale, float keep_prob,
                                  uint64_t seed, uint64_t offset, const uint64_t* rng_base, const float* W2,
                                  int64_t ldw2, float* H, int64_t ldh, float* C2, int64_t ldc2, void* stream) {
  if (M <= 0 || K <= 0 || F <= 0 || P <= 0 || !AX || !W1 || !W2 || !C2 || ldax < K || ldw1 < F || ldw2 < P ||
      ldc2 < P || (H && ldh < F)) {
    set_error("gcnk_dense_gc1_f32: bad sizes or null operand (M=%d K=%d F=%d P=%d)", M, K, F, P);
    return GCNK_EARG;
  }
  if (K > 128 || F > 16 * kWaves * kNTQ || F % 4 || P > kMaxP || ldw1 % 4 || !aligned16(W1) ||
      (bias && !aligned16(bias)) || (H && (ldh % 4 || !aligned16(H)))) {
    set_error("gcnk_dense_gc1_f32: unsupported shape (K=%d <= 128, F=%d <= 256 and %% 4, P=%d <= 32, "
              "16-B aligned W1 / b1 / H1 rows)", K, F, P);
    return GCNK_EUNSUP;
  }
  if (epilogue != GCNK_EPI_BIAS_RELU && epilogue != GCNK_EPI_BIAS_RELU_DROP && epilogue != GCNK_EPI_BIAS_RELU_HASH) {
    set_error("gcnk_dense_gc1_f32: epilogue %d is not a gc1 epilogue (bias + ReLU [+ dropout])", epilogue);
    return GCNK_EARG;
  }
  if (epilogue == GCNK_EPI_BIAS_RELU_DROP && (!drop_mask || ldm < F)) {
    set_error("gcnk_dense_gc1_f32: dropout epilogue needs a mask with ldm >= F");
    return GCNK_EARG;
  }
  DenseArgs a{};
  a.M = M; a.K = K; a.F = F; a.P = P;
  a.A = AX; a.lda = ldax; a.W = W1; a.ldw = ldw1; a.W2 = W2; a.ldw2 = ldw2;
  a.H = H; a.ldh = ldh; a.C2 = C2; a.ldc2 = ldc2;
  a.epi = make_epi(bias, epilogue, drop_mask, ldm, F, drop_scale, keep_prob, seed, offset, rng_base);
  a.ntiles = (M + 15) / 16;
  return launch(a, reinterpret_cast<hipStream_t>(stream));
}
