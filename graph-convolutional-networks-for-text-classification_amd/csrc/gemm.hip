// fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_16x16x4_f32), plus the
// deterministic column-sum used for bias gradients.
//
// Replaces th.spmm(dense H1, W2) (reference layer.py:102 in gc2 — ATen lowers
// a dense th.spmm to mm) and the dense autograd products of the GCN layers:
//   g_W2 = H1^T g      (transA; K = number of nodes -> split-K slabs)
//   g_H1 = g W2^T      (transB; fused relu/dropout backward epilogue)
// gfx950 has no xf32: the f32-input MFMA computes an exact fp32 fmaf chain
// over its 4-deep k step at the fp32 vector rate, and frees the VALU for the
// epilogue.
//
// Tile: BM x BN x 16, 256 threads = WM x WN waves, each wave FM x FN 16x16
// fragments.  Operands are staged k-major in LDS ([k][m], [k][n]) so every
// fragment read is 16 consecutive floats per k row.
#include "gcnk_common.h"

namespace gcnk {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct GemmEpi {
  const float* bias;
  const float* R;
  int64_t ldr;
  float scale;
  int32_t code;
};

__device__ __forceinline__ float gemm_epi(const GemmEpi& e, float acc, int64_t m, int64_t n) {
  switch (e.code) {
    case GCNK_GEMM_EPI_BIAS:
      return acc + (e.bias ? e.bias[n] : 0.f);
    case GCNK_GEMM_EPI_BIAS_RELU: {
      const float v = acc + (e.bias ? e.bias[n] : 0.f);
      return v > 0.f ? v : 0.f;
    }
    case GCNK_GEMM_EPI_MASK_POS:
      return e.R[m * e.ldr + n] > 0.f ? acc * e.scale : 0.f;
    default:
      return acc;
  }
}

constexpr int BK = 16;

template <int WM, int WN, int FM, int FN, bool TA, bool TB>
__global__ void __launch_bounds__(256)
gemm_f32_mfma_kernel(int32_t M, int32_t N, int32_t K, int32_t kchunk, const float* __restrict__ A,
                     int64_t lda, const float* __restrict__ B, int64_t ldb, float* __restrict__ C,
                     int64_t ldc, GemmEpi epi, float* __restrict__ slab) {
  constexpr int BM = WM * FM * 16;
  constexpr int BN = WN * FN * 16;
  static_assert(WM * WN == 4, "256 threads = 4 waves");
  __shared__ float As[BK][BM + 1];
  __shared__ float Bs[BK][BN + 1];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int64_t n0 = (int64_t)blockIdx.y * BN;
  const int32_t kb = blockIdx.z * kchunk;
  const int32_t ke = min(K, kb + kchunk);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // k tiles are register double-buffered: tile t + 1's global loads are in
  // flight while tile t is multiplied out of LDS
  constexpr int PA = (BM * BK + 255) / 256, PB = (BN * BK + 255) / 256;
  float ra[PA], rb[PB];
  // A and B through buffer resources when both fit 32-bit offsets: an element
  // outside the tile's rows or past this K chunk gets an offset past the
  // resource and reads 0 -- no branch per load (guarded, each of the tile's
  // loads compiled into a branch with its own vmcnt(0): the double buffer's
  // next tile arrived one load at a time)
  const int64_t a_bytes = (TA ? (int64_t)K : (int64_t)M) * lda * 4, b_bytes = (TB ? (int64_t)N : (int64_t)K) * ldb * 4;
  const bool use_buf = a_bytes < 0x7ff00000 && b_bytes < 0x7ff00000;   // (uniform)
  const __amdgpu_buffer_rsrc_t rsa =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), (short)0, use_buf ? (int)a_bytes : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B), (short)0, use_buf ? (int)b_bytes : 0, 0x00020000);
  auto fetch_buf = [&](int32_t k0) {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int e = tid + p * 256;
      int m, k;
      if (!TA) { m = e / BK; k = e % BK; }
      else { k = e / BM; m = e % BM; }
      const int gm = (int)m0 + m, gk = k0 + k;
      const bool ok = e < BM * BK && gm < M && gk < ke;
      ra[p] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          rsa, ok ? (TA ? (gk * (int)lda + gm) * 4 : (gm * (int)lda + gk) * 4) : 0x7ffffff0, 0, 0));
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int e = tid + p * 256;
      int n, k;
      if (!TB) { k = e / BN; n = e % BN; }
      else { n = e / BK; k = e % BK; }
      const int gn = (int)n0 + n, gk = k0 + k;
      const bool ok = e < BN * BK && gn < N && gk < ke;
      rb[p] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          rsb, ok ? (TB ? (gn * (int)ldb + gk) * 4 : (gk * (int)ldb + gn) * 4) : 0x7ffffff0, 0, 0));
    }
  };
  auto fetch_ptr = [&](int32_t k0) {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int e = tid + p * 256;
      int m, k;
      if (!TA) { m = e / BK; k = e % BK; }
      else { k = e / BM; m = e % BM; }
      const int64_t gm = m0 + m;
      const int32_t gk = k0 + k;
      ra[p] = (e < BM * BK && gm < M && gk < ke) ? (TA ? A[(int64_t)gk * lda + gm] : A[gm * lda + gk]) : 0.f;
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int e = tid + p * 256;
      int n, k;
      if (!TB) { k = e / BN; n = e % BN; }
      else { n = e / BK; k = e % BK; }
      const int64_t gn = n0 + n;
      const int32_t gk = k0 + k;
      rb[p] = (e < BN * BK && gn < N && gk < ke) ? (TB ? B[gn * ldb + gk] : B[(int64_t)gk * ldb + gn]) : 0.f;
    }
  };
  auto fetch = [&](int32_t k0) {
    if (use_buf) fetch_buf(k0);
    else fetch_ptr(k0);
  };
  if (kb < ke) fetch(kb);
  for (int32_t k0 = kb; k0 < ke; k0 += BK) {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int e = tid + p * 256;
      if (e >= BM * BK) break;
      if (!TA) As[e % BK][e / BK] = ra[p];
      else As[e / BM][e % BM] = ra[p];
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int e = tid + p * 256;
      if (e >= BN * BK) break;
      if (!TB) Bs[e / BN][e % BN] = rb[p];
      else Bs[e % BK][e / BK] = rb[p];
    }
    __syncthreads();
    if (k0 + BK < ke) fetch(k0 + BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const int kr = kk + (lane >> 4);
      float af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = As[kr][(wm * FM + i) * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = Bs[kr][(wn * FN + j) * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // C/D map of 16x16 f32 MFMA: reg r -> row (lane>>4)*4 + r, col lane&15
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = m0 + (wm * FM + i) * 16 + (lane >> 4) * 4 + r;
        const int64_t gn = n0 + (wn * FN + j) * 16 + (lane & 15);
        if (gm < M && gn < N) {
          if (slab) slab[((int64_t)blockIdx.z * M + gm) * N + gn] = acc[i][j][r];
          else C[gm * ldc + gn] = gemm_epi(epi, acc[i][j][r], gm, gn);
        }
      }
}

// Skinny-N GEMM (N <= 16 * NT, A row-major with 16-B aligned rows, B
// row-major): C = epi(A B), the gc2 support H1 W2 ([nodes x 200] x [200 x
// classes]; R8: 8 classes, 20ng: 20).  K is split over the 4 waves of a
// workgroup: the workgroup owns 16 rows, wave w the 16-deep k blocks
// [w*KB, (w+1)*KB) (lane l: row l&15, 16-B k slice l>>4 of each block; the k
// order inside a block is permuted consistently for A and B, k = 16c + 4(l>>4)
// + j at MFMA step j), so a wave holds KB float4 of A and runs a 4*KB-deep
// MFMA chain per 16-column tile instead of the whole of K; the four waves'
// accumulators meet in LDS and wave 0 adds them in wave order (fixed order:
// bitwise reproducible).  A is read once for all NT column tiles.
template <int KB, int NT>
__global__ void __launch_bounds__(256)
gemm_skinny_ksplit_kernel(int32_t M, int32_t N, int32_t K, const float* __restrict__ A, int64_t lda,
                          const float* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc,
                          GemmEpi epi) {
  __shared__ f32x4 s_acc[3][NT][64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * 16;
  const int r = lane & 15, q = lane >> 4;
  const int64_t row = m0 + r;
  const bool rok = row < M;
  float4 a[KB];
#pragma unroll
  for (int c = 0; c < KB; ++c) {
    const int k = 16 * (w * KB + c) + 4 * q;
    if (rok && k + 3 < K) {
      a[c] = *reinterpret_cast<const float4*>(A + row * lda + k);
    } else {
      a[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rok) {
        if (k + 0 < K) a[c].x = A[row * lda + k + 0];
        if (k + 1 < K) a[c].y = A[row * lda + k + 1];
        if (k + 2 < K) a[c].z = A[row * lda + k + 2];
      }
    }
  }
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int n = 16 * t + (lane & 15);
    const bool nok = n < N;
#pragma unroll
    for (int c = 0; c < KB; ++c) {
      const int k = 16 * (w * KB + c) + 4 * q;
      const float b0 = (nok && k + 0 < K) ? B[(int64_t)(k + 0) * ldb + n] : 0.f;
      const float b1 = (nok && k + 1 < K) ? B[(int64_t)(k + 1) * ldb + n] : 0.f;
      const float b2 = (nok && k + 2 < K) ? B[(int64_t)(k + 2) * ldb + n] : 0.f;
      const float b3 = (nok && k + 3 < K) ? B[(int64_t)(k + 3) * ldb + n] : 0.f;
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c].x, b0, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c].y, b1, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c].z, b2, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c].w, b3, acc[t], 0, 0, 0);
    }
  }
  if (w > 0)
#pragma unroll
    for (int t = 0; t < NT; ++t) s_acc[w - 1][t][lane] = acc[t];
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      const f32x4 o = s_acc[v][t][lane];
      acc[t][0] += o[0]; acc[t][1] += o[1]; acc[t][2] += o[2]; acc[t][3] += o[3];
    }
    const int n = 16 * t + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t gm = m0 + q * 4 + j;
      if (gm < M && n < N) C[gm * ldc + n] = gemm_epi(epi, acc[t][j], gm, n);
    }
  }
}

// Short-K, wide-N GEMM (NN; K <= 16 * KCH, K % 4 == 0, N % 4 == 0, A and B
// rows 16-B aligned): C = epi(A B) for a dense gensim-style X W1 ([nodes x
// 100] x [100 x 200]: the 20ng-shaped graph, R8 with 100-d features), where
// the tiled kernel above spends its time in 7 barrier-separated k tiles of a
// 64 x 64 tile.  One workgroup = 64 rows x NT n-tiles (16 NT columns): its B
// slice [K x 16 NT] is staged in LDS ONCE (float4 copies, rows padded by 4
// floats), all of it in flight with the A loads, and each wave multiplies its
// 16 rows by it with no further barrier: lane l holds A[row l&15][16c +
// 4(l>>4) .. +3] for every 16-deep k chunk c (the k order inside a chunk is
// permuted the same way for A and B, as in the skinny kernel) and runs
// 4 * KCH k-steps over NT independent accumulators.
// NT = 3 (48 columns, 23 KB of LDS, ~5 workgroups per CU) against round 3's 7
// (112 columns, 52 KB, 3 per CU): [70 x 100] x [100 x 200] 8.1 -> 4.7 us,
// [1000 x ..] 8.2 -> 4.9, the 20ng-shaped X W1 [18846 x ..] 18.2-18.6 ->
// 16.4-16.5 (profiles/r04_shortk_nt.log).
#ifndef GCNK_SHORTK_NT
#define GCNK_SHORTK_NT 3
#endif
constexpr int kShortkNT = GCNK_SHORTK_NT;
template <int KCH, int NT = kShortkNT>
__global__ void __launch_bounds__(256)
gemm_shortk_kernel(int32_t M, int32_t N, int32_t K, const float* __restrict__ A, int64_t lda,
                   const float* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc, GemmEpi epi) {
  constexpr int BN = 16 * NT, LW = BN + 4, KP = 16 * KCH, NQ = BN / 4;
  constexpr int PT = (KP * NQ + 255) / 256;
  __shared__ __attribute__((aligned(16))) float s_B[KP * LW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  // XCD-aware order (1-D grid): workgroups b and b + 8 share an XCD, so the
  // column tiles of one 64-row block run on one XCD -- its L2 serves their A
  // rows and merges their parts of each C line before the write-back
  const int nct = (N + BN - 1) / BN;
  const int b = blockIdx.x, grp = b / (8 * nct), rem = b % (8 * nct);
  const int64_t rb = (int64_t)grp * 8 + rem % 8;
  if (rb * 64 >= M) return;  // tail of the last group of 8 row blocks (no barrier passed yet)
  const int64_t m0 = rb * 64 + 16 * w;
  const int64_t n0 = (int64_t)(rem / 8) * BN;
  const int64_t row = m0 + r;
  const bool rok = row < M;
  // every load of the workgroup is issued before the first LDS store; invalid
  // pieces read the operand's first float4 and are zeroed afterwards
  float4 a[KCH];
  uint32_t aok = 0;
#pragma unroll
  for (int c = 0; c < KCH; ++c) {
    const int k = 16 * c + 4 * q;
    const bool ok = rok && k < K;  // K % 4 == 0: the whole float4 is inside the row
    a[c] = *reinterpret_cast<const float4*>(A + (ok ? row * lda + k : 0));
    aok |= (uint32_t)ok << c;
  }
  float4 v[PT];
  uint32_t bok = 0;
#pragma unroll
  for (int p = 0; p < PT; ++p) {
    const int e = tid + 256 * p;
    const int k = e / NQ;
    const int64_t n = n0 + 4 * (e % NQ);
    const bool ok = e < KP * NQ && k < K && n < N;  // N % 4 == 0
    v[p] = *reinterpret_cast<const float4*>(B + (ok ? (int64_t)k * ldb + n : 0));
    bok |= (uint32_t)ok << p;
  }
#pragma unroll
  for (int p = 0; p < PT; ++p) {
    const int e = tid + 256 * p;
    if (e >= KP * NQ) break;
    const bool ok = (bok >> p) & 1;
    *reinterpret_cast<float4*>(s_B + (e / NQ) * LW + 4 * (e % NQ)) = ok ? v[p] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // B fragments of chunk c + 1 are read from LDS while chunk c's MFMAs run
  // (left to itself the compiler waited on each ds_read2 before its two MFMAs)
  float bf[2][4][NT];
  auto fetch = [&](int c, float (&b)[4][NT]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t) b[j][t] = s_B[(16 * c + 4 * q + j) * LW + r + 16 * t];
  };
  fetch(0, bf[0]);
#pragma unroll
  for (int c = 0; c < KCH; ++c) {
    if (c + 1 < KCH) fetch(c + 1, bf[(c + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
    const bool ok = (aok >> c) & 1;
    const float av[4] = {ok ? a[c].x : 0.f, ok ? a[c].y : 0.f, ok ? a[c].z : 0.f, ok ? a[c].w : 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bf[c & 1][j][t], acc[t], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  // C/D map: reg jj -> row 4q + jj, column lane & 15
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int64_t n = n0 + 16 * t + r;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int64_t gm = m0 + 4 * q + jj;
      if (gm < M && n < N) C[gm * ldc + n] = gemm_epi(epi, acc[t][jj], gm, n);
    }
  }
}

// Small-M, long-K GEMM with the K split INSIDE the workgroup (round 6; NN, M <=
// 64, N % 4 == 0, lda % 4 == 0, A 16-B aligned): X[hubs] W1 of the factored
// gc1 with dense hub rows, R8-shaped [50 x 7463] x [7463 x 200].  Round 4's
// kernel here staged a 64-deep chunk of B in LDS per workgroup and left one
// slab per chunk (117 slabs, 4.7 MB of partials; 7.7 + 4.7 us with its reduce,
// profiles/r04_smallm_*).  Here workgroup (s, g) owns slab s (8 x 16 KBW k deep)
// and 16 NTG columns: wave w takes k blocks [KBW w, KBW w + KBW) of the slab
// for ALL four 16-row tiles (its B fragments feed four MFMA chains), the eight
// waves' products meet in LDS in wave order and one slab partial [M x 16 NTG]
// is written: 30 slabs (1.2 MB) at R8's shape, 1,680 waves carrying the MFMAs.
// A's 16-deep k block is read as one float4 per lane (k = 16 c + 4 q + j for
// quadrant q, step j) and B's rows in the same permuted order, so each MFMA
// still pairs A[row][k] with B[k][col].  Fixed-order sums: reproducible.
template <int KBW, int NTG>
__global__ void __launch_bounds__(512)
gemm_smallm_wk_kernel(int32_t M, int32_t N, int32_t K, const float* __restrict__ A, int64_t lda,
                      const float* __restrict__ B, int64_t ldb, float* __restrict__ slab) {
  constexpr int kW = 8, RT = 4;   // waves, 16-row tiles (M <= 64)
  __shared__ __attribute__((aligned(16))) f32x4 s_acc[kW][RT * NTG][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int64_t kb0 = ((int64_t)blockIdx.x * kW + w) * KBW;   // this wave's first 16-deep k block
  const int64_t n0 = (int64_t)blockIdx.y * 16 * NTG;
  // A and B through buffer resources sized to them (the dispatch keeps both
  // under 2 GB): rows of A past M and rows of B past K read 0 with no compare
  // or 64-bit address per load (that prologue was ~300 instructions a wave,
  // issued at 4 cycles each before the last load left); a column of B past N
  // only feeds an output column that is never stored.  A's components past K
  // are still zeroed: its row padding is not ours, and 0 x a NaN pad is NaN.
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), (short)0, M * (int)lda * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B), (short)0, K * (int)ldb * 4, 0x00020000);
  f32x4 a4[RT][KBW];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int c = 0; c < KBW; ++c) {
      const int row = 16 * t + r, k = 16 * ((int)kb0 + c) + 4 * q;
      a4[t][c] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, (row * (int)lda + (k < K ? k : 0)) * 4, 0, 0));
    }
  float b[KBW][4][NTG];
#pragma unroll
  for (int c = 0; c < KBW; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < NTG; ++u) {
        const int k = 16 * ((int)kb0 + c) + 4 * q + j, n = (int)n0 + 16 * u + r;
        b[c][j][u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, (k * (int)ldb + n) * 4, 0, 0));
      }
  // A's components past K zeroed by bit masks once every load is issued (as a
  // select, each A load compiled into a branch with its own vmcnt(0): eight
  // serial round trips; left to itself the scheduler also spread the loads
  // over the MFMAs, each waited for right after it left)
  __builtin_amdgcn_sched_barrier(0);
  float4 a[RT][KBW];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int c = 0; c < KBW; ++c) {
      const int k = 16 * ((int)kb0 + c) + 4 * q;
      a[t][c] = make_float4(__int_as_float(__float_as_int(a4[t][c][0]) & (k < K ? -1 : 0)),
                            __int_as_float(__float_as_int(a4[t][c][1]) & (k + 1 < K ? -1 : 0)),
                            __int_as_float(__float_as_int(a4[t][c][2]) & (k + 2 < K ? -1 : 0)),
                            __int_as_float(__float_as_int(a4[t][c][3]) & (k + 3 < K ? -1 : 0)));
    }
  f32x4 acc[RT][NTG];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int u = 0; u < NTG; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < KBW; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const float av = j == 0 ? a[t][c].x : j == 1 ? a[t][c].y : j == 2 ? a[t][c].z : a[t][c].w;
#pragma unroll
        for (int u = 0; u < NTG; ++u) acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b[c][j][u], acc[t][u], 0, 0, 0);
      }
    }
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int u = 0; u < NTG; ++u) s_acc[w][t * NTG + u][lane] = acc[t][u];
  __syncthreads();
  // the eight waves' tiles summed in wave order; thread e owns (tile e / 64, lane e % 64)
  float* out = slab + (int64_t)blockIdx.x * M * N;
  for (int e = tid; e < RT * NTG * 64; e += 512) {
    const int ti = e / 64, l = e % 64;
    f32x4 v = s_acc[0][ti][l];
#pragma unroll
    for (int ww = 1; ww < kW; ++ww) v += s_acc[ww][ti][l];
    const int t = ti / NTG, u = ti % NTG;
    const int64_t n = n0 + 16 * u + (l & 15);
    // C/D map: reg jj -> row 4 (l >> 4) + jj of the tile, column l & 15
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int64_t m = 16 * t + 4 * (l >> 4) + jj;
      if (m < M && n < N) out[m * N + n] = v[jj];
    }
  }
}

// Sum S slabs [S][M][N] (M N % 4 == 0) into C: a workgroup owns 16 float4 of
// the output; thread group g (16 of them) sums the slabs [g P, g P + P) of
// them in slab order with all its loads in flight, and group 0 adds the 16
// group sums in group order (a fixed order: bitwise reproducible), then
// applies the epilogue.
constexpr int kRedItems = 16, kRedGroups = 16, kRedBatch = 8;
__global__ void __launch_bounds__(256)
gemm_slab_reduce4_kernel(int32_t M, int32_t N, int32_t S, const float* __restrict__ slab, float* __restrict__ C,
                         int64_t ldc, GemmEpi epi) {
  __shared__ float4 s_part[kRedGroups][kRedItems];
  const int i = threadIdx.x % kRedItems, g = threadIdx.x / kRedItems;
  const int64_t total4 = (int64_t)M * N / 4;
  const int64_t o = (int64_t)blockIdx.x * kRedItems + i;
  const int per = (S + kRedGroups - 1) / kRedGroups;
  const int s0 = g * per, s1 = min(S, s0 + per);
  const float4* sl = reinterpret_cast<const float4*>(slab);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (o < total4) {
    for (int sb = s0; sb < s1; sb += kRedBatch) {
      float4 v[kRedBatch];
#pragma unroll
      for (int j = 0; j < kRedBatch; ++j) v[j] = sb + j < s1 ? sl[(int64_t)(sb + j) * total4 + o] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int j = 0; j < kRedBatch; ++j)
        if (sb + j < s1) { acc.x += v[j].x; acc.y += v[j].y; acc.z += v[j].z; acc.w += v[j].w; }
    }
  }
  s_part[g][i] = acc;
  __syncthreads();
  if (g != 0 || o >= total4) return;
  float4 t = s_part[0][i];
#pragma unroll
  for (int gg = 1; gg < kRedGroups; ++gg) {
    const float4 u = s_part[gg][i];
    t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
  }
  const int64_t e = 4 * o, m = e / N, n = e % N;  // N % 4 == 0: one row
  float* c = C + m * ldc + n;
  c[0] = gemm_epi(epi, t.x, m, n + 0);
  c[1] = gemm_epi(epi, t.y, m, n + 1);
  c[2] = gemm_epi(epi, t.z, m, n + 2);
  c[3] = gemm_epi(epi, t.w, m, n + 3);
}

// Sum split-K slabs in slab order, then apply the epilogue.
__global__ void gemm_splitk_reduce_kernel(int32_t M, int32_t N, int32_t S, const float* __restrict__ slab,
                                          float* __restrict__ C, int64_t ldc, GemmEpi epi) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)M * N;
  if (idx >= total) return;
  float acc = 0.f;
  for (int s0 = 0; s0 < S; s0 += 16) {  // 16 loads in flight, summed in slab order
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = s0 + j < S ? slab[(int64_t)(s0 + j) * total + idx] : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (s0 + j < S) acc += v[j];
  }
  const int64_t m = idx / N, n = idx % N;
  C[m * ldc + n] = gemm_epi(epi, acc, m, n);
}

template <int WM, int WN, int FM, int FN>
int launch_gemm(bool ta, bool tb, int32_t M, int32_t N, int32_t K, const float* A, int64_t lda,
                const float* B, int64_t ldb, float* C, int64_t ldc, const GemmEpi& e, int32_t split,
                float* ws, hipStream_t s) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  int32_t kchunk = (K + split - 1) / split;
  kchunk = (kchunk + BK - 1) / BK * BK;
  if (kchunk <= 0) kchunk = BK;
  const int32_t nsplit = (K + kchunk - 1) / kchunk > 0 ? (K + kchunk - 1) / kchunk : 1;
  dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((N + BN - 1) / BN), (unsigned)nsplit);
  float* slab = nsplit > 1 ? ws : nullptr;
#define GCNK_GEMM_LAUNCH(TA_, TB_)                                                                      \
  hipLaunchKernelGGL((gemm_f32_mfma_kernel<WM, WN, FM, FN, TA_, TB_>), grid, dim3(256), 0, s, M, N, K,  \
                     kchunk, A, lda, B, ldb, C, ldc, e, slab)
  if (!ta && !tb) GCNK_GEMM_LAUNCH(false, false);
  else if (ta && !tb) GCNK_GEMM_LAUNCH(true, false);
  else if (!ta && tb) GCNK_GEMM_LAUNCH(false, true);
  else GCNK_GEMM_LAUNCH(true, true);
#undef GCNK_GEMM_LAUNCH
  int rc = launch_check("gemm_f32_mfma_kernel");
  if (rc || nsplit <= 1) return rc;
  const int64_t total = (int64_t)M * N;
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, M, N,
                     nsplit, ws, C, ldc, e);
  return launch_check("gemm_splitk_reduce_kernel");
}

// ---------------------------------------------------------------------------
// Column sum: pass 1 sums kColsumRows-row blocks, pass 2 sums blocks in order.
constexpr int kColsumRows = 64;

__global__ void colsum_pass1_kernel(const float* __restrict__ X, int64_t ldx, int32_t M, int32_t N,
                                    float* __restrict__ part) {
  const int64_t n = (int64_t)blockIdx.y * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int64_t r0 = (int64_t)blockIdx.x * kColsumRows;
  const int64_t r1 = min<int64_t>(r0 + kColsumRows, M);
  float acc = 0.f;
  for (int64_t r = r0; r < r1; r += 16) {  // 16 loads in flight, summed in row order
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = r + j < r1 ? X[(r + j) * ldx + n] : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (r + j < r1) acc += v[j];
  }
  part[(int64_t)blockIdx.x * N + n] = acc;
}

__global__ void colsum_pass2_kernel(const float* __restrict__ part, int32_t nblk, int32_t N,
                                    float* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float acc = 0.f;
  for (int b0 = 0; b0 < nblk; b0 += 16) {  // 16 loads in flight, summed in block order
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = b0 + j < nblk ? part[(int64_t)(b0 + j) * N + n] : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (b0 + j < nblk) acc += v[j];
  }
  out[n] = acc;
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int64_t gcnk_gemm_workspace_bytes(int32_t M, int32_t N, int32_t K, int32_t split_k) {
  (void)K;
  if (split_k <= 1) return 0;
  return (int64_t)split_k * M * N * 4;
}

extern "C" int gcnk_gemm_f32(int32_t transA, int32_t transB, int32_t M, int32_t N, int32_t K,
                             const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                             int64_t ldc, const float* bias, int32_t epilogue, const float* R,
                             int64_t ldr, float scale, int32_t split_k, float* workspace,
                             int64_t workspace_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0) {
    set_error("gcnk_gemm_f32: negative size");
    return GCNK_EARG;
  }
  if (M == 0 || N == 0) return GCNK_OK;
  if (!A || !B || !C) {
    set_error("gcnk_gemm_f32: null pointer");
    return GCNK_EARG;
  }
  if ((!transA && lda < K) || (transA && lda < M) || (!transB && ldb < N) || (transB && ldb < K) || ldc < N) {
    set_error("gcnk_gemm_f32: leading dimension too small");
    return GCNK_EARG;
  }
  if (epilogue == GCNK_GEMM_EPI_MASK_POS && (!R || ldr < N)) {
    set_error("gcnk_gemm_f32: MASK_POS epilogue needs R with ldr >= N");
    return GCNK_EARG;
  }
  if (epilogue != GCNK_GEMM_EPI_NONE && epilogue != GCNK_GEMM_EPI_BIAS && epilogue != GCNK_GEMM_EPI_BIAS_RELU &&
      epilogue != GCNK_GEMM_EPI_MASK_POS) {
    set_error("gcnk_gemm_f32: unknown epilogue %d", epilogue);
    return GCNK_EARG;
  }
  if (split_k < 1) split_k = 1;
  if (split_k > 1 && (!workspace || workspace_bytes < gcnk_gemm_workspace_bytes(M, N, K, split_k))) {
    set_error("gcnk_gemm_f32: split_k=%d needs %lld B of workspace", split_k,
              (long long)gcnk_gemm_workspace_bytes(M, N, K, split_k));
    return GCNK_EARG;
  }
  GemmEpi e{bias, R, ldr, scale, epilogue};
  hipStream_t s = (hipStream_t)stream;
  const bool ta = transA != 0, tb = transB != 0;
#ifndef GCNK_GEMM_NARROW_SHORTK
#define GCNK_GEMM_NARROW_SHORTK 1
#endif
  if (GCNK_GEMM_NARROW_SHORTK && !ta && !tb && M >= 16384 && N > 16 && N <= 32 && N % 4 == 0 && K > 128 &&
      K <= 256 && K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && aligned16(A) && aligned16(B) && split_k == 1) {
    // gc2's support H1 W2 at many rows ([nodes x 200] x [200 x classes]):
    // 64-row workgroups, each wave one whole K chain per output (no cross-wave
    // sum), W2's slice staged in LDS once per workgroup.  Against the skinny
    // K-split kernel (profiles/r04_narrow.log): [18846 x 200] x [200 x 20] 8.9 ->
    // 8.2 us, but [4000 x ..] 4.6 -> 5.5 and [7724 x 200] x [200 x 8] 3.5 -> 4.2:
    // only past 16k rows and 16 columns
    const int64_t nrb8 = ((int64_t)M + 64 * 8 - 1) / (64 * 8);
    const dim3 grid((unsigned)(nrb8 * 8));
#define GCNK_NARROW(KCH_, NT_) \
  hipLaunchKernelGGL((gemm_shortk_kernel<KCH_, NT_>), grid, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc, e)
    if (K <= 208)  // N in (16, 32]: two n-tiles
      GCNK_NARROW(13, 2);
    else GCNK_NARROW(16, 2);
#undef GCNK_NARROW
    return launch_check("gemm_shortk_kernel");
  }
  if (!ta && !tb && N <= 64 && K <= 1024 && lda % 4 == 0 && aligned16(A) && split_k == 1) {
    // 16 rows per workgroup, K split over its 4 waves (k blocks of 16 per wave),
    // every column tile of N from the same A registers
    const int kbw = ((K + 15) / 16 + 3) / 4;
    const int nt = (N + 15) / 16;
    const unsigned blocks = (unsigned)(((int64_t)M + 15) / 16);
#define GCNK_SKINNY_KS(KB_, NT_)                                                                              \
  hipLaunchKernelGGL((gemm_skinny_ksplit_kernel<KB_, NT_>), dim3(blocks), dim3(256), 0, s, M, N, K, A, lda, B, \
                     ldb, C, ldc, e)
#define GCNK_SKINNY_NT(NT_)              \
  if (kbw <= 1) GCNK_SKINNY_KS(1, NT_);  \
  else if (kbw <= 2) GCNK_SKINNY_KS(2, NT_); \
  else if (kbw <= 4) GCNK_SKINNY_KS(4, NT_); \
  else if (kbw <= 8) GCNK_SKINNY_KS(8, NT_); \
  else GCNK_SKINNY_KS(16, NT_);
    if (nt == 1) { GCNK_SKINNY_NT(1) }
    else if (nt == 2) { GCNK_SKINNY_NT(2) }
    else { GCNK_SKINNY_NT(4) }
#undef GCNK_SKINNY_NT
#undef GCNK_SKINNY_KS
    return launch_check("gemm_skinny_ksplit_kernel");
  }
#ifndef GCNK_GEMM_SHORTK
#define GCNK_GEMM_SHORTK 1
#endif
  if (GCNK_GEMM_SHORTK && !ta && !tb && K > 0 && K <= 128 && K % 4 == 0 && N > 64 && N % 4 == 0 && lda % 4 == 0 &&
      ldb % 4 == 0 && aligned16(A) && aligned16(B) && split_k == 1) {
    const int64_t nrb8 = ((int64_t)M + 64 * 8 - 1) / (64 * 8);  // groups of 8 row blocks
    const dim3 grid((unsigned)(nrb8 * 8 * ((N + 16 * kShortkNT - 1) / (16 * kShortkNT))));
    const int kch = (K + 15) / 16;
#define GCNK_SHORTK(KCH_) \
  hipLaunchKernelGGL((gemm_shortk_kernel<KCH_>), grid, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc, e)
    switch (kch) {
      case 1: GCNK_SHORTK(1); break;
      case 2: GCNK_SHORTK(2); break;
      case 3: GCNK_SHORTK(3); break;
      case 4: GCNK_SHORTK(4); break;
      case 5: GCNK_SHORTK(5); break;
      case 6: GCNK_SHORTK(6); break;
      case 7: GCNK_SHORTK(7); break;
      default: GCNK_SHORTK(8); break;
    }
#undef GCNK_SHORTK
    return launch_check("gemm_shortk_kernel");
  }
#ifndef GCNK_GEMM_SMALLM_WK
#define GCNK_GEMM_SMALLM_WK 1
#endif
#ifndef GCNK_WK_KBW   // 16-deep k blocks per wave (a slab is 8 waves of them)
#define GCNK_WK_KBW 2
#endif
#ifndef GCNK_WK_NTG   // 16-column n-tiles per workgroup
#define GCNK_WK_NTG 2
#endif
  // small M, long K: the in-workgroup K split (gemm_smallm_wk_kernel), slabs of
  // 8 waves x 16 KBW k, summed by gemm_slab_reduce4_kernel
  const int64_t wk_S = ((int64_t)K + 8 * 16 * GCNK_WK_KBW - 1) / (8 * 16 * GCNK_WK_KBW);
  if (GCNK_GEMM_SMALLM_WK && !ta && !tb && M <= 64 && K >= 512 && N % 4 == 0 && lda % 4 == 0 && aligned16(A) &&
      split_k > 1 && wk_S <= split_k && wk_S <= 65535 &&
      (int64_t)M * lda * 4 < INT32_MAX && ((int64_t)K + 16) * ldb * 4 < INT32_MAX) {   // (its buffer offsets)
    const dim3 grid((unsigned)wk_S, (unsigned)((N + 16 * GCNK_WK_NTG - 1) / (16 * GCNK_WK_NTG)));
    hipLaunchKernelGGL((gemm_smallm_wk_kernel<GCNK_WK_KBW, GCNK_WK_NTG>), grid, dim3(512), 0, s, M, N, K, A, lda, B,
                       ldb, workspace);
    int rc = launch_check("gemm_smallm_wk_kernel");
    if (rc) return rc;
    const int64_t total4 = (int64_t)M * N / 4;
    hipLaunchKernelGGL(gemm_slab_reduce4_kernel, dim3((unsigned)((total4 + kRedItems - 1) / kRedItems)),
                       dim3(kRedItems * kRedGroups), 0, s, M, N, (int32_t)wk_S, workspace, C, ldc, e);
    return launch_check("gemm_slab_reduce4_kernel");
  }
  if (N <= 16) return launch_gemm<4, 1, 2, 1>(ta, tb, M, N, K, A, lda, B, ldb, C, ldc, e, split_k, workspace, s);
  return launch_gemm<2, 2, 2, 2>(ta, tb, M, N, K, A, lda, B, ldb, C, ldc, e, split_k, workspace, s);
}

extern "C" int64_t gcnk_colsum_workspace_bytes(int32_t M, int32_t N) {
  const int64_t nblk = ((int64_t)M + kColsumRows - 1) / kColsumRows;
  return nblk * N * 4;
}

extern "C" int gcnk_colsum_f32(const float* X, int64_t ldx, int32_t M, int32_t N, float* out,
                               float* workspace, int64_t workspace_bytes, void* stream) {
  if (M < 0 || N < 0 || ldx < N) {
    set_error("gcnk_colsum_f32: bad shape");
    return GCNK_EARG;
  }
  if (N == 0) return GCNK_OK;
  hipStream_t s = (hipStream_t)stream;
  if (M == 0) {
    return hip_check(hipMemsetAsync(out, 0, (size_t)N * 4, s), "colsum memset");
  }
  if (!X || !out || !workspace || workspace_bytes < gcnk_colsum_workspace_bytes(M, N)) {
    set_error("gcnk_colsum_f32: null pointer or workspace too small");
    return GCNK_EARG;
  }
  const int32_t nblk = (M + kColsumRows - 1) / kColsumRows;
  hipLaunchKernelGGL(colsum_pass1_kernel, dim3((unsigned)nblk, (unsigned)((N + 255) / 256)), dim3(256), 0, s, X,
                     ldx, M, N, workspace);
  int rc = launch_check("colsum_pass1_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(colsum_pass2_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, workspace, nblk, N,
                     out);
  return launch_check("colsum_pass2_kernel");
}
