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
constexpr int kHP = 64 + 4;      // wave-private H1 tile row stride (floats): 16 x (64 + 4)
constexpr int kMaxP = 32;
constexpr int kTail0 = 192;      // NI = 3: the rotating tail n-tile's first column (4 waves x 48)
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

typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));

__device__ __forceinline__ float mask_bits(float v, int m) { return __int_as_float(__float_as_int(v) & m); }

// KS k-steps of W1; NI n-tiles per wave, interleaved by lane (NI = 4: F <= 256;
// NI = 3: F <= 208, columns 192.. as one rotating tail n-tile); NPM 16-column
// MFMA tiles of P, and PV (0 or 4) columns of P past them on the VALU
template <int KS, int NI, int NPM, int PV>
__global__ void __launch_bounds__(kThreads, 2)
dense_gc1_kernel(DenseArgs a) {
  resolve_rng(a.epi);
  constexpr int KP = a_stride(KS);
  constexpr int kAPer = (16 * 4 * KS + kThreads - 1) / kThreads;   // A-tile elements per thread
  constexpr int JS = 4 * NI;       // projection k-steps over a wave's 16 NI columns
  constexpr bool kTail = NI == 3;
  constexpr int kSlots = kWaves + (kTail ? 1 : 0);   // partial-sum slots: the waves', then the tail's
  __shared__ __attribute__((aligned(16))) float s_A[2][16 * KP];
  __shared__ __attribute__((aligned(16))) float s_h[kWaves][16 * kHP];
  __shared__ __attribute__((aligned(16))) float s_red[2][kSlots][NPM][64 * 4];
  __shared__ __attribute__((aligned(16))) float s_redv[2][kSlots][PV ? 64 : 1];
  __shared__ __attribute__((aligned(16))) float s_w2v[PV ? PV : 1][PV ? 256 : 4];   // W2[:, 16 NPM + pc], transposed
  __shared__ __attribute__((aligned(16))) float s_wt[kTail ? 4 * KS : 1][16];          // W1[:, 192 .. 207]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int F = a.F, K = a.K, P = a.P;
  const int base = 16 * NI * w;      // the wave's first column
  const int col0 = base + NI * c;    // this lane's NI physical columns col0 + t (n-tile t)
  const bool tail = kTail && F > kTail0;   // (uniform)

  // ---- registers for the whole launch: W1 fragments (k = 4 s + q, columns
  //      col0 + t; the tail n-tile's in LDS), W2 fragments of this wave's columns (local column 4 js + q
  //      of projection step js is physical column base + 4 js + q), b1.  All
  //      in flight at once (staging them through LDS in rounds -- a barrier per
  //      16 W1 rows -- measured 2x slower: eleven dependent memory round trips).
  //      Every load is unconditional from a clamped address and its value
  //      masked by bits (a guarded load compiles into a branch of ~10 scalar
  //      instructions, 4 cycles each), and the masked values are pinned here
  //      (left alone, the compiler re-applied the masks inside the tile loop).
  stamp(a.epi, 0);
  float* hw = s_h[w];
  // the A tile [16 x 4 KS] (zero past K and M): thread element e -> row e / (4 KS),
  // k e % (4 KS) -- consecutive threads, consecutive k: coalesced
  // The A tile through a buffer resource over the tile's rows (rows past M,
  // and every row of a tile past the last, read 0): thread element i has a
  // fixed offset inside the tile, and an element past K or past the tile gets
  // an offset past any tile's resource, so it reads 0 too -- one load
  // instruction per element, no compares or selects in the tile loop.
  int voff[kAPer];
#pragma unroll
  for (int i = 0; i < kAPer; ++i) {
    const int e = tid + kThreads * i, r = e / (4 * KS), k = e % (4 * KS);
    voff[i] = (e < 16 * 4 * KS && k < K) ? (r * (int)a.lda + k) * 4 : 0x7ffffff0;
  }
  auto load_a = [&](int tile, float (&av)[kAPer]) {
    const int64_t row0 = (int64_t)tile * 16;
    const int rows = row0 < a.M ? (int)min<int64_t>(16, a.M - row0) : 0;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.A + (rows ? row0 : 0) * a.lda), (short)0, rows * (int)a.lda * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < kAPer; ++i) av[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ra, voff[i], 0, 0));
  };
  auto put_a = [&](int buf, const float (&av)[kAPer]) {
#pragma unroll
    for (int i = 0; i < kAPer; ++i) {
      const int e = tid + kThreads * i;
      if (e < 16 * 4 * KS) s_A[buf][(e / (4 * KS)) * KP + e % (4 * KS)] = av[i];
    }
  };
  //      Every operand is read through a buffer resource sized to it, so a
  //      row past K (W1), F (W2) or a missing b1 reads 0 with no compare, and
  //      columns are clamped into [0, F): what a lane computes for a column
  //      past F is finite and is multiplied by W2's zero rows (and never
  //      stored).  The prologue's instruction count is its time (4 cycles an
  //      instruction, next to the other workgroup's MFMAs): a clamped,
  //      compared and masked load costs ~12 instructions, a buffer load with
  //      a scalar offset 1-2.
  const __amdgpu_buffer_rsrc_t rw1 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.W), (short)0, K * (int)a.ldw * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw2 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.W2), (short)0, F * (int)a.ldw2 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb1 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.epi.bias ? a.epi.bias : a.W), (short)0,
                                        a.epi.bias ? F * 4 : 0, 0x00020000);
  //      1. every load issued (the first A tile last) ...
  float wf[KS][NI];
  // NI = 3: a lane whose three columns cross F reads the row's last three and
  // shifts them down (sh = 1 or 2; 0 for every lane once F >= 192)
  const int cl = NI == 4 ? (col0 < F ? col0 : 0) : (col0 + 2 < F ? col0 : F - 3);
  const int sh = col0 - cl;   // (NI = 3: 0, 1 or 2 on the lanes that matter)
  {
    const int vo = (q * (int)a.ldw + cl) * 4;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int so = 16 * s * (int)a.ldw;
      if constexpr (NI == 4) {
        const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rw1, vo + so, 0, 0));
        wf[s][0] = v[0]; wf[s][1] = v[1]; wf[s][2] = v[2]; wf[s][3] = v[3];
      } else {
        const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rw1, vo + so, 0, 0);
        wf[s][0] = __uint_as_float(v.x); wf[s][1] = __uint_as_float(v.y); wf[s][2] = __uint_as_float(v.z);
      }
    }
  }
  //      (the tail n-tile's W1 columns once per workgroup, into LDS: held by
  //      every wave as registers they were 4x the loads of its 6.4 KB)
  constexpr int kTPer = kTail ? (64 * KS + kThreads - 1) / kThreads : 1;
  float tv[kTPer];
  if constexpr (kTail) {
#pragma unroll
    for (int i = 0; i < kTPer; ++i) {
      const int e = tid + kThreads * i, k = e >> 4, ct = kTail0 + (e & 15);
      tv[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw1, (k * (int)a.ldw + (ct < F ? ct : 0)) * 4, 0, 0));
    }
  }
  float w2f[JS][NPM];
  float w2t[kTail ? 4 : 1][NPM];
#pragma unroll
  for (int js = 0; js < JS + (kTail ? 4 : 0); ++js)
#pragma unroll
    for (int p = 0; p < NPM; ++p) {   // (columns of P past P: their S2 columns are never stored)
      const int col = js < JS ? base + 4 * js + q : kTail0 + 4 * (js - JS) + q, pc = 16 * p + c;
      float& dst = js < JS ? w2f[js < JS ? js : 0][p] : w2t[js < JS ? 0 : js - JS][p];
      dst = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw2, (col * (int)a.ldw2 + pc) * 4, 0, 0));
    }
  float bv[NI], btl = 0.f;
#pragma unroll
  for (int t = 0; t < NI; ++t)
    bv[t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb1, (cl + t) * 4, 0, 0));
  if constexpr (kTail)
    btl = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb1, (kTail0 + c < F ? kTail0 + c : F) * 4, 0, 0));
  float av0[kAPer];
  load_a(blockIdx.x, av0);
  float pv[PV ? PV : 1];
#pragma unroll
  for (int i = 0; i < PV; ++i)   // W2[tid][16 NPM + i] (rows past F read 0)
    pv[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw2, (tid * (int)a.ldw2 + 16 * NPM + i) * 4, 0, 0));
  //      2. ... then the NI = 3 shift (skipped, uniformly, once F >= 192) and
  //      the values pinned (left alone, the compiler re-derived them inside
  //      the tile loop)
  if constexpr (NI == 3) {
    if (F < 16 * NI * kWaves) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float e0 = sh == 0 ? wf[s][0] : sh == 1 ? wf[s][1] : wf[s][2];
        const float e1 = sh == 0 ? wf[s][1] : wf[s][2];
        wf[s][0] = e0; wf[s][1] = e1;
      }
      const float b0 = sh == 0 ? bv[0] : sh == 1 ? bv[1] : bv[2], b1 = sh == 0 ? bv[1] : bv[2];
      bv[0] = b0; bv[1] = b1;
    }
  }
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int t = 0; t < NI; ++t) asm volatile("" : "+v"(wf[s][t]));
#pragma unroll
  for (int js = 0; js < JS; ++js)
#pragma unroll
    for (int p = 0; p < NPM; ++p) asm volatile("" : "+v"(w2f[js][p]));
  if constexpr (kTail) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int p = 0; p < NPM; ++p) asm volatile("" : "+v"(w2t[j][p]));
    asm volatile("" : "+v"(btl));
  }
#pragma unroll
  for (int t = 0; t < NI; ++t) asm volatile("" : "+v"(bv[t]));
  if constexpr (kTail) {   // (tail columns past F zeroed: the rotating wave's H1 there must be 0)
#pragma unroll
    for (int i = 0; i < kTPer; ++i) {
      const int e = tid + kThreads * i;
      if (e < 64 * KS) s_wt[e >> 4][e & 15] = kTail0 + (e & 15) < F ? tv[i] : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < PV; ++i) s_w2v[i][tid] = pv[i];
  put_a(0, av0);
#ifdef GCNK_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(a.epi, 1);
#endif
  __syncthreads();

  // one 16-row tile from LDS buffer `buf`; the next tile's A is loaded under
  // its MFMAs and written to buffer buf ^ 1 before the barrier.  `rot` is the
  // wave that also runs the tail n-tile this tile (NI = 3): it moves from tile
  // to tile and between the workgroups that share a CU, so no SIMD carries it
  // every time.  The tail's projection goes to a partial slot of its own,
  // summed last: S2 does not depend on which wave ran it.
  auto tile_step = [&](int tile, int buf, int rot) {
    float av[kAPer];
    load_a(tile + gridDim.x, av);
    const bool mine = tail && w == rot;   // (uniform)
    // ---- 1. Z = A W1[:, cols_w]; lane (row c, quadrant q) reads A[c][4 s + q]
    //      All KS fragments read before the MFMAs (one LDS wait), and every
    //      wave issues NI MFMAs per k-step: an absent column's W1 fragments
    //      are zero (a branch per MFMA broke the back-to-back issue and put an
    //      LDS wait on every k-step)
    const float* sa = &s_A[buf][c * KP + q];
    float af[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) af[s] = sa[4 * s];
    f32x4 acc[NI];
#pragma unroll
    for (int t = 0; t < NI; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int t = 0; t < NI; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], wf[s][t], acc[t], 0, 0, 0);
    f32x4 acct = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (kTail) {
      if (mine) {
        float wt[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) wt[s] = s_wt[4 * s + q][c];
#pragma unroll
        for (int s = 0; s < KS; ++s) acct = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], wt[s], acct, 0, 0, 0);
      }
    }
    // ---- 2. epilogue (C/D map: reg r -> row 4 q + r, column c), H1 store,
    //      tile into wave-private LDS (local column NI c + t; the tail's 48 + c)
    const int64_t row0 = (int64_t)tile * 16;
    const bool plain = a.epi.code == GCNK_EPI_BIAS_RELU;
    //      (the plain / dropout choice is one uniform branch around all the
    //      tile's elements: tested per element, it compiled into ~50
    //      instructions and 5 branches per element on the plain path too)
    auto emit = [&](int r, const float (&h)[NI], float ht) __attribute__((always_inline)) {
      const int64_t row = row0 + 4 * q + r;
      if constexpr (NI == 4) {
        const f32x4 h4 = {h[0], h[1], h[2], h[3]};
        if (a.H && row < a.M && col0 < F) __builtin_nontemporal_store(h4, reinterpret_cast<f32x4*>(a.H + row * a.ldh + col0));
        *reinterpret_cast<f32x4*>(&hw[(4 * q + r) * kHP + 4 * c]) = h4;
      } else {
        if (a.H) {
#pragma unroll
          for (int t = 0; t < NI; ++t)
            if (row < a.M && col0 + t < F) __builtin_nontemporal_store(h[t], a.H + row * a.ldh + col0 + t);
          if (mine && row < a.M && kTail0 + c < F) __builtin_nontemporal_store(ht, a.H + row * a.ldh + kTail0 + c);
        }
#pragma unroll
        for (int t = 0; t < NI; ++t) hw[(4 * q + r) * kHP + NI * c + t] = h[t];
        if (mine) hw[(4 * q + r) * kHP + 48 + c] = ht;
      }
    };
    if (plain) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float h[NI];
#pragma unroll
        for (int t = 0; t < NI; ++t) h[t] = fmaxf(acc[t][r] + bv[t], 0.f);
        emit(r, h, fmaxf(acct[r] + btl, 0.f));
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = row0 + 4 * q + r;
        float h[NI];
#pragma unroll
        for (int t = 0; t < NI; ++t)
          h[t] = (row < a.M && col0 + t < F) ? apply_epi(a.epi, acc[t][r], bv[t], row, col0 + t) : 0.f;
        emit(r, h, (mine && row < a.M && kTail0 + c < F) ? apply_epi(a.epi, acct[r], btl, row, kTail0 + c) : 0.f);
      }
    }
    // the wave's own LDS writes before its reads (other lanes' elements)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- 3. partial S2 = H1[:, cols_w] W2[cols_w, :]; A layout: lane (row c,
    //      quadrant q) reads local column 4 js + q
    f32x4 pacc[NPM];
#pragma unroll
    for (int p = 0; p < NPM; ++p) pacc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      float ha[JS];
#pragma unroll
      for (int js = 0; js < JS; ++js) ha[js] = hw[c * kHP + 4 * js + q];
#pragma unroll
      for (int js = 0; js < JS; ++js)   // (absent columns: zero H1 x zero W2, no branch)
#pragma unroll
        for (int p = 0; p < NPM; ++p) pacc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[js], w2f[js][p], pacc[p], 0, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < NPM; ++p) *reinterpret_cast<f32x4*>(&s_red[buf][w][p][4 * lane]) = pacc[p];
    if constexpr (kTail) {
      if (mine) {
        f32x4 tacc[NPM];
#pragma unroll
        for (int p = 0; p < NPM; ++p) tacc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
        float ha[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) ha[j] = hw[c * kHP + 48 + 4 * j + q];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int p = 0; p < NPM; ++p) tacc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[j], w2t[j][p], tacc[p], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < NPM; ++p) *reinterpret_cast<f32x4*>(&s_red[buf][kWaves][p][4 * lane]) = tacc[p];
      }
    }
    if constexpr (PV > 0) {
      // P's columns 16 NPM + pc on the VALU (an MFMA tile for these few would
      // be mostly padding): lane -> row lane / 4, pc = lane % 4, sum over the
      // wave's columns in order
      const int vr = lane >> 2, pc = lane & 3;
      const float* hr = &hw[vr * kHP];
      const float* wv = &s_w2v[pc][base];
      float vs = 0.f;
#pragma unroll
      for (int i = 0; i < 4 * NI; ++i) {
        const f32x4 h4 = *reinterpret_cast<const f32x4*>(hr + 4 * i);
        const f32x4 w4 = *reinterpret_cast<const f32x4*>(wv + 4 * i);
        vs = fmaf(h4[0], w4[0], vs); vs = fmaf(h4[1], w4[1], vs);
        vs = fmaf(h4[2], w4[2], vs); vs = fmaf(h4[3], w4[3], vs);
      }
      s_redv[buf][w][lane] = vs;
      if constexpr (kTail) {
        if (mine) {
          const float* wt4 = &s_w2v[pc][kTail0];
          float ts = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const f32x4 h4 = *reinterpret_cast<const f32x4*>(hr + 48 + 4 * i);
            const f32x4 w4 = *reinterpret_cast<const f32x4*>(wt4 + 4 * i);
            ts = fmaf(h4[0], w4[0], ts); ts = fmaf(h4[1], w4[1], ts);
            ts = fmaf(h4[2], w4[2], ts); ts = fmaf(h4[3], w4[3], ts);
          }
          s_redv[buf][kWaves][lane] = ts;
        }
      }
    }
    put_a(buf ^ 1, av);     // the next tile's A (its readers passed the previous barrier)
    // (double-buffered by tile parity: wave 0 reads buffer `buf` before it
    // reaches the next barrier, and buffer `buf` is written again only after it)
    __syncthreads();
    // the partials summed in slot order (waves 0..3, then the tail) by the
    // whole workgroup (partial (row 4 q + r, column 16 p + c) at
    // s_red[.][slot][p][4 (16 q + c) + r])
    const int nslot = tail ? kWaves + 1 : kWaves;
#pragma unroll
    for (int i = 0; i < NPM; ++i) {
      const int e = tid + kThreads * i, tr = e / (16 * NPM), col = e % (16 * NPM);
      const int p = col >> 4, cc = col & 15, idx = 4 * (16 * (tr >> 2) + cc) + (tr & 3);
      float sum = s_red[buf][0][p][idx];
#pragma unroll
      for (int v = 1; v < kSlots; ++v)
        if (v < nslot) sum += s_red[buf][v][p][idx];
      if (row0 + tr < a.M && col < P) a.C2[(row0 + tr) * a.ldc2 + col] = sum;
    }
    if constexpr (PV > 0) {
      if (tid < 64) {
        float sum = s_redv[buf][0][tid];
#pragma unroll
        for (int v = 1; v < kSlots; ++v)
          if (v < nslot) sum += s_redv[buf][v][tid];
        const int tr = tid >> 2, col = 16 * NPM + (tid & 3);
        if (row0 + tr < a.M && col < P) a.C2[(row0 + tr) * a.ldc2 + col] = sum;
      }
    }
    // the wave-private H1 tile is rewritten next tile after these reads (in
    // order within the wave): no barrier needed
    __builtin_amdgcn_wave_barrier();
  };
  int buf = 0;
  // the tail's wave: moves by one each tile; workgroups b, b + 8 (the next on
  // the same XCD) and b + 256 start one apart
  int rot = ((int)(blockIdx.x >> 3) + (int)(blockIdx.x >> 8)) & 3;
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x, buf ^= 1, rot = (rot + 1) & 3) {
    tile_step(tile, buf, rot);
    if (tile == (int)blockIdx.x) stamp(a.epi, 2);
  }
  stamp(a.epi, 3);
}

// NI = 3 (the rotating tail) while F <= 208, P <= 20 and KS <= 25 (past those
// its registers spill); otherwise NI = 4 with one or two MFMA tiles of P
template <int KS>
int launch_ks(const DenseArgs& a, unsigned grid, hipStream_t s) {
  if constexpr (KS <= 25) {
    if (a.F <= kTail0 + 16 && a.P <= 20) {
      if (a.P <= 16)
        hipLaunchKernelGGL((dense_gc1_kernel<KS, 3, 1, 0>), dim3(grid), dim3(kThreads), 0, s, a);
      else
        hipLaunchKernelGGL((dense_gc1_kernel<KS, 3, 1, 4>), dim3(grid), dim3(kThreads), 0, s, a);
      return launch_check("dense_gc1_kernel");
    }
  }
  if (a.P <= 16) {
    hipLaunchKernelGGL((dense_gc1_kernel<KS, 4, 1, 0>), dim3(grid), dim3(kThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL((dense_gc1_kernel<KS, 4, 2, 0>), dim3(grid), dim3(kThreads), 0, s, a);
  }
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
  const int ks = (a.K + 3) / 4;
  if (ks <= 8) return launch_ks<8>(a, grid, s);
  if (ks <= 13) return launch_ks<13>(a, grid, s);
  if (ks <= 16) return launch_ks<16>(a, grid, s);
  if (ks <= 25) return launch_ks<25>(a, grid, s);
  return launch_ks<32>(a, grid, s);
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
  if (K > 128 || F > 256 || F % 4 || P > kMaxP || ldw1 % 4 || !aligned16(W1) ||
      (int64_t)K * ldw1 * 4 >= INT32_MAX || (int64_t)F * ldw2 * 4 >= INT32_MAX ||   // (32-bit buffer offsets;
      (int64_t)16 * ldax * 4 >= 0x7ff00000 ||                                        //  A's tile sentinel past them)
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
