// Hub-factored first GCN layer for gfx950: gc1 of the reference's doc-topic
// graph without the topic rows' gather-and-combine.
//
// Reference (layer.py:102,106,110,182,185 inside GCN.forward, layer.py:164-190):
//   H1 = dropout(relu(A-hat (X W1) + b1)),   S2 = H1 W2   (gc2's support, layer.py:102)
//
// Structure used (checked on the host, factor.py): the rows of A-hat split into
// a few hub rows (R8: the 50 topics) and light rows (the 7,674 documents) whose
// nonzeros are hub columns plus their own diagonal, and X's light rows are
// supported on a small contiguous column range Kc (R8: the 50 topic-weight
// columns).  Then, with S_T = X_hubs W1 (the hub rows of X W1, computed by the
// tile GEMM beforehand),
//   light row d:  (A X W1)[d] = (A_dd X[d, Kc]) W1[Kc] + sum_t A[d, t] S_T[t]
//   hub row t:    (A X W1)[t] = (sum_d A[t, d] X[d, Kc]) W1[Kc] + sum_t' A[t, t'] S_T[t']
// i.e. Z = U W1[Kc] + A_H S_T with U [M x Kc] dense and A_H [M x hubs] sparse,
// both fixed by (A-hat, X) and built once (factor.py).  The topic rows' sums over
// ~600 document rows each -- the north-star SpMM's long pole -- move into U's
// hub rows (the (A X) W association; fp32 rounding differs from A (X W) by
// ~1e-6 relative), and the document rows never read or write their S1 rows.
//
// One workgroup = 32 rows (512 threads, 8 waves: 2 row strips x 4 quarters of the
// F columns):
//   0. every operand of the block in one round of loads: W1[Kc] and S_T into LDS,
//      the block's U rows into LDS (16-B DMA; or its U fragments into registers),
//      its A_H record and W2 into LDS;
//   1. Z_strip = U_strip W1[Kc] on v_mfma_f32_16x16x4_f32 (exact fp32 FMA chains);
//   2. Z through LDS to row-major; + A_H S_T, + b1, ReLU, dropout (mask or hash,
//      the row kernel's epilogue); H1 stored only when a backward needs it;
//   3. S2 = H1 W2 on MFMA from the same LDS tile (K split over the two halves,
//      summed in a fixed order).
// No atomics, no hand-off between workgroups: bitwise reproducible.
#include "gcnk_common.h"


#include <algorithm>

namespace gcnk {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRB = 32;         // rows per workgroup
constexpr int kThreads = 512;   // 8 waves: 2 row strips x 4 column quarters
constexpr int kMaxKsteps = 32;  // Kc <= 128
constexpr int kProjMax = 32;    // projection width: P <= 32 (NP = 1 or 2 MFMA n-tiles)
// zero floats after the staged W1[Kc]: the n-tiles past F read up to column
// 64 NTQ - 1 of the last k-row, so the pad covers 64 NTQ - F of them (at least 64)
__host__ __device__ constexpr int bpad(int f, int ntq) { return 64 * ntq - f > 64 ? 64 * ntq - f : 64; }
// block record (factor.py): 33 row offsets, 3 pad | 32 row ids (-1 past M) |
// A_H items int2 {hub, value}.  Block b holds rows perm[32 b .. 32 b + 31]: the
// host spreads the hub rows (long item lists) over the blocks, U's rows are in
// that order, outputs go to the row ids.
constexpr int kRecRow = 36, kRecHead = 68;
// compile-time shapes (every MFMA unconditional, operands in fixed registers):
// KS k-steps of U W1[Kc] (Kc <= 4 KS; U columns past Kc read as zero, W1 rows
// past Kc staged as zero) and NTQ 16-column tiles per quarter of F (F <= 64 NTQ;
// columns past F are computed from zeroed or W1 LDS words and never used)
// (18: the 20ng-shaped X's 70 topic-weight columns, whose W1 rows at 25 k-steps
// would take the block's LDS past 160 KiB)
__host__ __device__ constexpr int pick_ks(int kc) { return kc <= 52 ? 13 : kc <= 72 ? 18 : kc <= 100 ? 25 : 32; }
__host__ __device__ constexpr int pick_ntq(int f) { return f <= 128 ? 2 : f <= 192 ? 3 : 4; }

struct FactorArgs {
  int32_t M, F, Kc, nhub, P;
  const float* U; int64_t ldu;          // [M x >= Kc], rows in block order
  const float* W; int64_t ldw; int32_t k0;  // W1 rows k0 .. k0 + Kc - 1 (ldw == F: staged flat)
  const float* S; int64_t lds;          // S_T [nhub x F]
  const int32_t* rec; int32_t rec_words;  // per 32-row block: off[33] | pad | row ids | items int2 {hub, val}
  const float* W2; int64_t ldw2;        // [F x P]
  int32_t u_lds;                        // 1: the block's U rows staged in LDS by 16-B DMA (ldu % 4 == 0, aligned)
  float* H; int64_t ldh;                // nullable
  float* C2; int64_t ldc2;              // [M x P]
  Epi epi;
};

// 1 (default): the item loop skips the last column slot where it lies past F
// (R8: hubfactor_gc1 10.09 -> 9.78 us, profiles/r05_factor_lastu.log)
#ifndef GCNK_FACTOR_LASTU
#define GCNK_FACTOR_LASTU 1
#endif

// 1 (default): U's rows staged in LDS by DMA where the block's LDS allows
#ifndef GCNK_FACTOR_ULDS
#define GCNK_FACTOR_ULDS 1
#endif

template <int KS>
__host__ __device__ constexpr int region1_floats(int F, int ntq) {
  return (4 * KS * F + bpad(F, ntq)) > kRB * (64 * ntq + 4) ? (4 * KS * F + bpad(F, ntq)) : kRB * (64 * ntq + 4);
}

template <int KS, int NTQ, int NP>
__global__ void __launch_bounds__(kThreads)
hubfactor_gc1_kernel(FactorArgs a) {
  resolve_rng(a.epi);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int strip = wv & 1, quarter = wv >> 1;
  const int F = a.F, Q = F / 4;
  constexpr int Fp = 64 * NTQ, Fz = Fp + 4;  // s_Z row stride: 16-B rows, conflict-free MFMA-layout accesses
  constexpr int Kr = 4 * KS;
  const int blk = (int)blockIdx.x;
  const int64_t m0 = (int64_t)blk * kRB;  // position in the block order (U's rows)
  // LDS: region1 = s_B [Kr][F] + bpad zeros (phase 1), then s_Z [kRB][Fz]
  //      | s_S [nhub][F] | s_W2 [F][P] | s_bias [F] | s_rec | s_red [NP][3][2][64][4]
  // Every global operand is staged here in the one round of loads that opens the
  // kernel: a global load behind an LDS-read index costs a full memory round trip
  // under load (~1-2 us each, measured), so nothing after the first wait touches
  // global memory except the stores.
  const int r1 = region1_floats<KS>(F, NTQ);
  float* s_B = smem;
  float* s_Z = smem;
  float* s_S = smem + r1;
  float* s_W2 = s_S + a.nhub * F;
  float* s_bias = s_W2 + ((F * a.P + 3) & ~3);
  int32_t* s_rec = reinterpret_cast<int32_t*>(s_bias + F);
  float* s_red = reinterpret_cast<float*>(s_rec + a.rec_words);
  // u_lds: U's 32 rows [kRB][KPU] after s_red; row stride = 4 (mod 64), so lane
  // (row c, quadrant q) reading k = 4 s + q hits bank 4 c + q (conflict-free)
  constexpr int KPU = 64 * ((4 * KS - 4 + 63) / 64) + 4;
  float* s_U = s_red + NP * 3 * 2 * 64 * 4;

  // ---- 0. loads, all issued before the first wait: zeros first (no LDS-DMA in
  //      flight yet), then LDS-DMA of W1[Kc] (flat), U's rows (u_lds; else the
  //      U fragments straight into registers below), the block's record, S_T,
  //      W2 and b1
  for (int e = a.Kc * F + tid; e < Kr * F + bpad(F, NTQ); e += kThreads) s_B[e] = 0.f;
  if (!a.epi.bias)
    for (int e = tid; e < F; e += kThreads) s_bias[e] = 0.f;
  // (splitting these loads by wave role -- waves 0-3 phase 1's operands, the
  // first barrier waiting only for those -- measured 9.28 against 9.35 us:
  // profiles/r05_factor_ulds_ab.log; not kept)
  {
    const int n4 = a.Kc * Q;  // float4 pieces of W1[k0 .. k0 + Kc) (rows of F floats, ldw == F)
    const float* wsrc = a.W + (int64_t)a.k0 * a.ldw;
    for (int e0 = wv * 64; e0 < n4; e0 += kThreads)
      if (e0 + lane < n4) lds_dma16(wsrc + 4 * (e0 + lane), s_B + 4 * e0);
    // U's rows by 16-B DMA (the per-lane fragment loads -- 16 rows x 16 B per
    // instruction -- cost ~1.1 us of the block: profiles/r05_factor_ulds_ab.log);
    // one instruction per row, pieces covering Kc (inside the row: ldu % 4 == 0)
    if (a.u_lds)
      for (int r = wv; r < kRB; r += kThreads / 64)
        if (m0 + r < a.M && 4 * lane < a.Kc) lds_dma16(a.U + (m0 + r) * a.ldu + 4 * lane, s_U + r * KPU);
    const int32_t* rec = a.rec + (int64_t)blk * a.rec_words;
    for (int e0 = wv * 64; e0 < a.rec_words / 4; e0 += kThreads)
      if (e0 + lane < a.rec_words / 4) lds_dma16(rec + 4 * (e0 + lane), s_rec + 4 * e0);
    const int s4 = a.nhub * Q;  // S_T [nhub x F] flat (lds == F)
    for (int e0 = wv * 64; e0 < s4; e0 += kThreads)
      if (e0 + lane < s4) lds_dma16(a.S + 4 * (e0 + lane), s_S + 4 * e0);
    const int w1 = F * a.P;     // W2 [F x P] flat (ldw2 == P), dword pieces
    for (int e0 = wv * 64; e0 < w1; e0 += kThreads)
      if (e0 + lane < w1) lds_dma4(a.W2 + e0 + lane, s_W2 + e0);
    if (a.epi.bias)
      for (int e0 = wv * 64; e0 < Q; e0 += kThreads)
        if (e0 + lane < Q) lds_dma16(a.epi.bias + 4 * (e0 + lane), s_bias + 4 * e0);
  }
  float af[KS];
  const int64_t urow = m0 + 16 * strip + (lane & 15);
  if (!a.u_lds) {
    const float* up = a.U + urow * a.ldu + (lane >> 4);
#pragma unroll
    for (int s = 0; s < KS; ++s)
      af[s] = (urow < a.M && 4 * s + (lane >> 4) < a.Kc) ? up[4 * s] : 0.f;
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's DMA and fragment loads have landed
  __syncthreads();
  if (a.u_lds) {   // (cells past Kc or past M were not written: selected away)
    const float* su = s_U + (16 * strip + (lane & 15)) * KPU + (lane >> 4);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      // bit mask, not a select: a select let the compiler sink each read into a
      // branch with its own LDS wait (13 round trips)
      const bool ok = urow < a.M && 4 * s + (lane >> 4) < a.Kc;
      af[s] = __int_as_float(__float_as_int(su[4 * s]) & (ok ? -1 : 0));
    }
  }
  stamp(a.epi, 0);

  // ---- 1. Z = U W1[Kc] for this wave's strip and column quarter
  f32x4 acc[NTQ];
#pragma unroll
  for (int i = 0; i < NTQ; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int c0 = quarter * NTQ * 16 + (lane & 15);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const float* br = s_B + (4 * s + (lane >> 4)) * F + c0;
    float bf[NTQ];
#pragma unroll
    for (int i = 0; i < NTQ; ++i) bf[i] = br[i * 16];
#pragma unroll
    for (int i = 0; i < NTQ; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], bf[i], acc[i], 0, 0, 0);
  }
  __syncthreads();  // s_B is overwritten by s_Z below
  stamp(a.epi, 1);
  // C/D map of the 16x16 f32 MFMA: reg r -> row (lane >> 4) * 4 + r, col lane & 15
#pragma unroll
  for (int i = 0; i < NTQ; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      s_Z[(16 * strip + (lane >> 4) * 4 + r) * Fz + c0 - (lane & 15) + i * 16 + (lane & 15)] = acc[i][r];
  __syncthreads();

  // ---- 2. row-major epilogue, 16 threads per row, NTQ float4 columns each
  //      (q = c16 + 16 u; slots past F computed from finite LDS words and
  //      dropped): + A_H S_T, + b1, ReLU, dropout; H1 stored when a backward
  //      needs it.  No bounds test inside the item loop, so each item's NTQ
  //      LDS reads issue together.
  {
    const int r = tid >> 4, c16 = tid & 15;
    const int64_t row = s_rec[kRecRow + r];  // output row (-1 past M)
    float4 z[NTQ];
#pragma unroll
    for (int u = 0; u < NTQ; ++u) z[u] = *reinterpret_cast<const float4*>(s_Z + r * Fz + 4 * (c16 + 16 * u));
    // one item at a time: batching the items' loads (4 per round, selects past
    // the row) measured slower, 2.28 against 2.12 us per block (LDS throughput,
    // not the item chain, bounds this loop; profiles/r03_factor.md)
    const int2* it = reinterpret_cast<const int2*>(s_rec + kRecHead);
    const int k1 = s_rec[r + 1];
#pragma unroll 2
    for (int k = s_rec[r]; k < k1; ++k) {
      const int2 p = it[k];
      const float v = __int_as_float(p.y);
      const float* srow = s_S + p.x * F + 4 * c16;
      float4 sv[NTQ];
#pragma unroll
      for (int u = 0; u < NTQ; ++u) {
#if GCNK_FACTOR_LASTU
        // the last column slot only where it lies inside F (R8: 2 of 16 lanes):
        // inactive lanes move no LDS bytes, and this loop is LDS-bandwidth-bound
        if (u == NTQ - 1 && c16 + 16 * u >= Q) { sv[u] = make_float4(0.f, 0.f, 0.f, 0.f); continue; }
#endif
        sv[u] = *reinterpret_cast<const float4*>(srow + 64 * u);
      }
#pragma unroll
      for (int u = 0; u < NTQ; ++u) Vec<4>::fma(z[u], v, sv[u]);
    }
    if (row >= 0) {
      auto put = [&](int q, const float4& h) __attribute__((always_inline)) {
        if (a.H) {  // H1 for the backward: streaming store (no dirty L2 lines at the kernel's end)
          typedef float f4a __attribute__((ext_vector_type(4), aligned(16)));
          __builtin_nontemporal_store(f4a{h.x, h.y, h.z, h.w}, reinterpret_cast<f4a*>(a.H + row * a.ldh + 4 * q));
        }
        *reinterpret_cast<float4*>(s_Z + r * Fz + 4 * q) = h;
      };
      // eval / no-dropout: one uniform branch around all the elements (tested
      // per element, the dropout path's code sat on the plain path: ~50
      // instructions and several branches per float4)
      if (a.epi.code == GCNK_EPI_BIAS_RELU) {
#pragma unroll
        for (int u = 0; u < NTQ; ++u) {
          const int q = c16 + 16 * u;
          if (q < Q) {
            const float4 bv = *reinterpret_cast<const float4*>(s_bias + 4 * q);
            put(q, make_float4(fmaxf(z[u].x + bv.x, 0.f), fmaxf(z[u].y + bv.y, 0.f), fmaxf(z[u].z + bv.z, 0.f),
                               fmaxf(z[u].w + bv.w, 0.f)));
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < NTQ; ++u) {
          const int q = c16 + 16 * u;
          if (q < Q) put(q, Vec<4>::epi(a.epi, z[u], *reinterpret_cast<const float4*>(s_bias + 4 * q), row, 4 * (int64_t)q));
        }
      }
    }
  }
  __syncthreads();
  stamp(a.epi, 2);

  // ---- 3. S2 = H1 W2 on MFMA: strip x quarter of the K = F sum each (W2's rows
  //      past F and columns past P as zero), NP 16-column n-tiles of P, quarters
  //      added in order
  f32x4 pc[NP];
  {
    const int n = lane & 15;
    constexpr int kq = Fp / 16;  // k-steps per quarter
    float av[kq];
#pragma unroll
    for (int j = 0; j < kq; ++j) av[j] = s_Z[(16 * strip + (lane & 15)) * Fz + 4 * (quarter * kq + j) + (lane >> 4)];
#pragma unroll
    for (int t = 0; t < NP; ++t) {
      float bw[kq];
#pragma unroll
      for (int j = 0; j < kq; ++j) {
        const int k = 4 * (quarter * kq + j) + (lane >> 4);
        bw[j] = (k < F && 16 * t + n < a.P) ? s_W2[k * a.P + 16 * t + n] : 0.f;
      }
      f32x4 p0 = f32x4{0.f, 0.f, 0.f, 0.f}, p1 = p0;
#pragma unroll
      for (int j = 0; j < kq; j += 2) {
        p0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bw[j], p0, 0, 0, 0);
        p1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j + 1], bw[j + 1], p1, 0, 0, 0);
      }
      pc[t] = p0 + p1;
    }
  }
  if (quarter > 0)
#pragma unroll
    for (int t = 0; t < NP; ++t)
      *reinterpret_cast<f32x4*>(s_red + (((t * 3 + quarter - 1) * 2 + strip) * 64 + lane) * 4) = pc[t];
  __syncthreads();
  if (quarter == 0) {
#pragma unroll
    for (int t = 0; t < NP; ++t) {
#pragma unroll
      for (int qq = 0; qq < 3; ++qq)
        pc[t] += *reinterpret_cast<const f32x4*>(s_red + (((t * 3 + qq) * 2 + strip) * 64 + lane) * 4);
      const int p = 16 * t + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = s_rec[kRecRow + 16 * strip + (lane >> 4) * 4 + r];
        if (row >= 0 && p < a.P) a.C2[row * a.ldc2 + p] = pc[t][r];
      }
    }
  }
  stamp(a.epi, 3);
}


// Debug/test aid: every workgroup fills the whole 160 KiB of LDS with `word`.
// LDS is not cleared between workgroups, so a kernel launched next on the same
// CUs starts from these words wherever it reads LDS it has not written (the
// tests poison it with NaN bits before the factored kernel).
__global__ void __launch_bounds__(1024) lds_poison_kernel(uint32_t word) {
  extern __shared__ uint32_t s_all[];
  for (int i = threadIdx.x; i < 160 * 1024 / 4; i += 1024) s_all[i] = word;
  __syncthreads();
  if (s_all[(threadIdx.x * 37) % (160 * 1024 / 4)] != word) s_all[0] = 0;  // keep the stores
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int gcnk_debug_poison_lds(uint32_t word, void* stream) {
  static std::atomic<uint64_t> done{0};
  const hipError_t attr = dyn_lds_attr(done, reinterpret_cast<const void*>(&lds_poison_kernel), 160 * 1024);
  if (attr != hipSuccess) return hip_check(attr, "lds_poison_kernel LDS attribute");
  hipLaunchKernelGGL(lds_poison_kernel, dim3(1024), dim3(1024), 160 * 1024, reinterpret_cast<hipStream_t>(stream), word);
  return launch_check("lds_poison_kernel");
}

static int pick_np(int32_t P) { return P <= 16 ? 1 : 2; }

static int64_t hubfactor_lds_bytes(int32_t F, int32_t Kc, int32_t nhub, int32_t rec_words, int32_t P) {
  const int64_t Fz = 64 * pick_ntq(F) + 4, Kr = 4 * pick_ks(Kc);
  const int64_t r1 = std::max<int64_t>(Kr * F + bpad(F, pick_ntq(F)), (int64_t)kRB * Fz);
  return 4 * (r1 + (int64_t)nhub * F + (((int64_t)F * P + 3) & ~3LL) + F + rec_words + pick_np(P) * 3 * 2 * 64 * 4);
}

// U's staged rows (u_lds): kRB rows of 4 KS floats at a stride of 4 (mod 64)
static int64_t hubfactor_u_bytes(int32_t Kc) {
  const int64_t ks = pick_ks(Kc);
  return 4 * (int64_t)kRB * (64 * ((4 * ks - 4 + 63) / 64) + 4);
}

extern "C" int64_t gcnk_hubfactor_lds_bytes(int32_t F, int32_t Kc, int32_t nhub, int32_t rec_words, int32_t P) {
  if (F <= 0 || Kc <= 0 || nhub <= 0 || rec_words < kRecHead || P <= 0 || P > kProjMax) return GCNK_EARG;
  return hubfactor_lds_bytes(F, Kc, nhub, rec_words, P);
}

// The dynamic-LDS limit is raised once per kernel instantiation and device
// (dyn_lds_attr), then the launch.
template <int KS, int NTQ, int NP>
static int launch_factor(const FactorArgs& a, int64_t nblk, int64_t lds_b, void* stream) {
  static std::atomic<uint64_t> done{0};
  const hipError_t attr =
      dyn_lds_attr(done, reinterpret_cast<const void*>(&hubfactor_gc1_kernel<KS, NTQ, NP>), 160 * 1024);
  if (attr != hipSuccess) return hip_check(attr, "hubfactor_gc1_kernel LDS attribute");
  hipLaunchKernelGGL((hubfactor_gc1_kernel<KS, NTQ, NP>), dim3((unsigned)nblk), dim3(kThreads), (size_t)lds_b,
                     reinterpret_cast<hipStream_t>(stream), a);
  return launch_check("hubfactor_gc1_kernel");
}

extern "C" int gcnk_hubfactor_gc1_f32(int32_t M, int32_t F, int32_t Kc, int32_t nhub, int32_t P, const float* U,
                                      int64_t ldu, const float* W, int64_t ldw, int32_t k0, const float* S,
                                      int64_t lds, const int32_t* rec, int32_t rec_words, const float* bias,
                                      int32_t epilogue, const uint8_t* drop_mask, int64_t ldm, float drop_scale,
                                      float keep_prob, uint64_t seed, uint64_t offset, const uint64_t* rng_base,
                                      const float* W2, int64_t ldw2, float* H, int64_t ldh, float* C2,
                                      int64_t ldc2, void* stream) {
  if (M <= 0 || F <= 0 || Kc <= 0 || nhub <= 0 || P <= 0 || !U || !W || !S || !rec || !W2 || !C2 || k0 < 0) {
    set_error("gcnk_hubfactor_gc1_f32: bad sizes or null operand (M=%d F=%d Kc=%d hubs=%d P=%d)", M, F, Kc, nhub, P);
    return GCNK_EARG;
  }
  if (ldu < Kc || ldw < F || lds < F || ldw2 < P || ldc2 < P || (H && ldh < F) || rec_words < kRecHead ||
      rec_words % 4) {
    set_error("gcnk_hubfactor_gc1_f32: leading dimension too small");
    return GCNK_EARG;
  }
  if (F % 4 || F > 256 || Kc > 4 * kMaxKsteps || P > kProjMax || ldw != F || lds != F || ldw2 != P ||
      !aligned16(W) || !aligned16(S) || (H && !aligned16(H)) || (H && ldh % 4) || (bias && !aligned16(bias))) {
    set_error("gcnk_hubfactor_gc1_f32: unsupported shape (F=%d %% 4, F <= 256, Kc <= 128, P <= 32, 16-B rows)", F);
    return GCNK_EUNSUP;
  }
  if (epilogue < GCNK_EPI_NONE || epilogue > GCNK_EPI_BIAS_RELU_HASH ||
      (epilogue == GCNK_EPI_BIAS_RELU_DROP && (!drop_mask || ldm < F))) {
    set_error("gcnk_hubfactor_gc1_f32: bad epilogue %d (dropout needs a mask with ldm >= F)", epilogue);
    return GCNK_EARG;
  }
  const int64_t lds_b = hubfactor_lds_bytes(F, Kc, nhub, rec_words, P);
  if (lds_b > 160 * 1024) {
    set_error("gcnk_hubfactor_gc1_f32: %lld B of LDS per workgroup > 160 KiB (F=%d Kc=%d hubs=%d)",
              (long long)lds_b, F, Kc, nhub);
    return GCNK_EUNSUP;
  }
  FactorArgs a;
  a.M = M; a.F = F; a.Kc = Kc; a.nhub = nhub; a.P = P;
  // U's rows through LDS where they fit (R8: 95 + 8.7 KB; the 20ng-shaped 70
  // topic-weight columns at 152 KB take the direct loads)
  a.u_lds = GCNK_FACTOR_ULDS && ldu % 4 == 0 && aligned16(U) && lds_b + hubfactor_u_bytes(Kc) <= 160 * 1024;
  a.U = U; a.ldu = ldu; a.W = W; a.ldw = ldw; a.k0 = k0;
  a.S = S; a.lds = lds; a.rec = rec; a.rec_words = rec_words;
  a.W2 = W2; a.ldw2 = ldw2; a.H = H; a.ldh = ldh; a.C2 = C2; a.ldc2 = ldc2;
  Epi& e = a.epi;
  e.bias = bias; e.mask = drop_mask; e.scale = drop_scale; e.keep_prob = keep_prob;
  e.seed_lo = (uint32_t)seed; e.seed_hi = (uint32_t)(seed >> 32); e.offset = offset; e.rng_base = rng_base;
  e.code = epilogue; e.stamps = debug_stamps();
  e.ldm = epilogue == GCNK_EPI_BIAS_RELU_HASH ? (ldm > 0 ? ldm : F) : ldm;
  const int64_t nblk = ((int64_t)M + kRB - 1) / kRB;
  const int ks = pick_ks(Kc), ntq = pick_ntq(F), np = pick_np(P);
  const int64_t lds_l = lds_b + (a.u_lds ? hubfactor_u_bytes(Kc) : 0);
#define GCNK_FACTOR_CASE(KS_, NTQ_)                                                   \
  if (ks == KS_ && ntq == NTQ_)                                                       \
    return np == 1 ? launch_factor<KS_, NTQ_, 1>(a, nblk, lds_l, stream)              \
                   : launch_factor<KS_, NTQ_, 2>(a, nblk, lds_l, stream);
  GCNK_FACTOR_CASE(13, 2) GCNK_FACTOR_CASE(13, 3) GCNK_FACTOR_CASE(13, 4)
  GCNK_FACTOR_CASE(18, 2) GCNK_FACTOR_CASE(18, 3) GCNK_FACTOR_CASE(18, 4)
  GCNK_FACTOR_CASE(25, 2) GCNK_FACTOR_CASE(25, 3) GCNK_FACTOR_CASE(25, 4)
  GCNK_FACTOR_CASE(32, 2) GCNK_FACTOR_CASE(32, 3) GCNK_FACTOR_CASE(32, 4)
#undef GCNK_FACTOR_CASE
  set_error("gcnk_hubfactor_gc1_f32: no kernel for Kc=%d F=%d", Kc, F);
  return GCNK_EUNSUP;
}
