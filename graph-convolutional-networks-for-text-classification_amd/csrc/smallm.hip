// Small-M, long-K GEMM in ONE launch (gfx950): C = A B (or C += A B) for the dense hub rows
// of X -- S_T = X[hubs] W1 of the factored gc1 (reference layer.py:102 on the
// topic rows; R8: [50 x 7463] x [7463 x 200], 7.5 MB of operands, read once
// per forward because W1 changes every step).
//
// The K split is coarse (kSplitDepth-deep ranges, ~20 for R8) and the column
// tiles narrow (16 columns, 13 for F = 200), so ~260 workgroups each stage one
// K range of one column tile, multiply it on fp32 MFMA and publish a 64 x 16
// partial.  The LAST workgroup of each column tile to arrive (agent-scope
// arrival counter, the hand-off form MI355X_MICROARCH.md lists as valid: every
// partial stored sc1 and drained before one lane's add, the last adder reading
// sc1 only after its add returned) sums the tile's partials in split order --
// a fixed order, so the result is bitwise reproducible -- and stores C.
// Round 4's two-launch form (split-K tile kernel + slab reduce) spent 6.8 +
// 4.9 us on this product; its one-launch form with ~117 64-deep slabs and two
// levels of last-arriver sums 12.1 us.  Here one level suffices: a column
// tile's partials are ~20 x 4 KB.
#include "gcnk_common.h"

#include <algorithm>

namespace gcnk {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32v4 __attribute__((ext_vector_type(4)));

constexpr int kRows = 64;                    // M <= 64 (4 waves x 16 rows)
constexpr int kCT = 16;                      // columns per tile (one MFMA n-tile)
constexpr int kMaxSplits = 48;               // K ranges per column tile (the last arriver's loads in flight)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base_uniform) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base_uniform), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ const float* uniform_ptr(const float* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return reinterpret_cast<const float*>(((uint64_t)hi << 32) | lo);
}
constexpr int kSc1 = 16;   // cache-policy aux bit sc1 (write-through / coherent past the XCD L2)
// experiment knob (variant builds only): 1 no hand-off, 2 no A loads, 3 no B loads, 4 no MFMA
#ifndef GCNK_SMALLM_EXP
#define GCNK_SMALLM_EXP 0
#endif

// KCH 16-deep chunks per K range (kSplitDepth = 16 KCH)
template <int KCH>
__global__ void __launch_bounds__(256)
gemm_smallm_onepass_kernel(int32_t M, int32_t N, int32_t K, int32_t nsplit, const float* __restrict__ A, int64_t lda,
                           const float* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc,
                           int32_t accumulate, float* __restrict__ part, int32_t* __restrict__ ctr) {
  constexpr int KR = 16 * KCH;
  constexpr int LS = KR + 4;   // s_Bt row stride (floats): 16-B reads of 4 consecutive k, banks spread
  __shared__ __attribute__((aligned(16))) float s_Bt[kCT * LS];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int nct = (N + kCT - 1) / kCT;
  // workgroup b -> (column tile t, K range s): the splits of one tile are b = t + nct s
  const int t = (int)blockIdx.x % nct, s = (int)blockIdx.x / nct;
  const int64_t k0 = (int64_t)s * KR, n0 = (int64_t)t * kCT;
  // ---- every load in flight at once: the B slab [KR x 16] (float4 pieces,
  //      transposed into LDS: s_Bt[col][k]) and this wave's A rows
  constexpr int PB = (KR * 4 + 255) / 256;   // float4 pieces of B per thread
  float4 bv[PB];
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int e = tid + 256 * p;             // piece e: k = e / 4, columns 4 (e % 4) ..
    const int64_t k = k0 + e / 4, n = n0 + 4 * (e % 4);
    const bool ok = e < KR * 4 && k < K && n + 3 < N && GCNK_SMALLM_EXP != 3;
    bv[p] = ok ? *reinterpret_cast<const float4*>(B + k * ldb + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < KR * 4 && k < K && !ok && n < N) {   // a partial float4 at the right edge
      float tmp[4] = {0.f, 0.f, 0.f, 0.f};
      for (int i = 0; i < 4 && n + i < N; ++i) tmp[i] = B[k * ldb + n + i];
      bv[p] = make_float4(tmp[0], tmp[1], tmp[2], tmp[3]);
    }
  }
  const int64_t row = 16 * w + c;
  const bool rok = row < M;
  float4 a[KCH];
#pragma unroll
  for (int ch = 0; ch < KCH; ++ch) {
    const int64_t k = k0 + 16 * ch + 4 * q;
    const bool ok = rok && k < K && GCNK_SMALLM_EXP != 2;   // lda % 4 == 0 and lda >= K rounded up to 4: the float4 lies in the row
    a[ch] = ok ? *reinterpret_cast<const float4*>(A + row * lda + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok && k + 3 >= K) {          // zero the pad columns past K
      if (k + 1 >= K) a[ch].y = 0.f;
      if (k + 2 >= K) a[ch].z = 0.f;
      if (k + 3 >= K) a[ch].w = 0.f;
    }
  }
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int e = tid + 256 * p;
    if (e < KR * 4) {
      const int k = e / 4, n = 4 * (e % 4);
      s_Bt[(n + 0) * LS + k] = bv[p].x;
      s_Bt[(n + 1) * LS + k] = bv[p].y;
      s_Bt[(n + 2) * LS + k] = bv[p].z;
      s_Bt[(n + 3) * LS + k] = bv[p].w;
    }
  }
  __syncthreads();
  // ---- MFMA: k order inside a 16-deep chunk permuted alike for A and B (lane
  //      quadrant q, step j multiplies k = 16 ch + 4 q + j); four accumulators
  //      (one per step j: independent chains, so the 40-cycle dependent latency
  //      of v_mfma_f32_16x16x4_f32 hides under its 32-cycle issue), summed in a
  //      fixed order
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* bcol = s_Bt + c * LS + 4 * q;
  // every chunk's B fragments read before the MFMAs (one LDS wait, not one per chunk)
  float4 bf[KCH];
#pragma unroll
  for (int ch = 0; ch < KCH; ++ch) bf[ch] = *reinterpret_cast<const float4*>(bcol + 16 * ch);
#pragma unroll
  for (int ch = 0; ch < (GCNK_SMALLM_EXP == 4 ? 0 : KCH); ++ch) {
    const float4 b4 = bf[ch];
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ch].x, b4.x, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ch].y, b4.y, acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ch].z, b4.z, acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ch].w, b4.w, acc[3], 0, 0, 0);
  }
  f32x4 pv = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  if (GCNK_SMALLM_EXP == 4) pv += f32x4{a[KCH - 1].x, a[0].y, bcol[0], bcol[KR - 1]};
  if (GCNK_SMALLM_EXP == 1) {
    float* pt1 = part + ((int64_t)t * nsplit + s) * (kRows * kCT);
#pragma unroll
    for (int r = 0; r < 4; ++r) pt1[(16 * w + 4 * q + r) * kCT + c] = pv[r];
    return;
  }
  // ---- publish this K range's partial [64 x 16] (C/D map: reg r -> row 4 q + r,
  //      column c), sc1 stores; every wave drained before the arrival
  float* pt = part + ((int64_t)t * nsplit + s) * (kRows * kCT);
  {
    const float* base = uniform_ptr(pt);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(pv[r]), rsrc(base),
                                            (int)(((16 * w + 4 * q + r) * kCT + c) * 4), 0, kSc1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int arrived = __hip_atomic_fetch_add(ctr + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = arrived == nsplit - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // ---- the last arriver: the tile's partials in split order (sc1 loads), C.
  //      Thread (row tid / 4, columns 4 (tid % 4) ..): one 16-B load per split,
  //      ALL of them in flight at once (one memory latency, not one per batch:
  //      batches of 8 took ~1 us each past the L2s)
  const float* base = uniform_ptr(part + (int64_t)t * nsplit * (kRows * kCT));
  const int rr = tid >> 2, c4 = 4 * (tid & 3);
  f32v4 sum = {0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nsplit; j0 += kMaxSplits) {   // (one batch unless K > 16 x 32 x kMaxSplits)
    f32v4 v[kMaxSplits];
#pragma unroll
    for (int j = 0; j < kMaxSplits; ++j)
      if (j0 + j < nsplit)
        v[j] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), (int)((((j0 + j) * kRows + rr) * kCT + c4) * 4), 0, kSc1);
#pragma unroll
    for (int j = 0; j < kMaxSplits; ++j)
      if (j0 + j < nsplit) sum += v[j];
  }
  if (rr < M) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t n = n0 + c4 + i;
      if (n < N) C[rr * ldc + n] = accumulate ? C[rr * ldc + n] + sum[i] : sum[i];
    }
  }
  if (tid == 0) __hip_atomic_store(ctr + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-armed
}

// K range depth (16 KCH) for a K: about kTargetSplits ranges (GCNK_SMALLM_SPLITS
// overrides it for probes), never below 64 deep; past 32 x 16 x kMaxSplits the
// last arriver sums the partials in batches of kMaxSplits
int target_splits() {
  static const int t = [] {
    const char* v = getenv("GCNK_SMALLM_SPLITS");
    const int n = v ? atoi(v) : 0;
    return n > 0 && n <= kMaxSplits ? n : 20;
  }();
  return t;
}
int pick_kch(int32_t K) {
  const int want = (int)((K + 16LL * target_splits() - 1) / (16LL * target_splits()));
  static const int opts[] = {4, 6, 8, 12, 16, 24, 32};
  for (int o : opts)
    if (want <= o && (K + 16LL * o - 1) / (16LL * o) <= kMaxSplits) return o;
  return 32;
}
int64_t nsplit_for(int32_t K) { return (K + 16 * pick_kch(K) - 1) / (16 * pick_kch(K)); }

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int64_t gcnk_gemm_smallm_workspace_bytes(int32_t M, int32_t N, int32_t K) {
  if (M <= 0 || N <= 0 || K <= 0 || M > kRows) return GCNK_EARG;
  const int64_t nsplit = (K + 16 * pick_kch(K) - 1) / (16 * pick_kch(K));
  const int64_t nct = (N + kCT - 1) / kCT;
  return nct * nsplit * kRows * kCT * 4;
}

extern "C" int64_t gcnk_gemm_smallm_counter_bytes(int32_t N) {
  if (N <= 0) return GCNK_EARG;
  return (int64_t)((N + kCT - 1) / kCT) * 4;
}

extern "C" int gcnk_gemm_smallm_f32(int32_t M, int32_t N, int32_t K, const float* A, int64_t lda, const float* B,
                                   int64_t ldb, float* C, int64_t ldc, int32_t accumulate, float* workspace,
                                   int64_t workspace_bytes, int32_t* counters, int64_t counter_bytes, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !A || !B || !C || lda < K || ldb < N || ldc < N) {
    set_error("gcnk_gemm_smallm_f32: bad sizes or null operand (M=%d N=%d K=%d)", M, N, K);
    return GCNK_EARG;
  }
  if (M > kRows || lda % 4 || !aligned16(A) || ldb % 4 || !aligned16(B) || nsplit_for(K) * kRows * kCT * 4 > INT32_MAX / 2) {
    set_error("gcnk_gemm_smallm_f32: unsupported (M=%d <= 64, lda %% 4, ldb %% 4, 16-B aligned A and B)", M);
    return GCNK_EUNSUP;
  }
  const int64_t need = gcnk_gemm_smallm_workspace_bytes(M, N, K), cneed = gcnk_gemm_smallm_counter_bytes(N);
  if (!workspace || workspace_bytes < need || !counters || counter_bytes < cneed) {
    set_error("gcnk_gemm_smallm_f32: needs %lld B of workspace and a zeroed counter region of %lld B",
              (long long)need, (long long)cneed);
    return GCNK_EARG;
  }
  const int kch = pick_kch(K);
  const int32_t nsplit = (int32_t)((K + 16 * kch - 1) / (16 * kch));
  const int32_t nct = (N + kCT - 1) / kCT;
  const dim3 grid((unsigned)(nct * nsplit));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define GCNK_SMALLM(KCH_)                                                                                     \
  hipLaunchKernelGGL((gemm_smallm_onepass_kernel<KCH_>), grid, dim3(256), 0, s, M, N, K, nsplit, A, lda, B, ldb, C, \
                     ldc, accumulate, workspace, counters)
  switch (kch) {
    case 4: GCNK_SMALLM(4); break;
    case 6: GCNK_SMALLM(6); break;
    case 8: GCNK_SMALLM(8); break;
    case 12: GCNK_SMALLM(12); break;
    case 16: GCNK_SMALLM(16); break;
    case 24: GCNK_SMALLM(24); break;
    default: GCNK_SMALLM(32); break;
  }
#undef GCNK_SMALLM
  return launch_check("gemm_smallm_onepass_kernel");
}
