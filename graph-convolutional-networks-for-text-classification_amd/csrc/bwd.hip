// Fused backward of gc2 and of gc1's ReLU + dropout (the autograd of
// reference layer.py:182-188 through layer.py:102-110, run by trainer.py:361):
//
//   gZ1[m, n] = H1[m, n] > 0 ? scale * (gS2[m, :] . W2[n, :]) : 0     [M x N]
//   gW2[n, p] = sum_m H1[m, n] gS2[m, p]                              [N x P]
//   gb1[n]    = sum_m gZ1[m, n]                                       [N]
//   gb2[p]    = sum_m G[m, p]          (optional)                     [P]
//
// with gS2 = A^T G computed before (spmm).  H1 is gc1's stored output (after
// ReLU and dropout), so H1 > 0 <=> kept and positive, and the scale is the
// dropout's 1/(1-p) (1 in eval / without dropout): ATen's mm(gS2, W2^T), mul
// by the dropout noise, threshold_backward and the two bias sums in one
// pass over H1 instead of a K = 8 GEMM, a split-K GEMM + its reduce and two
// two-pass column sums (profiles/r03_train_breakdown.json: 48 us of 85 us of
// the step's gcnk kernels).
//
// Kernel 1 (gcn_bwd2_kernel): one workgroup per run of rows x a 256-column
// slice.  Lane (rl, cu): column unit cu (VEC columns), rows rl, rl + RL, ...
// The lane's first batch of H1 rows is loaded before the rows' gS2 (and G)
// values are staged in LDS once (the two loads share one latency); each lane keeps its
// columns' W2 rows in registers, writes gZ1 and accumulates its columns' gW2 /
// gb1 terms in row order; the RL row lanes are then summed through LDS in
// lane order and the workgroup's partial goes to the workspace.
// Kernel 2 (gcn_bwd2_reduce_kernel): every output sums the workgroups'
// partials in workgroup order.  Fixed order everywhere: bitwise reproducible.
#include "gcnk_common.h"

#include <algorithm>

namespace gcnk {
namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr int kBwdBlock = 256;
constexpr int kBwdCols = 256;      // columns per workgroup slice
constexpr int kBwdRowsMax = 256;   // rows per workgroup (LDS staging of gS2 / G)
constexpr int kBwdBatch = 8;       // rows per lane whose H1 loads are in flight together
#ifndef GCNK_BWD_TARGET
#define GCNK_BWD_TARGET 256
#endif
constexpr int kBwdTarget = GCNK_BWD_TARGET;    // workgroups per slice (256: one per CU)
// 1 (default): the row lanes' gW2 / gb1 partials summed as float4 pieces where P == PM
#ifndef GCNK_BWD2_VSUM
#define GCNK_BWD2_VSUM 1
#endif
#ifndef GCNK_BWD2_STAMPV   // stamps-build timeline variant (2: around the lane sum)
#define GCNK_BWD2_STAMPV 1
#endif

template <int VEC>
struct VecIO;
template <>
struct VecIO<4> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[4]) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
  // streaming store (gZ1: written once, read by the next launch)
  static __device__ __forceinline__ void store_nt(float* p, const float (&v)[4]) {
    typedef float f4a __attribute__((ext_vector_type(4), aligned(16)));
    __builtin_nontemporal_store(f4a{v[0], v[1], v[2], v[3]}, reinterpret_cast<f4a*>(p));
  }
};
template <>
struct VecIO<2> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[2]) {
    const float2 x = *reinterpret_cast<const float2*>(p);
    v[0] = x.x; v[1] = x.y;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[2]) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  }
  static __device__ __forceinline__ void store_nt(float* p, const float (&v)[2]) {
    __builtin_nontemporal_store(v[0], p);
    __builtin_nontemporal_store(v[1], p + 1);
  }
};
template <>
struct VecIO<1> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[1]) { v[0] = *p; }
  static __device__ __forceinline__ void store(float* p, const float (&v)[1]) { *p = v[0]; }
  static __device__ __forceinline__ void store_nt(float* p, const float (&v)[1]) { __builtin_nontemporal_store(v[0], p); }
};

struct Bwd2Args {
  const float* H; int64_t ldh;
  const float* gS; int64_t ldgs;
  const float* W; int64_t ldw;
  const float* G; int64_t ldg;
  int32_t M, N, P;
  float scale;
  float* Z; int64_t ldz;
  float* part; int64_t part_ld;   // per workgroup row: gW2 [N*P] | gb1 [N] | gb2 [P]
  int32_t rpb;                    // rows per workgroup
  Epi stamps;                     // (debug timeline of a -DGCNK_STAMPS build only: .stamps)
};

template <int VEC, int PM>
__global__ void __launch_bounds__(kBwdBlock) gcn_bwd2_kernel(Bwd2Args a) {
  constexpr int KE = VEC * (PM + 1);  // accumulators per lane: gW2 terms + gb1
  __shared__ __attribute__((aligned(16))) float s_g[kBwdRowsMax * PM];
  __shared__ float s_gg[kBwdRowsMax * PM];
  __shared__ float s_red[kBwdBlock * KE];
  const int tid = threadIdx.x;
  const int32_t units = (a.N + VEC - 1) / VEC;
  const int32_t cu0 = (int32_t)blockIdx.y * (kBwdCols / VEC);
  const int CT = min(units - cu0, kBwdCols / VEC);  // column units of this slice (>= 1)
  const int RL = kBwdBlock / CT;                    // row lanes
  const int rl = tid / CT, cu = tid % CT;
  const bool act = rl < RL;
  const int64_t c = (int64_t)(cu0 + cu) * VEC;
  const int32_t r0 = (int32_t)blockIdx.x * a.rpb;
  const int32_t nr = min(a.M - r0, a.rpb);
  const bool with_g = a.G != nullptr && blockIdx.y == 0;
  const bool colok = act && c < a.N;  // VEC columns all valid (N % VEC == 0 on the vector paths)
  stamp(a.stamps, 0);   // (stamps build: 0 entry, 1 operands staged, 2 rows done, 3 partial stored)

  // the first batch's H1 rows: in flight together with the staging loads below
  float h[kBwdBatch][VEC];
#pragma unroll
  for (int j = 0; j < kBwdBatch; ++j) {
    const int32_t rr = rl + j * RL;
    if (colok && rr < nr) VecIO<VEC>::load(a.H + (int64_t)(r0 + rr) * a.ldh + c, h[j]);
    else
#pragma unroll
      for (int v = 0; v < VEC; ++v) h[j][v] = 0.f;
  }
  // gS2 (and G) rows of the workgroup -> LDS, padded to PM columns with zeros.
  // Unpadded contiguous rows (P == PM == ld, R8): LDS-DMA, no register round
  // trip before the barrier (a load -> LDS store pair waits on its load)
  const bool g_dma = a.P == PM && a.ldgs == PM && (!with_g || a.ldg == PM);
  if (g_dma) {
    const int n = nr * PM, lane = tid & 63;
    for (int e0 = tid & ~63; e0 < n; e0 += kBwdBlock) {   // (wave-uniform base)
      if (e0 + lane < n) {
        lds_dma4(a.gS + (int64_t)r0 * PM + e0 + lane, s_g + e0);
        if (with_g) lds_dma4(a.G + (int64_t)r0 * PM + e0 + lane, s_gg + e0);
      }
    }
  } else {
    for (int i = tid; i < nr * PM; i += kBwdBlock) {
      const int rr = i / PM, p = i % PM;
      s_g[i] = p < a.P ? a.gS[(int64_t)(r0 + rr) * a.ldgs + p] : 0.f;
      if (with_g) s_gg[i] = p < a.P ? a.G[(int64_t)(r0 + rr) * a.ldg + p] : 0.f;
    }
  }
  // this lane's columns of W2 (rows of W2: W2[n, :]).  (Issued before the
  // staging above instead: staging 2.7 -> 4.2 us, profiles/r04_bwd2_stamps_v2.log.)
  // (W2 rows are ldw apart; with ldw == P == PM a lane's VEC rows are one run
  // of VEC PM floats: 16-B loads instead of VEC PM 4-B loads 32 lanes apart)
  float w[VEC][PM];
  if (a.ldw == PM && a.P == PM && (reinterpret_cast<uintptr_t>(a.W) & 15) == 0) {
    // (clamped row, value masked by bits: the guarded load compiled to a branch
    // per load with its own vmcnt(0) -- eight serialised round trips)
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const bool ok = act && c + v < a.N;
      const int m = ok ? -1 : 0;
      const float* wr = a.W + (ok ? c + v : 0) * a.ldw;
#pragma unroll
      for (int p = 0; p < PM; p += 4) {
        const float4 q = *reinterpret_cast<const float4*>(wr + p);
        w[v][p] = __int_as_float(__float_as_int(q.x) & m); w[v][p + 1] = __int_as_float(__float_as_int(q.y) & m);
        w[v][p + 2] = __int_as_float(__float_as_int(q.z) & m); w[v][p + 3] = __int_as_float(__float_as_int(q.w) & m);
      }
    }
  } else {
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
      for (int p = 0; p < PM; ++p)
        w[v][p] = (act && c + v < a.N && p < a.P) ? a.W[(c + v) * a.ldw + p] : 0.f;
  }
  float gw[VEC][PM], gb[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    gb[v] = 0.f;
#pragma unroll
    for (int p = 0; p < PM; ++p) gw[v][p] = 0.f;
  }
  if (g_dma) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's DMA (and loads) landed
  __syncthreads();
#if GCNK_BWD2_STAMPV != 2
  stamp(a.stamps, 1);
#endif

  for (int32_t b0 = rl; b0 < nr; b0 += RL * kBwdBatch) {
    // the batch's H1 loads first (one latency; the first batch's are in flight
    // since entry), then the rows in order
    if (b0 != rl) {
#pragma unroll
      for (int j = 0; j < kBwdBatch; ++j) {
        const int32_t rr = b0 + j * RL;
        if (colok && rr < nr) VecIO<VEC>::load(a.H + (int64_t)(r0 + rr) * a.ldh + c, h[j]);
        else
#pragma unroll
          for (int v = 0; v < VEC; ++v) h[j][v] = 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < kBwdBatch; ++j) {
      const int32_t rr = b0 + j * RL;
      if (!colok || rr >= nr) break;
      float g[PM];
#pragma unroll
      for (int p = 0; p < PM; p += 4) {
        const float4 q = *reinterpret_cast<const float4*>(s_g + rr * PM + p);
        g[p] = q.x; g[p + 1] = q.y; g[p + 2] = q.z; g[p + 3] = q.w;
      }
      float z[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        float dot = 0.f;
#pragma unroll
        for (int p = 0; p < PM; ++p) dot = fmaf(g[p], w[v][p], dot);
        z[v] = h[j][v] > 0.f ? dot * a.scale : 0.f;
        gb[v] += z[v];
#pragma unroll
        for (int p = 0; p < PM; ++p) gw[v][p] = fmaf(h[j][v], g[p], gw[v][p]);
      }
      // gZ1 streamed out (nontemporal: no dirty L2 lines left at the kernel's end)
      VecIO<VEC>::store_nt(a.Z + (int64_t)(r0 + rr) * a.ldz + c, z);
    }
  }

#if GCNK_BWD2_STAMPV == 2
  stamp(a.stamps, 1);   // (variant timeline: 1 rows done, 2 after the lane-sum barrier, 3 partial stored)
#else
  stamp(a.stamps, 2);
#endif
  float* prow = a.part + (int64_t)blockIdx.x * a.part_ld;
#if GCNK_BWD2_VSUM
  // P == PM with 16-B partial rows: the thread's VEC x PM gW2 terms then its VEC
  // gb1 terms as float4 pieces in LDS, each output float4 (8 of gW2 + 1 of gb1
  // per column unit) summed over the row lanes in lane order and stored as one
  // 16-B piece -- the partial's layout in global memory is unchanged (gW2
  // [N x P] row-major | gb1 [N] | gb2 [P]).  (The per-float form below spends
  // ~7 dword iterations of index math, eight LDS reads and a 4-B store per
  // element: the phase measured ~3.7 us at R8, profiles/r05_bwd2_stamps_v2.log.)
  if (VEC == 4 && a.P == PM && (a.part_ld & 3) == 0 && (a.N * a.P) % 4 == 0) {
    constexpr int KE4 = KE / 4;   // VEC (PM + 1) / 4 float4 per thread (PM % 4 == 0)
    f32x4v* mine = reinterpret_cast<f32x4v*>(s_red) + tid * KE4;
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
      for (int p = 0; p < PM; p += 4) mine[(v * PM + p) / 4] = f32x4v{gw[v][p], gw[v][p + 1], gw[v][p + 2], gw[v][p + 3]};
#pragma unroll
    for (int v = 0; v < VEC; v += 4) {
      f32x4v g4;
#pragma unroll
      for (int i = 0; i < 4; ++i) g4[i] = v + i < VEC ? gb[v + i] : 0.f;
      mine[(VEC * PM + v) / 4] = g4;
    }
    __syncthreads();
#if GCNK_BWD2_STAMPV == 2
    stamp(a.stamps, 2);
#endif
    const f32x4v* red = reinterpret_cast<const f32x4v*>(s_red);
    for (int e = tid; e < CT * KE4; e += kBwdBlock) {
      const int u = e / KE4, k4 = e - u * KE4;
      f32x4v sum = red[u * KE4 + k4];
      for (int l = 1; l < RL; ++l) sum += red[(l * CT + u) * KE4 + k4];
      const int64_t c0 = (int64_t)(cu0 + u) * VEC;
      if (c0 >= a.N) continue;
      if (k4 < VEC * PM / 4) {   // gW2 rows c0 .. c0 + VEC - 1: VEC PM contiguous floats
        *reinterpret_cast<f32x4v*>(prow + c0 * a.P + 4 * k4) = sum;
      } else {                   // gb1 [c0 .. c0 + VEC): VEC floats
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (4 * (k4 - VEC * PM / 4) + i < VEC) prow[(int64_t)a.N * a.P + c0 + 4 * (k4 - VEC * PM / 4) + i] = sum[i];
      }
    }
  } else
#endif
  {
  // row lanes -> one partial per column, summed in lane order
  {
    float* mine = s_red + tid * KE;
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
#pragma unroll
      for (int p = 0; p < PM; ++p) mine[v * (PM + 1) + p] = gw[v][p];
      mine[v * (PM + 1) + PM] = gb[v];
    }
  }
  __syncthreads();
#if GCNK_BWD2_STAMPV == 2
  stamp(a.stamps, 2);
#endif
  for (int e = tid; e < CT * KE; e += kBwdBlock) {
    const int u = e / KE, k = e % KE;
    const int v = k / (PM + 1), p = k % (PM + 1);
    const int64_t col = (int64_t)(cu0 + u) * VEC + v;
    // the row lanes' values eight at a time (loads together), added in lane order
    float s = 0.f;
    // (clamped reads and selected adds: no branch per read, all eight in flight
    // behind one wait -- the guarded form compiled to a branch per read and took
    // ~2 us at R8's shape)
    for (int l0 = 0; l0 < RL; l0 += 8) {
      float rv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) rv[j] = s_red[(min(l0 + j, RL - 1) * CT + u) * KE + k];
#pragma unroll
      for (int j = 0; j < 8; ++j) s = l0 + j < RL ? s + rv[j] : s;
    }
    if (col >= a.N) continue;
    if (p < PM) {
      if (p < a.P) prow[col * a.P + p] = s;
    } else {
      prow[(int64_t)a.N * a.P + col] = s;
    }
  }
  }
  if (with_g && tid < a.P) {  // gb2: the G rows, in row order (eight LDS reads in flight)
    float s = 0.f;
    for (int r8 = 0; r8 < nr; r8 += 16) {
      float gv[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) gv[j] = s_gg[min(r8 + j, nr - 1) * PM + tid];
#pragma unroll
      for (int j = 0; j < 16; ++j) s = r8 + j < nr ? s + gv[j] : s;
    }
    prow[(int64_t)a.N * a.P + a.N + tid] = s;
  }
  stamp(a.stamps, 3);
}

// gW2 / gb1 / gb2 from the per-workgroup partials (side_reduce_body, gcnk_common.h)
__global__ void __launch_bounds__(256) gcn_bwd2_reduce_kernel(SideReduce r) {
  __shared__ float s[16][17];
  side_reduce_body(r, blockIdx.x, s);
}

struct Bwd2Geom {
  int vec, pm, slices, nblk, rpb;
  int64_t part_ld;
};

bool bwd2_geometry(int32_t M, int32_t N, int32_t P, bool vec4_ok, bool vec2_ok, Bwd2Geom& g) {
  if (P < 1 || P > 32 || N < 1 || M < 1) return false;
  g.pm = P <= 8 ? 8 : P <= 16 ? 16 : 32;
  g.vec = (g.pm <= 16 && vec4_ok) ? 4 : vec2_ok ? 2 : 1;
  const int units = (N + g.vec - 1) / g.vec;
  g.slices = (units + kBwdCols / g.vec - 1) / (kBwdCols / g.vec);
  g.rpb = (int)std::min<int64_t>(kBwdRowsMax, std::max<int64_t>(1, ((int64_t)M + kBwdTarget - 1) / kBwdTarget));
  g.nblk = (int)(((int64_t)M + g.rpb - 1) / g.rpb);
  g.part_ld = (((int64_t)N * P + N + P) + 3) & ~3LL;
  return true;
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int64_t gcnk_gcn_bwd2_workspace_bytes(int32_t M, int32_t N, int32_t P) {
  Bwd2Geom g;
  if (!bwd2_geometry(M, N, P, true, true, g)) return 0;
  return (int64_t)g.nblk * g.part_ld * 4;
}

int gcnk::side_reduce_launch(const SideReduce& side, void* stream) {
  hipLaunchKernelGGL(gcn_bwd2_reduce_kernel, dim3((unsigned)side_reduce_blocks(side)), dim3(256), 0,
                     (hipStream_t)stream, side);
  return launch_check("gcn_bwd2_reduce_kernel");
}

extern "C" int gcnk_gcn_bwd2_f32(const float* H, int64_t ldh, const float* gS, int64_t ldgs, const float* W,
                                 int64_t ldw, const float* G, int64_t ldg, int32_t M, int32_t N, int32_t P,
                                 float scale, float* Z, int64_t ldz, float* gW, float* gb1, float* gb2,
                                 void* workspace, int64_t workspace_bytes, void* stream) {
  SideReduce side;
  const int rc = gcn_bwd2_main(H, ldh, gS, ldgs, W, ldw, G, ldg, M, N, P, scale, Z, ldz, gW, gb1, gb2, workspace,
                               workspace_bytes, stream, &side);
  return rc ? rc : side_reduce_launch(side, stream);
}

int gcnk::gcn_bwd2_main(const float* H, int64_t ldh, const float* gS, int64_t ldgs, const float* W, int64_t ldw,
                        const float* G, int64_t ldg, int32_t M, int32_t N, int32_t P, float scale, float* Z,
                        int64_t ldz, float* gW, float* gb1, float* gb2, void* workspace, int64_t workspace_bytes,
                        void* stream, SideReduce* side) {
  if (M < 0 || N < 0 || P < 0) {
    set_error("gcnk_gcn_bwd2_f32: negative size (M=%d N=%d P=%d)", M, N, P);
    return GCNK_EARG;
  }
  if (P > 32) {
    set_error("gcnk_gcn_bwd2_f32: P = %d classes > 32 (use gcnk_gemm_f32 + gcnk_colsum_f32)", P);
    return GCNK_EUNSUP;
  }
  if (M == 0 || N == 0 || P == 0) {
    set_error("gcnk_gcn_bwd2_f32: empty operand (M=%d N=%d P=%d)", M, N, P);
    return GCNK_EUNSUP;
  }
  if (!H || !gS || !W || !Z || (G && ldg < P) || ldh < N || ldgs < P || ldw < P || ldz < N) {
    set_error("gcnk_gcn_bwd2_f32: null operand or leading dimension too small");
    return GCNK_EARG;
  }
  const bool v4 = N % 4 == 0 && ldh % 4 == 0 && ldz % 4 == 0 && aligned16(H) && aligned16(Z);
  const bool v2 = N % 2 == 0 && ldh % 2 == 0 && ldz % 2 == 0 && ((uintptr_t)H & 7u) == 0 && ((uintptr_t)Z & 7u) == 0;
  Bwd2Geom g;
  bwd2_geometry(M, N, P, v4, v2, g);
  const int64_t need = (int64_t)g.nblk * g.part_ld * 4;
  if (!workspace || workspace_bytes < need) {
    set_error("gcnk_gcn_bwd2_f32: workspace %lld B < %lld B", (long long)workspace_bytes, (long long)need);
    return GCNK_EARG;
  }
  Bwd2Args a{H, ldh, gS, ldgs, W, ldw, G, ldg, M, N, P, scale, Z, ldz, (float*)workspace, g.part_ld, g.rpb, Epi{}};
  a.stamps.stamps = debug_stamps();
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)g.nblk, (unsigned)g.slices);
#define GCNK_BWD2(V_, PM_) hipLaunchKernelGGL((gcn_bwd2_kernel<V_, PM_>), grid, dim3(kBwdBlock), 0, s, a)
  if (g.vec == 4) {
    if (g.pm == 8) GCNK_BWD2(4, 8);
    else GCNK_BWD2(4, 16);
  } else if (g.vec == 2) {
    if (g.pm == 8) GCNK_BWD2(2, 8);
    else if (g.pm == 16) GCNK_BWD2(2, 16);
    else GCNK_BWD2(2, 32);
  } else {
    if (g.pm == 8) GCNK_BWD2(1, 8);
    else if (g.pm == 16) GCNK_BWD2(1, 16);
    else GCNK_BWD2(1, 32);
  }
#undef GCNK_BWD2
  *side = SideReduce{(const float*)workspace, g.part_ld, g.nblk, N, P, G ? 1 : 0, gW, gb1, gb2};
  return launch_check("gcn_bwd2_kernel");
}
