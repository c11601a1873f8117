// S_T = X_hubs W1: the hub rows of gc1's support (reference layer.py:102,
// th.spmm(infeatn, W) restricted to the rows the factored gc1 needs, factor.py).
//
// R8: 50 hub rows, K = 7,463 features, F = 200: the product reads all of W1
// (6 MB) and X_hubs (1.5 MB) once and writes 40 KB -- a short, wide
// reduction.  One launch, no slab-reduce kernel:
//
//  * grid = T column tiles (32 columns = two 16-wide MFMA n-tiles) x S K-slabs;
//    a slab's T workgroups sit on one XCD (blockIdx % 8 == slab % 8), so that
//    XCD's L2 serves the slab's X_hubs piece to all of them;
//  * a workgroup's 4 waves take interleaved 16-deep k-blocks of its slab, all
//    64 (padded) hub rows x 32 columns on v_mfma_f32_16x16x4_f32, A = X_hubs
//    rows as 16-B loads, B = W1 rows; the waves' tiles meet in LDS in wave
//    order;
//  * the slabs' partial tiles are summed by deterministic last-arriver
//    hand-offs in two levels (groups of G slabs, then the NG group sums), all
//    in a fixed order: bitwise reproducible, no float atomics.  Hand-off form
//    as csrc/spmm.hip's heavy rows: every store and load of a partial coherent
//    (sc1), each storing wave drained before one lane's agent-scope add, the
//    last adder reading only after its add returned.
#include "gcnk_common.h"

#include <algorithm>

namespace gcnk {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRows = 64;        // padded hub rows (4 MFMA row tiles)
constexpr int kCols = 32;        // columns per workgroup (2 MFMA n-tiles)
constexpr int kTileF = kRows * kCols;
constexpr int kKB = 16;          // k per block (4 MFMA steps)
constexpr int kWaves = 4;
constexpr int kNB = 4;          // k-blocks per wave loaded together
// arrival counters kCntStride words (256 B) apart: agent-scope atomics resolve
// past the per-XCD L2s, and a few hundred of them on one line serialise
constexpr int kCntStride = 64;
constexpr int kMaxG = 8;        // partials per hand-off level (loaded together): S <= 64

struct HubXW {
  const float* X;  // [H x >= roundup4(K)] zero past K
  int64_t ldx;
  const float* W;  // [K x F]
  int64_t ldw;
  float* out;      // S_T [H x F]
  int64_t ldo;
  float* part1;    // [S][T] tiles
  float* part2;    // [NG][T] tiles
  int32_t* cnt;    // [T][NG] group counters, then [T] final counters, kCntStride words apart
  int32_t H, K, F, T, S, Ks, G, NG;
};

// a wave-uniform pointer in SGPRs (the buffer resource must be scalar)
__device__ __forceinline__ float* uni(float* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return reinterpret_cast<float*>(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void st_sc1(float* base, int off, const float4& v) {
  const f32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000),
                                         off * 4, 0, 16);
}
__device__ __forceinline__ float4 ld_sc1(const float* base, int off) {
  const f32x4 x = __builtin_amdgcn_raw_buffer_load_b128(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000), off * 4, 0, 16);
  return make_float4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

// One thread's 8 values of a 64 x 32 tile in "tile order": float4 j of thread
// tid is tile element (tid + 256 j) * 4 .. +3, j = 0, 1 (row-major 64 x 32).
__global__ void __launch_bounds__(256) hub_xw_kernel(HubXW a) {
  __shared__ float4 s_red[kWaves][kTileF / 4 / 1];  // 4 x 512 float4 = 32 KB
  __shared__ int s_flag;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // blockIdx -> (slab, column tile): slab % 8 == blockIdx % 8
  const int b = blockIdx.x, xcd = b & 7, i = b >> 3;
  const int t = i % a.T, s = xcd + 8 * (i / a.T);
  if (s >= a.S) return;  // grid rounds S up to a multiple of 8: whole workgroups exit
  const int k_beg = s * a.Ks, k_end = min(a.K, k_beg + a.Ks);
  const int n0 = t * kCols;

  f32x4 acc[4][2];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[r][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int li = lane & 15, kq = lane >> 4;
  const bool colok0 = n0 + li < a.F, colok1 = n0 + 16 + li < a.F;
  // all of a wave's k-blocks (up to kNB per round; one round at the slab
  // sizes hub_xw_shape picks) are loaded before the first MFMA, so the wave
  // waits for one round of load latency, not one per block
  for (int kb0 = k_beg + kKB * w; kb0 < k_end; kb0 += kKB * kWaves * kNB) {
    float4 xa[kNB][4];
    float wb[kNB][4][2];
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb) {
      const int kx = kb0 + kKB * kWaves * nb + 4 * kq;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * r + li;
        xa[nb][r] = (row < a.H && kx < k_end) ? *reinterpret_cast<const float4*>(a.X + (int64_t)row * a.ldx + kx)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = kx + j;
        const float* wr = a.W + (int64_t)k * a.ldw + n0 + li;
        wb[nb][j][0] = (k < k_end && colok0) ? wr[0] : 0.f;
        wb[nb][j][1] = (k < k_end && colok1) ? wr[16] : 0.f;
      }
    }
    // (X values past k_end -- only at K, inside the zero pad -- meet W zeros;
    // blocks wholly past k_end skip their MFMAs, a wave-uniform test)
#pragma unroll
    for (int nb = 0; nb < kNB; ++nb) {
      if (kb0 + kKB * kWaves * nb >= k_end) break;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float av = j == 0 ? xa[nb][r].x : j == 1 ? xa[nb][r].y : j == 2 ? xa[nb][r].z : xa[nb][r].w;
          acc[r][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, wb[nb][j][0], acc[r][0], 0, 0, 0);
          acc[r][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, wb[nb][j][1], acc[r][1], 0, 0, 0);
        }
    }
  }
  // C map of the 16x16 f32 MFMA: reg q -> row 4 * (lane >> 4) + q, col lane & 15.
  // Into LDS as the 64 x 32 row-major tile of this wave.
  float* sw = reinterpret_cast<float*>(s_red[w]);
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int q = 0; q < 4; ++q) sw[(16 * r + 4 * kq + q) * kCols + 16 * n + li] = acc[r][n][q];
  __syncthreads();
  float4 v[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int e = tid + 256 * j;
    v[j] = s_red[0][e];
#pragma unroll
    for (int u = 1; u < kWaves; ++u) add4(v[j], s_red[u][e]);
  }
  int32_t* cnt1 = a.cnt + (int64_t)t * a.NG * kCntStride;          // + g * kCntStride
  int32_t* cnt2 = a.cnt + ((int64_t)a.T * a.NG + t) * kCntStride;
  if (a.S > 1) {
    // level 1: publish this slab's tile; the group's last arriver sums the group's
    float* p1 = a.part1 + (int64_t)t * kTileF;  // slot (s, t) at p1 + s * T * kTileF
    const int64_t slot_ld = (int64_t)a.T * kTileF;
#pragma unroll
    for (int j = 0; j < 2; ++j) st_sc1(uni(p1 + s * slot_ld), 4 * (tid + 256 * j), v[j]);
    const int g = s / a.G, g0 = g * a.G, gn = min(a.S, g0 + a.G) - g0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores have completed
    __syncthreads();
    if (tid == 0) s_flag = __hip_atomic_fetch_add(cnt1 + g * kCntStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gn - 1;
    __syncthreads();
    if (!s_flag) return;
    if (tid == 0) __hip_atomic_store(cnt1 + g * kCntStride, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every partial of the group loaded before the first add (one latency), then summed in order
    float4 gs[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    {
      float4 pv[kMaxG][2];
#pragma unroll
      for (int u = 0; u < kMaxG; ++u)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          pv[u][j] = u < gn ? ld_sc1(uni(p1 + (g0 + u) * slot_ld), 4 * (tid + 256 * j)) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < kMaxG; ++u)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (u < gn) add4(gs[j], pv[u][j]);
    }
    if (a.NG > 1) {
      // level 2: publish the group sum; the last group sums the groups in order
      float* p2 = a.part2 + (int64_t)t * kTileF;
#pragma unroll
      for (int j = 0; j < 2; ++j) st_sc1(uni(p2 + g * slot_ld), 4 * (tid + 256 * j), gs[j]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) s_flag = __hip_atomic_fetch_add(cnt2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.NG - 1;
      __syncthreads();
      if (!s_flag) return;
      if (tid == 0) __hip_atomic_store(cnt2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int j = 0; j < 2; ++j) gs[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      float4 pv[kMaxG][2];
#pragma unroll
      for (int u = 0; u < kMaxG; ++u)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          pv[u][j] = u < a.NG ? ld_sc1(uni(p2 + u * slot_ld), 4 * (tid + 256 * j)) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < kMaxG; ++u)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (u < a.NG) add4(gs[j], pv[u][j]);
    }
    v[0] = gs[0];
    v[1] = gs[1];
  }
  // the finished 64 x 32 tile: rows < H, columns < F
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int e = 4 * (tid + 256 * j), row = e / kCols, col = n0 + e % kCols;
    if (row >= a.H) continue;
    float* o = a.out + (int64_t)row * a.ldo + col;
    const float f[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (col + c < a.F) o[c] = f[c];
  }
}

struct Shape {
  int T, S, Ks, G, NG;
};

Shape hub_xw_shape(int32_t K, int32_t F) {
  Shape sh;
  sh.T = (F + kCols - 1) / kCols;
  // about 256 workgroups (one per CU), S a multiple of 8 (whole XCD rounds),
  // at most kMaxG^2 slabs (two hand-off levels of at most kMaxG partials)
  int S = (256 + sh.T - 1) / sh.T;
  S = std::min((S + 7) / 8 * 8, kMaxG * kMaxG);
  int Ks = ((K + S - 1) / S + kKB - 1) / kKB * kKB;
  if (Ks < kKB * kWaves) Ks = kKB * kWaves;
  sh.Ks = Ks;
  sh.S = (K + Ks - 1) / Ks;
  int G = 1;
  while (G * G < sh.S) ++G;
  if (G > kMaxG) G = kMaxG;
  sh.G = G;
  sh.NG = (sh.S + G - 1) / G;
  return sh;
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int64_t gcnk_hub_xw_workspace_bytes(int32_t H, int32_t K, int32_t F) {
  if (H <= 0 || H > kRows || K <= 0 || F <= 0) return GCNK_EARG;
  const Shape sh = hub_xw_shape(K, F);
  const int64_t tiles = (int64_t)(sh.S + sh.NG) * sh.T * kTileF * 4;
  return tiles + (int64_t)sh.T * (sh.NG + 1) * kCntStride * 4;
}

extern "C" int gcnk_hub_xw_f32(int32_t H, int32_t K, int32_t F, const float* X, int64_t ldx, const float* W,
                               int64_t ldw, float* S, int64_t lds, void* workspace, int64_t workspace_bytes,
                               void* stream) {
  if (H <= 0 || K <= 0 || F <= 0 || !X || !W || !S || ldw < F || lds < F) {
    set_error("gcnk_hub_xw_f32: bad sizes or null operand (H=%d K=%d F=%d)", H, K, F);
    return GCNK_EARG;
  }
  if (H > kRows || ldx < ((K + 3) & ~3) || ldx % 4 || !aligned16(X)) {
    set_error("gcnk_hub_xw_f32: unsupported operand (H=%d <= 64, ldx=%lld >= K rounded to 4, 16-B X rows)", H,
              (long long)ldx);
    return GCNK_EUNSUP;
  }
  const Shape sh = hub_xw_shape(K, F);
  const int64_t need = gcnk_hub_xw_workspace_bytes(H, K, F);
  if (!workspace || workspace_bytes < need || !aligned16(workspace)) {
    set_error("gcnk_hub_xw_f32: workspace of %lld B needed (16-B aligned, counters zeroed once)", (long long)need);
    return GCNK_EARG;
  }
  HubXW a;
  a.X = X; a.ldx = ldx; a.W = W; a.ldw = ldw; a.out = S; a.ldo = lds;
  a.part1 = static_cast<float*>(workspace);
  a.part2 = a.part1 + (int64_t)sh.S * sh.T * kTileF;
  a.cnt = reinterpret_cast<int32_t*>(a.part2 + (int64_t)sh.NG * sh.T * kTileF);
  a.H = H; a.K = K; a.F = F; a.T = sh.T; a.S = sh.S; a.Ks = sh.Ks; a.G = sh.G; a.NG = sh.NG;
  const int s8 = (sh.S + 7) / 8 * 8;
  hipLaunchKernelGGL(hub_xw_kernel, dim3((unsigned)(s8 * sh.T)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  return launch_check("hub_xw_kernel");
}
