// Hub plan: CSR SpMM for gfx950  C = epi(A_csr * B)  on graphs whose rows
// split into a few heavy "hub" rows and many light rows that reference only
// hub columns and themselves -- the reference's doc-topic adjacency
// (layer.py:106 th.spmm(adj, support); R8: 50 topic rows of 191..1807
// nonzeros, 7,674 document rows of 2..14 nonzeros, each a topic subset plus
// its own diagonal).
//
// Why this schedule.  Row by row, R8 A-hat at F = 200 gathers
// 69k B rows x 800 B = 55 MB from L2 into the CUs for a product whose
// compulsory traffic is 12.9 MB, and every gather waits behind a dependent
// load of its column index; the 50 topic rows (30,990 nonzeros) were cut into
// segments whose partials met through arrival counters, a chain of four
// dependent memory round trips that set the launch length.  Here:
//   * light rows are cut into G groups of consecutive rows (light row l of
//     the operand is row l below the hub range, l + H above it) and F into C
//     column slices; workgroup (g, c) copies, by LDS-DMA straight from
//     blockIdx arithmetic (no index load in front), the c-slices of its
//     group's B rows and of the H hub rows of B, plus the group's record of
//     the plan, into LDS -- every load of the launch is issued in its first
//     microseconds;
//   * it computes its light rows' c-slices from LDS (a light row references
//     hub rows and itself only) and stores them with the epilogue;
//   * it computes the hub rows TRANSPOSED from the same LDS image: hub t's
//     nonzeros over the group's rows (A[t, j] * B[j], j in the group) are one
//     partial c-slice per (hub, group).  Column slicing is what keeps these
//     few: G = 32 groups of 240 rows at F = 200 leave 32 partials per hub
//     (1.28 MB for R8), where one-row-group-per-CU would leave 256;
//   * hub x hub nonzeros ride along in the partial of group t % G;
//   * a second small kernel sums each hub row's G partials in group order and
//     applies the epilogue.
// Two launches; the kernel boundary is the only hand-off (plain stores, no
// counters, no atomics), so concurrent calls with different workspaces never
// interact, and every sum has a fixed order (bitwise reproducible).
// Workgroups (g, c) with equal g run on one XCD (blockIdx = c * G + g, G a
// multiple of 8 under round-robin placement): the 128-B lines that two
// adjacent column slices share are fetched from HBM into one L2.
#include "gcnk_common.h"

#include <algorithm>
#include <climits>
#include <mutex>
#include <vector>

namespace gcnk {
namespace {

#ifndef GCNK_HUB_BLOCK
#define GCNK_HUB_BLOCK 256
#endif
#ifndef GCNK_HUB_SLICE_VECS
#define GCNK_HUB_SLICE_VECS 8
#endif
constexpr int kGroupBlock = GCNK_HUB_BLOCK;      // threads per row-group workgroup
constexpr int kSliceVecs = GCNK_HUB_SLICE_VECS;  // column vectors per slice (launch choice)
constexpr int kSumBlock = 256;        // threads per hub-sum workgroup
constexpr int kMaxHub = 256;          // hub rows per plan
constexpr int kMaxGroupRows = 512;    // light rows per group
constexpr int kMaxSlices = 64;        // column slices per launch
constexpr int kLdsMax = 163840;       // gfx950: 160 KiB per workgroup
constexpr int kTargetBlocks = 256;    // row-group workgroups per launch (one per CU)

__host__ __device__ inline int64_t align4(int64_t x) { return (x + 3) & ~3LL; }

// ---------------------------------------------------------------------------
// Plan layout (int32 words):
//   header[16]: 0 magic 'GNH2'  1 M  2 K  3 lane groups (gcnk_spmm_groups)
//               4 G (row groups)  5 R (record stride, words)  6 H (hub rows)
//               7 h0 (first hub row)  8 nL (light rows)  9 nnz  10 gs (light
//               rows per group)  11 hub degree threshold  12 max items per
//               record  13..15 0
//   records[G][R]
// Record of group g (light rows l = g * gs + i, i < n):
//   0 n  1 nout (= n + H)  2 nitems  3 0
//   4 .. 4 + nout   item offsets: output k's items are [off[k], off[k + 1])
//                   (outputs 0..n-1: the light rows; n + t: hub t's partial)
//   o_it = align4(5 + nout):  items int2 {slot, value bits}, CSR column order;
//                   slot t < H: hub row h0 + t of B; slot H + i: light row i
//                   of the group (its own diagonal, or a hub's nonzero on it)
struct HubLayout {
  int64_t G, R, H, h0, nL, gs, total;
  explicit HubLayout(const int32_t* h) {
    G = h[4]; R = h[5]; H = h[6]; h0 = h[7]; nL = h[8]; gs = h[10];
    total = 16 + G * R;
  }
};

__device__ __forceinline__ int64_t light_row(int64_t l, int32_t h0, int32_t H) { return l < h0 ? l : l + H; }
inline int64_t light_row_host(int64_t l, int64_t h0, int64_t H) { return l < h0 ? l : l + H; }

// One 16-B LDS-DMA load per lane: global gsrc -> LDS at lds_wave + 16 * lane
// (lds_wave wave-uniform).  Asynchronous: covered by the wave's vmcnt.
__device__ __forceinline__ void lds_dma16(const void* gsrc, void* lds_wave) {
  __builtin_amdgcn_global_load_lds(const_cast<void*>(gsrc), (__attribute__((address_space(3))) void*)lds_wave, 16, 0, 0);
}
__device__ __forceinline__ void lds_dma4(const void* gsrc, void* lds_wave) {
  __builtin_amdgcn_global_load_lds(const_cast<void*>(gsrc), (__attribute__((address_space(3))) void*)lds_wave, 4, 0, 0);
}

// ---------------------------------------------------------------------------
// Row-group kernel.  Grid G * nslices, block (g, c) = (b % G, b / G).
// LDS: record [R words] | rows [(H + n) x w] vectors (slot-major) | bias [w].
template <int VEC>
__global__ void __launch_bounds__(kGroupBlock)
hub_group_kernel(const int32_t* __restrict__ recs, int32_t R, int32_t G, int32_t gs, int32_t h0, int32_t H, int32_t nL,
                 int32_t nslices, const float* __restrict__ B, int64_t ldb, int32_t F, float* __restrict__ C,
                 int64_t ldc, Epi epi, float* __restrict__ part, int64_t part_ld) {
  using V = Vec<VEC>;
  using T = typename V::T;
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];
  int32_t* s_rec = smem;
  T* s_rows = reinterpret_cast<T*>(smem + R);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int NW = kGroupBlock / 64;
  const int g = blockIdx.x % G, c = blockIdx.x / G;
  const int32_t Q = VEC == 4 ? F / 4 : F;  // column vectors of a row
  const int32_t q0 = (int32_t)((int64_t)c * Q / nslices), q1 = (int32_t)((int64_t)(c + 1) * Q / nslices);
  const int32_t w = q1 - q0;
  const int64_t l0 = (int64_t)g * gs;
  const int32_t n = (int32_t)min((int64_t)gs, (int64_t)nL - l0);
  stamp(epi, 0);

  // ---- every load of the workgroup, issued before any is waited for:
  //      the record (16-B pieces), then the slot rows' c-slices (slot-major,
  //      element e = s * w + j lands at s_rows[e])
  for (int32_t k = wv * 64; k < R / 4; k += NW * 64) {
    if (k + lane < R / 4) lds_dma16(recs + (int64_t)g * R + 4 * (int64_t)(k + lane), s_rec + 4 * k);
  }
  const int32_t ne = (H + n) * w;
  const float* Bc = B + (int64_t)q0 * VEC;
  for (int32_t e0 = wv * 64; e0 < ne; e0 += NW * 64) {
    const int32_t e = e0 + lane;
    if (e < ne) {
      const int32_t s = e / w, j = e - s * w;
      const int64_t row = s < H ? (int64_t)h0 + s : light_row(l0 + (s - H), h0, H);
      const float* src = Bc + row * ldb + (int64_t)j * VEC;
      if (VEC == 4)
        lds_dma16(src, s_rows + e0);
      else
        lds_dma4(src, s_rows + e0);
    }
  }
  // the bias slice, so the output loop issues no global load (one there would
  // make every iteration wait for all the stores issued before it)
  T* s_bias = s_rows + ne;
  if (epi.bias && tid < w) s_bias[tid] = V::load(epi.bias + (int64_t)(q0 + tid) * VEC);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(epi, 1);

  // ---- outputs: task e = o * w + j (output o, column vector j of the slice)
  const int32_t nout = s_rec[1];
  const int32_t o_it = (int32_t)align4(5 + nout);
  const int2* s_items = reinterpret_cast<const int2*>(s_rec + o_it);
  const int32_t nt = nout * w;
  for (int32_t e = tid; e < nt; e += kGroupBlock) {
    const int32_t o = e / w, j = e - o * w;
    const int32_t ib = s_rec[4 + o], ie = s_rec[5 + o];
    const T* col = s_rows + j;
    T acc = V::zero();
#pragma unroll 4
    for (int32_t k = ib; k < ie; ++k) {
      const int2 it = s_items[k];
      V::fma(acc, __int_as_float(it.y), col[it.x * w]);
    }
    const int64_t cv = (int64_t)(q0 + j) * VEC;
    if (o < n) {
      const int64_t row = light_row(l0 + o, h0, H);
      const T bv = epi.bias ? s_bias[j] : V::zero();
      V::store_aligned(C + row * ldc + cv, V::epi(epi, acc, bv, row, cv));
    } else {
      V::store_aligned(part + ((int64_t)(o - n) * G + g) * part_ld + cv, acc);
    }
  }
  stamp(epi, 2);
}

// Hub rows: C[h0 + t] = epi(sum over g of part[t][g] in group order).  Grid
// (H, column tiles of LQ vectors); PL = kSumBlock / LQ partial lanes, lane p
// sums groups [p G / PL, (p + 1) G / PL) in order, then a fixed-order LDS tree.
template <int VEC, int LQ>
__global__ void __launch_bounds__(kSumBlock)
hub_sum_kernel(const float* __restrict__ part, int64_t part_ld, int32_t G, int32_t h0, int32_t F,
               float* __restrict__ C, int64_t ldc, Epi epi) {
  using V = Vec<VEC>;
  using T = typename V::T;
  constexpr int PL = kSumBlock / LQ;
  constexpr int U = 8;
  __shared__ T s_red[PL][LQ];
  const int tid = threadIdx.x, p = tid / LQ, lq = tid % LQ;
  const int32_t t = blockIdx.x;
  const int32_t Q = VEC == 4 ? F / 4 : F;
  const int32_t j = blockIdx.y * LQ + lq;
  const bool ok = j < Q;
  const int64_t cv = (int64_t)(ok ? j : 0) * VEC;
  const T bv = (epi.bias && ok) ? V::load(epi.bias + cv) : V::zero();  // first: no wait behind the partials
  const int32_t g0 = (int32_t)((int64_t)p * G / PL), g1 = (int32_t)((int64_t)(p + 1) * G / PL);
  const float* p0 = part + (int64_t)t * G * part_ld + cv;
  T acc = V::zero();
  for (int32_t gb = g0; gb < g1; gb += U) {
    T pv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) pv[u] = V::load(p0 + (int64_t)min(gb + u, g1 - 1) * part_ld);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      T x = acc;
      V::add(x, pv[u]);
      if (gb + u < g1) acc = x;
    }
  }
  s_red[p][lq] = acc;
  __syncthreads();
#pragma unroll
  for (int s = PL / 2; s >= 1; s >>= 1) {
    if (p < s) V::add(s_red[p][lq], s_red[p + s][lq]);
    __syncthreads();
  }
  if (p == 0 && ok) {
    const int64_t row = (int64_t)h0 + t;
    V::store(C + row * ldc + cv, V::epi(epi, s_red[0][lq], bv, row, cv));
  }
}

// Column slices for a launch: about 8 vectors per slice (R8 F = 200: 7 slices
// of 7-8 float4), then more until the LDS image fits.
int64_t choose_slices(const HubLayout& L, int32_t Q, size_t vbytes, int64_t* lds_out) {
  int64_t c = std::max<int64_t>(1, std::min<int64_t>(kMaxSlices, (Q + kSliceVecs - 1) / kSliceVecs));
  for (; c <= std::min<int64_t>(Q, kMaxSlices); ++c) {
    const int64_t w = (Q + c - 1) / c;
    const int64_t lds = L.R * 4 + (L.H + L.gs + 1) * w * (int64_t)vbytes;
    if (lds <= kLdsMax) {
      *lds_out = lds;
      return c;
    }
  }
  return -1;
}

template <int VEC, int LQ>
int launch_sum(const float* part, int64_t part_ld, const HubLayout& L, int32_t F, float* C, int64_t ldc, const Epi& e,
               hipStream_t s) {
  const int32_t Q = VEC == 4 ? F / 4 : F;
  hipLaunchKernelGGL((hub_sum_kernel<VEC, LQ>), dim3((unsigned)L.H, (unsigned)((Q + LQ - 1) / LQ)), dim3(kSumBlock), 0,
                     s, part, part_ld, (int32_t)L.G, (int32_t)L.h0, F, C, ldc, e);
  return launch_check("hub_sum_kernel");
}

template <int VEC>
int hub_launch(const int32_t* plan, const HubLayout& L, const float* B, int64_t ldb, int32_t F, float* C, int64_t ldc,
               const Epi& e, float* part, int64_t part_ld, hipStream_t s) {
  const int32_t Q = VEC == 4 ? F / 4 : F;
  int64_t lds = 0;
  const int64_t nslices = choose_slices(L, Q, sizeof(typename Vec<VEC>::T), &lds);
  if (nslices < 0 || L.G * nslices > INT32_MAX) {
    set_error("gcnk_spmm (hub plan): F = %d does not fit %lld hub + %lld group rows of LDS", F, (long long)L.H,
              (long long)L.gs);
    return GCNK_EUNSUP;
  }
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hub_group_kernel<VEC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax);
  });
  hipLaunchKernelGGL((hub_group_kernel<VEC>), dim3((unsigned)(L.G * nslices)), dim3(kGroupBlock), (size_t)lds, s,
                     plan + 16, (int32_t)L.R, (int32_t)L.G, (int32_t)L.gs, (int32_t)L.h0, (int32_t)L.H, (int32_t)L.nL,
                     (int32_t)nslices, B, ldb, F, C, ldc, e, part, part_ld);
  int rc = launch_check("hub_group_kernel");
  if (rc) return rc;
  Epi eb = e;  // debug stamps of the sum kernel follow the group kernel's
  if (eb.stamps) eb.stamps += 4 * L.G * nslices;
  if (Q > 32) return launch_sum<VEC, 64>(part, part_ld, L, F, C, ldc, eb, s);
  if (Q > 16) return launch_sum<VEC, 32>(part, part_ld, L, F, C, ldc, eb, s);
  if (Q > 8) return launch_sum<VEC, 16>(part, part_ld, L, F, C, ldc, eb, s);
  if (Q > 4) return launch_sum<VEC, 8>(part, part_ld, L, F, C, ldc, eb, s);
  if (Q > 2) return launch_sum<VEC, 4>(part, part_ld, L, F, C, ldc, eb, s);
  return launch_sum<VEC, 2>(part, part_ld, L, F, C, ldc, eb, s);
}

}  // namespace

// ---------------------------------------------------------------------------
// Host plan.  Returns GCNK_OK with `img` filled, 1 when the operand does not
// have the structure (the caller builds the row-unit plan), or a negative
// error code.  Structure: square; the rows of degree >= the hub threshold form
// ONE contiguous range of at most kMaxHub rows; every other row's nonzeros lie
// in hub columns or on its own diagonal.
int hub_plan_host(const int32_t* rp, const int32_t* ci, const float* vv, int32_t M, int32_t K, int64_t nnz,
                  int32_t groups, int32_t hub_min, int32_t block_rows, std::vector<int32_t>& img) {
  if (M <= 0 || nnz <= 0 || hub_min < 0 || M != K || groups <= 0) return 1;
  // hub threshold: 8x the mean degree, at least 64 nonzeros (R8 A-hat: mean 9,
  // threshold 72: the 50 topic rows, 191..1807 nonzeros; uniform 1M/20M: mean
  // 20, threshold 160, max degree ~45: no hubs)
  const int64_t hmin = hub_min == 0 ? std::max<int64_t>(64, 8 * ((nnz + M - 1) / M)) : hub_min;
  int64_t h0 = -1, h1 = -1;
  for (int32_t r = 0; r < M; ++r) {
    if ((int64_t)rp[r + 1] - rp[r] < hmin) continue;
    if (h0 < 0) {
      h0 = r;
    } else if (r != h1) {
      return 1;  // hubs not contiguous
    }
    h1 = r + 1;
  }
  if (h0 < 0) return 1;
  const int64_t H = h1 - h0, nL = (int64_t)M - H;
  if (H > kMaxHub || nL <= 0) return 1;
  auto is_hub = [&](int64_t c) { return c >= h0 && c < h1; };
  auto light_index = [&](int64_t c) { return c < h0 ? c : c - H; };
  for (int64_t l = 0; l < nL; ++l) {
    const int64_t r = l < h0 ? l : l + H;
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k)
      if (!is_hub(ci[k]) && ci[k] != r) return 1;  // a light row references another light row
  }
  // rows per group: the lane-group count says the width class the plan serves
  // (gcnk_spmm_groups: 1 = F > 128, wider at narrow F); about 256 workgroups per
  // launch with the slice count the launch picks (8 vectors per slice)
  int64_t gs;
  if (block_rows > 0) {
    gs = block_rows;
  } else {
    const int64_t lpr = 64 / groups;                          // ~ column vectors per row
    const int64_t c_exp = std::max<int64_t>(1, std::min<int64_t>(8, (lpr + kSliceVecs - 1) / kSliceVecs));
    int64_t G0 = std::max<int64_t>(8, (kTargetBlocks / c_exp + 7) / 8 * 8);
    gs = (nL + G0 - 1) / G0;
  }
  gs = std::max<int64_t>(1, std::min<int64_t>(gs, kMaxGroupRows));
  const int64_t G = (nL + gs - 1) / gs;

  // hub nonzeros bucketed by group: light columns by the group that owns them,
  // hub x hub columns by t % G; CSR (column) order within a bucket
  std::vector<std::vector<int64_t>> hub_k((size_t)(G * H));
  for (int64_t t = 0; t < H; ++t) {
    const int64_t r = h0 + t;
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
      const int64_t cidx = ci[k];
      const int64_t g = is_hub(cidx) ? t % G : light_index(cidx) / gs;
      hub_k[(size_t)(g * H + t)].push_back(k);
    }
  }
  std::vector<std::vector<int32_t>> recs((size_t)G);
  int64_t R = 4, max_items = 0;
  for (int64_t g = 0; g < G; ++g) {
    const int64_t l0 = g * gs, n = std::min(gs, nL - l0), nout = n + H;
    int64_t nit = 0;
    for (int64_t i = 0; i < n; ++i) {
      const int64_t r = light_row_host(l0 + i, h0, H);
      nit += (int64_t)rp[r + 1] - rp[r];
    }
    for (int64_t t = 0; t < H; ++t) nit += (int64_t)hub_k[(size_t)(g * H + t)].size();
    const int64_t o_it = align4(5 + nout);
    std::vector<int32_t>& w = recs[(size_t)g];
    w.assign((size_t)align4(o_it + 2 * nit), 0);
    w[0] = (int32_t)n;
    w[1] = (int32_t)nout;
    w[2] = (int32_t)nit;
    int64_t it = 0;
    auto item = [&](int64_t col, int64_t k) {
      const int64_t slot = is_hub(col) ? col - h0 : H + (light_index(col) - l0);
      w[(size_t)(o_it + 2 * it)] = (int32_t)slot;
      w[(size_t)(o_it + 2 * it + 1)] = vv ? __builtin_bit_cast(int32_t, vv[k]) : 0;
      ++it;
    };
    for (int64_t i = 0; i < n; ++i) {
      const int64_t r = light_row_host(l0 + i, h0, H);
      w[(size_t)(4 + i)] = (int32_t)it;
      for (int64_t k = rp[r]; k < rp[r + 1]; ++k) item(ci[k], k);
    }
    for (int64_t t = 0; t < H; ++t) {
      w[(size_t)(4 + n + t)] = (int32_t)it;
      for (int64_t k : hub_k[(size_t)(g * H + t)]) item(ci[k], k);
    }
    w[(size_t)(4 + nout)] = (int32_t)it;
    R = std::max<int64_t>(R, (int64_t)w.size());
    max_items = std::max(max_items, nit);
  }
  R = align4(R);
  const int64_t words = 16 + G * R;
  if (words >= INT32_MAX || R * 4 > kLdsMax / 2) {
    if (hub_min == 0) return 1;
    set_error("gcnk_spmm_plan (hub): a group record of %lld words does not fit LDS (rows per group %lld)",
              (long long)R, (long long)gs);
    return GCNK_EUNSUP;
  }
  img.assign((size_t)words, 0);
  const int32_t hdr[16] = {kHubMagic,       M,           K,           groups,   (int32_t)G, (int32_t)R,
                           (int32_t)H,      (int32_t)h0, (int32_t)nL, (int32_t)nnz,       (int32_t)gs,
                           (int32_t)hmin,   (int32_t)max_items, 0, 0, 0};
  std::copy(hdr, hdr + 16, img.begin());
  for (int64_t g = 0; g < G; ++g) std::copy(recs[(size_t)g].begin(), recs[(size_t)g].end(), img.begin() + 16 + g * R);
  return GCNK_OK;
}

int64_t hub_plan_words(const int32_t* hdr) { return HubLayout(hdr).total; }

int64_t hub_workspace_bytes(const int32_t* hdr, int32_t F) {
  const HubLayout L(hdr);
  const int64_t ld = ((int64_t)F + 3) & ~3LL;
  return ((L.H * L.G * ld * 4) + 255) & ~255LL;
}

int hub_spmm(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F, float* C, int64_t ldc,
             const Epi& e, float* workspace, bool vec4, hipStream_t s) {
  const HubLayout L(hdr);
  if (L.H <= 0 || L.G <= 0) {
    set_error("gcnk_spmm (hub plan): empty hub plan");
    return GCNK_EARG;
  }
  const int64_t part_ld = ((int64_t)F + 3) & ~3LL;
  if (vec4) return hub_launch<4>((const int32_t*)plan, L, B, ldb, F, C, ldc, e, workspace, part_ld, s);
  return hub_launch<1>((const int32_t*)plan, L, B, ldb, F, C, ldc, e, workspace, part_ld, s);
}

}  // namespace gcnk
