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
#include "combine.h"

#include <algorithm>
#include <climits>
#include <mutex>
#include <vector>

namespace gcnk {
namespace {

#ifndef GCNK_HUB_BLOCK
#define GCNK_HUB_BLOCK 1024
#endif
#ifndef GCNK_HUB_SLICE_VECS
#define GCNK_HUB_SLICE_VECS 8
#endif
constexpr int kGroupBlock = GCNK_HUB_BLOCK;      // threads per row-group workgroup
constexpr int kSliceVecs = GCNK_HUB_SLICE_VECS;  // column vectors per slice (launch choice)
constexpr int kMaxHub = 256;          // hub rows per plan
constexpr int kMaxGroupRows = 512;    // light rows per group
constexpr int kTargetBlocks = 256;    // row-group workgroups per launch (one per CU)
constexpr int kLightBatch = 4;        // items per light-row batch (plan pads light rows to a multiple)
constexpr int kHubBatch = 8;          // items per hub batch (plan pads each hub's items to a multiple)


// ---------------------------------------------------------------------------
// Plan layout (int32 words):
//   header[16]: 0 magic 'GNH2'  1 M  2 K  3 lane groups (gcnk_spmm_groups)
//               4 G (row groups)  5 R (record stride, words)  6 H (hub rows)
//               7 h0 (first hub row)  8 nL (light rows)  9 nnz  10 gs (light
//               rows per group)  11 hub degree threshold  12 max items per
//               record  13 max hub batches per record  14..15 0
//   records[G][R]
// Record of group g (light rows l = g * gs + i, i < n):
//   0 n  1 nhb (hub batches)  2 nitems  3 o_it (word offset of the items)
//   4 ..           light entries int2 {i | batches << 16, first item}, sorted
//                  by batch count (so a wave's lanes walk the same number);
//                  a light row's items: kLightBatch-item batches
//   4 + 2n ..      hub batch entries int2 {t, first item}: kHubBatch items
//                  each, hub-major (hub t's nonzeros over the group's rows in
//                  CSR order, then its hub x hub nonzeros when t % G == g)
//   4 + 2n + 2nhb  hub batch offsets [H + 1]: hub t's batches are
//                  [off[t], off[t + 1])
//   o_it           items int2 {slot, value bits}, CSR column order; slot t < H:
//                  hub row h0 + t of B; slot H + i: light row i of the group;
//                  padding {H + n, 0} (slot H + n: a zero row of the LDS image)
struct HubLayout {
  int64_t G, R, H, h0, nL, gs, max_hb, total;
  explicit HubLayout(const int32_t* h) {
    G = h[4]; R = h[5]; H = h[6]; h0 = h[7]; nL = h[8]; gs = h[10]; max_hb = h[13];
    total = 16 + G * R;
  }
};


// ---------------------------------------------------------------------------
// Row-group kernel.  Grid G * nslices, block (g, c) = (b % G, b / G).
// LDS: record [R words] | rows [(H + n) x w] vectors (slot-major) | zero row [w] |
// bias [w] | hub batch sums [nhb x w].
template <int VEC, bool PROJ, bool BSUM>
__global__ void __launch_bounds__(kGroupBlock)
hub_group_kernel(const int32_t* __restrict__ recs, int32_t R, int32_t roff, int32_t G, int32_t gs, int32_t h0, int32_t H, int32_t nL,
                 int32_t nslices, const float* __restrict__ B, int64_t ldb, int32_t F, float* __restrict__ C,
                 int64_t ldc, Epi epi, float* __restrict__ part, int64_t part_ld, uint64_t* __restrict__ ctr, int32_t K,
                 HubExtra x, int32_t max_hb) {
  using V = Vec<VEC>;
  using T = typename V::T;
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];
  int32_t* s_rec = smem;
  T* s_rows = reinterpret_cast<T*>(smem + roff);  // roff >= R: the record area doubles as the combine's scratch
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (the compiler cannot tell)
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
  if constexpr (BSUM) {
    // B = sum of nsum operands, summed in order on the way into LDS
    for (int32_t e = tid; e < ne; e += kGroupBlock) {
      const int32_t s = e / w, j = e - s * w;
      const int64_t row = s < H ? (int64_t)h0 + s : light_row(l0 + (s - H), h0, H);
      const float* src = Bc + row * ldb + (int64_t)j * VEC;
      T acc = V::load(src);
#pragma unroll 8
      for (int32_t k = 1; k < x.nsum; ++k) V::add(acc, V::load(src + (int64_t)k * x.bstride));
      s_rows[e] = acc;
    }
  } else {
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
  }
  // slot H + n: the zero row the plan's padding items read; then the bias
  // slice, so the output loop issues no global load (one there would make
  // every iteration wait for all the stores issued before it)
  if (tid < w) s_rows[ne + tid] = V::zero();
  T* s_bias = s_rows + ne + w;
  if (epi.bias && tid < w) s_bias[tid] = V::load(epi.bias + (int64_t)(q0 + tid) * VEC);
  // PROJ: the slice's W rows (4 w x kProjMax, zero past P) and the projection
  // partials' scratch, after the hub batch sums
  float* s_w = reinterpret_cast<float*>(s_bias + w + max_hb * w);
  float* s_proj = s_w + 4 * w * kProjMax;
  if constexpr (PROJ) {
    for (int32_t e = tid; e < 4 * w * kProjMax; e += kGroupBlock) {
      const int32_t r = e / kProjMax, pp = e - r * kProjMax;
      s_w[e] = pp < x.P ? x.W[(int64_t)(q0 * VEC + r) * x.ldw + pp] : 0.f;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(epi, 1);

  // ---- outputs.  Light rows and hub batches run on separate waves,
  //      concurrently, split by their item counts.  A task is (row or batch,
  //      column vector j of the slice); its items are read a batch at a time,
  //      then the batch's row vectors, so it waits for two LDS round trips per
  //      batch.  Light rows are sorted by batch count (the lanes of a wave walk
  //      alike); hub batches are all kHubBatch long, summed per hub afterwards.
  const int32_t nhb = s_rec[1], o_it = s_rec[3];
  const int2* s_items = reinterpret_cast<const int2*>(s_rec + o_it);
  const int2* s_light = reinterpret_cast<const int2*>(s_rec + 4);
  const int2* s_hb = s_light + n;
  const int32_t* s_hoff = s_rec + 4 + 2 * n + 2 * nhb;
  T* s_hsum = s_bias + w;
  const int32_t il = nhb > 0 ? s_hb[0].y : s_rec[2], ih = s_rec[2] - il;  // light / hub items
  int nwh = 0;
  if (nhb > 0) {
    nwh = (int)(((int64_t)NW * ih + (il + ih) / 2) / max(il + ih, 1));
    nwh = min(max(nwh, 1), NW - 1);
  }
  const bool hub_wave = wv < nwh;
  if (hub_wave) {
    for (int32_t e = wv * 64 + lane; e < nhb * w; e += nwh * 64) {
      const int32_t b = e / w, j = e - b * w;
      const int4* ip = reinterpret_cast<const int4*>(s_items + s_hb[b].y);
      const T* col = s_rows + j;
      int4 p[kHubBatch / 2];
#pragma unroll
      for (int u = 0; u < kHubBatch / 2; ++u) p[u] = ip[u];
      T r[kHubBatch];
#pragma unroll
      for (int u = 0; u < kHubBatch / 2; ++u) {
        r[2 * u] = col[p[u].x * w];
        r[2 * u + 1] = col[p[u].z * w];
      }
      T acc = V::zero();
#pragma unroll
      for (int u = 0; u < kHubBatch / 2; ++u) {
        V::fma(acc, __int_as_float(p[u].y), r[2 * u]);
        V::fma(acc, __int_as_float(p[u].w), r[2 * u + 1]);
      }
      s_hsum[e] = acc;
    }
  } else {
    for (int32_t e = (wv - nwh) * 64 + lane; e < n * w; e += (NW - nwh) * 64) {
      const int32_t lo = e / w, j = e - lo * w;
      const int2 le = s_light[lo];
      const int32_t i = le.x & 0xffff, nb = le.x >> 16;
      const int4* ip = reinterpret_cast<const int4*>(s_items + le.y);
      const T* col = s_rows + j;
      T acc = V::zero();
#if defined(GCNK_HUB_EXP) && (GCNK_HUB_EXP & 4)  // ablation: no item loop
      for (int32_t b = 0; b < 0; ++b) {
#else
      for (int32_t b = 0; b < nb; ++b) {
#endif
        int4 p[kLightBatch / 2];
#pragma unroll
        for (int u = 0; u < kLightBatch / 2; ++u) p[u] = ip[u];
        ip += kLightBatch / 2;
        T r[kLightBatch];
#pragma unroll
        for (int u = 0; u < kLightBatch / 2; ++u) {
          r[2 * u] = col[p[u].x * w];
          r[2 * u + 1] = col[p[u].z * w];
        }
#pragma unroll
        for (int u = 0; u < kLightBatch / 2; ++u) {
          V::fma(acc, __int_as_float(p[u].y), r[2 * u]);
          V::fma(acc, __int_as_float(p[u].w), r[2 * u + 1]);
        }
      }
#if defined(GCNK_HUB_EXP) && (GCNK_HUB_EXP & 1)  // ablation: no light stores
      if (reinterpret_cast<const float*>(&acc)[0] == 1234.5f) V::store(C, acc);  // keeps the sum live
      continue;
#endif
      const int64_t cv = (int64_t)(q0 + j) * VEC;
      const int64_t row = light_row(l0 + i, h0, H);
      const T bv = epi.bias ? s_bias[j] : V::zero();
      const T v = V::epi(epi, acc, bv, row, cv);
      if (!PROJ || C) V::store_aligned(C + row * ldc + cv, v);
      if constexpr (PROJ) project4(v, j, s_w, x.P, s_proj + (int64_t)e * kProjMax);
    }
  }
  __syncthreads();
  // ---- this group's hub partials (hub t's batch sums in batch order), stored
  //      write-through (sc1) for the in-launch combine below
  const float* part_u = uniform_ptr(part);
  for (int32_t e = tid; e < H * w; e += kGroupBlock) {
    const int32_t t = e / w, j = e - t * w;
    T acc = V::zero();
    for (int32_t b = s_hoff[t]; b < s_hoff[t + 1]; ++b) V::add(acc, s_hsum[b * w + j]);
#if defined(GCNK_HUB_EXP) && (GCNK_HUB_EXP & 2)  // ablation: no partial stores
    if (reinterpret_cast<const float*>(&acc)[0] == 1234.5f) V::store(C, acc);
    continue;
#endif
    store_sc1(part_u, ((int64_t)t * G + g) * part_ld + (int64_t)(q0 + j) * VEC, acc);
  }
  if constexpr (PROJ) {  // light rows' projection partials: sum over the slice's vectors in order
    for (int32_t e = tid; e < n * x.P; e += kGroupBlock) {
      const int32_t lo = e / x.P, pp = e - lo * x.P;
      float a = 0.f;
      for (int32_t j = 0; j < w; ++j) a += s_proj[(int64_t)(lo * w + j) * kProjMax + pp];
      const int64_t row = light_row(l0 + (s_light[lo].x & 0xffff), h0, H);
      x.C2[(int64_t)c * x.c2_stride + row * x.ldc2 + pp] = a;
    }
    __syncthreads();  // s_proj is reused by the combine
  }
  hub_combine<kGroupBlock, VEC, PROJ>(ctr, K, s_rec, G, c, h0, H, w, q0, part_u, part_ld, C, ldc, epi, s_bias, s_w, s_proj, x, tid);
  stamp(epi, 3);  // 2: arrival (combine.h), 3: exit
}

// LDS words before the row image: the record, at least the combine's scratch
int64_t rec_words(const HubLayout& L) { return std::max<int64_t>(L.R, 4 * kGroupBlock); }

// LDS bytes of a launch with slices of at most w vectors
int64_t lds_bytes(const HubLayout& L, int64_t w, size_t vbytes, bool proj) {
  int64_t b = rec_words(L) * 4 + (L.H + L.gs + 2 + L.max_hb) * w * (int64_t)vbytes;
  if (proj) b += (4 * w + std::max<int64_t>(L.gs, (L.H + kCombineChunks - 1) / kCombineChunks + 1) * w) * kProjMax * 4;
  return b;
}

// Column slices for a launch: about 8 vectors per slice (R8 F = 200: 7 slices
// of 7-8 float4), then more until the LDS image fits.
int64_t choose_slices(const HubLayout& L, int32_t Q, size_t vbytes, bool proj, int64_t* lds_out) {
  int64_t c = std::max<int64_t>(1, std::min<int64_t>(kMaxSlices, (Q + kSliceVecs - 1) / kSliceVecs));
  for (; c <= std::min<int64_t>(Q, kMaxSlices); ++c) {
    const int64_t lds = lds_bytes(L, (Q + c - 1) / c, vbytes, proj);
    if (lds <= kLdsDyn) {
      *lds_out = lds;
      return c;
    }
  }
  return -1;
}

template <int VEC, bool PROJ, bool BSUM>
int hub_launch(const int32_t* plan, const HubLayout& L, const float* B, int64_t ldb, int32_t F, float* C, int64_t ldc,
               const Epi& e, float* part, int64_t part_ld, uint64_t* ctr, const HubExtra& x, hipStream_t s) {
  const int32_t Q = VEC == 4 ? F / 4 : F;
  int64_t lds = 0;
  const int64_t nslices = choose_slices(L, Q, sizeof(typename Vec<VEC>::T), PROJ, &lds);
  if (nslices < 0 || nslices > kMaxSlices || L.G * nslices > INT32_MAX) {
    set_error("gcnk_spmm (hub plan): F = %d does not fit %lld hub + %lld group rows of LDS", F, (long long)L.H,
              (long long)L.gs);
    return GCNK_EUNSUP;
  }
  // one workgroup per CU (the in-launch hand-off is the form measured at one
  // workgroup per CU; 1024 threads and > 80 KB of LDS admit no second)
  lds = std::max<int64_t>(lds, kLdsMax / 2 + 16);
  // dynamic LDS up to kLdsDyn (the kernel's static LDS takes the rest of the 160 KiB)
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&hub_group_kernel<VEC, PROJ, BSUM>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, kLdsDyn);
  if (attr != hipSuccess) return hip_check(attr, "hub_group_kernel LDS attribute");
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 0;
    return n;
  }();
  const int32_t K = L.G * nslices <= cus ? (int32_t)std::min<int64_t>(kCombineChunks, L.G) : 1;
  hipLaunchKernelGGL((hub_group_kernel<VEC, PROJ, BSUM>), dim3((unsigned)(L.G * nslices)), dim3(kGroupBlock),
                     (size_t)lds, s, plan + 16, (int32_t)L.R, (int32_t)rec_words(L), (int32_t)L.G, (int32_t)L.gs,
                     (int32_t)L.h0, (int32_t)L.H, (int32_t)L.nL, (int32_t)nslices, B, ldb, F, C, ldc, e, part, part_ld,
                     ctr, K, x, (int32_t)L.max_hb);
  return launch_check("hub_group_kernel");
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
  int64_t R = 4, max_items = 0, max_hb = 0;
  std::vector<int64_t> ord;
  for (int64_t g = 0; g < G; ++g) {
    const int64_t l0 = g * gs, n = std::min(gs, nL - l0);
    auto light_batches = [&](int64_t i) {
      const int64_t r = light_row_host(l0 + i, h0, H);
      return ((int64_t)rp[r + 1] - rp[r] + kLightBatch - 1) / kLightBatch;
    };
    int64_t nit = 0, nhb = 0;
    for (int64_t i = 0; i < n; ++i) nit += light_batches(i) * kLightBatch;
    for (int64_t t = 0; t < H; ++t) {
      const int64_t b = ((int64_t)hub_k[(size_t)(g * H + t)].size() + kHubBatch - 1) / kHubBatch;
      nhb += b;
      nit += b * kHubBatch;
    }
    if (n >= 65536 || light_batches(0) >= 32768) return 1;
    const int64_t o_it = align4(4 + 2 * n + 2 * nhb + H + 1);
    std::vector<int32_t>& w = recs[(size_t)g];
    w.assign((size_t)align4(o_it + 2 * nit), 0);
    w[0] = (int32_t)n;
    w[1] = (int32_t)nhb;
    w[2] = (int32_t)nit;
    w[3] = (int32_t)o_it;
    int64_t it = 0;
    auto item = [&](int64_t col, int64_t k) {
      const int64_t slot = is_hub(col) ? col - h0 : H + (light_index(col) - l0);
      w[(size_t)(o_it + 2 * it)] = (int32_t)slot;
      w[(size_t)(o_it + 2 * it + 1)] = vv ? __builtin_bit_cast(int32_t, vv[k]) : 0;
      ++it;
    };
    // padding items read the zero row (slot H + n) with value 0
    auto pad = [&](int64_t m, int64_t start) {
      while ((it - start) % m) {
        w[(size_t)(o_it + 2 * it)] = (int32_t)(H + n);
        w[(size_t)(o_it + 2 * it + 1)] = 0;
        ++it;
      }
    };
    // light rows, most batches first (stable: row order among equals)
    ord.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) ord[(size_t)i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return light_batches(a) > light_batches(b); });
    for (int64_t lo = 0; lo < n; ++lo) {
      const int64_t i = ord[(size_t)lo];
      const int64_t r = light_row_host(l0 + i, h0, H);
      w[(size_t)(4 + 2 * lo)] = (int32_t)(i | (light_batches(i) << 16));
      const int64_t start = it;
      w[(size_t)(4 + 2 * lo + 1)] = (int32_t)it;
      for (int64_t k = rp[r]; k < rp[r + 1]; ++k) item(ci[k], k);
      pad(kLightBatch, start);
    }
    int64_t hb = 0;
    const int64_t o_hb = 4 + 2 * n, o_off = o_hb + 2 * nhb;
    for (int64_t t = 0; t < H; ++t) {
      w[(size_t)(o_off + t)] = (int32_t)hb;
      const std::vector<int64_t>& ks = hub_k[(size_t)(g * H + t)];
      const int64_t start = it;
      for (size_t q = 0; q < ks.size(); ++q) {
        if (q % kHubBatch == 0) {
          w[(size_t)(o_hb + 2 * hb)] = (int32_t)t;
          w[(size_t)(o_hb + 2 * hb + 1)] = (int32_t)it;
          ++hb;
        }
        item(ci[ks[q]], ks[q]);
      }
      pad(kHubBatch, start);
    }
    w[(size_t)(o_off + H)] = (int32_t)hb;
    R = std::max<int64_t>(R, (int64_t)w.size());
    max_items = std::max(max_items, it);
    max_hb = std::max(max_hb, nhb);
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
                           (int32_t)hmin,   (int32_t)max_items, (int32_t)max_hb, 0, 0};
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

int64_t hub_counter_bytes(const int32_t* hdr) {
  (void)hdr;
  return combine_counter_bytes();
}

int32_t hub_proj_slices(const int32_t* hdr, int32_t F) {
  const HubLayout L(hdr);
  int64_t lds = 0;
  return (int32_t)choose_slices(L, F / 4, 16, true, &lds);
}

int hub_spmm(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F, float* C, int64_t ldc,
             const Epi& e, float* workspace, int32_t* counters, bool vec4, const HubSide& side, hipStream_t s) {
  const HubLayout L(hdr);
  if (L.H <= 0 || L.G <= 0) {
    set_error("gcnk_spmm (hub plan): empty hub plan");
    return GCNK_EARG;
  }
  if ((reinterpret_cast<uintptr_t>(counters) & 7) != 0) {
    set_error("gcnk_spmm (hub plan): counter region must be 8-byte aligned");
    return GCNK_EARG;
  }
  const int64_t part_ld = ((int64_t)F + 3) & ~3LL;
  uint64_t* ctr = reinterpret_cast<uint64_t*>(counters);
  const int32_t* p = (const int32_t*)plan;
  HubExtra x{side.W, side.ldw, side.P, side.C2, side.c2_stride, side.ldc2, side.nsum, side.bstride};
  const bool proj = side.W != nullptr, bsum = side.nsum > 1;
  if (proj && !vec4) {
    set_error("gcnk_spmm (hub plan): a fused projection needs float4-aligned operands");
    return GCNK_EUNSUP;
  }
  if (proj && (side.P < 1 || side.P > kProjMax || !side.C2)) {
    set_error("gcnk_spmm (hub plan): fused projection width P = %d (1..%d)", side.P, kProjMax);
    return GCNK_EUNSUP;
  }
  if (proj && bsum) {
    set_error("gcnk_spmm (hub plan): a fused projection of a summed operand is not supported");
    return GCNK_EUNSUP;
  }
  if (proj) return hub_launch<4, true, false>(p, L, B, ldb, F, C, ldc, e, workspace, part_ld, ctr, x, s);
  if (bsum && vec4 && x.bstride % 4 == 0)
    return hub_launch<4, false, true>(p, L, B, ldb, F, C, ldc, e, workspace, part_ld, ctr, x, s);
  if (bsum) return hub_launch<1, false, true>(p, L, B, ldb, F, C, ldc, e, workspace, part_ld, ctr, x, s);
  if (vec4) return hub_launch<4, false, false>(p, L, B, ldb, F, C, ldc, e, workspace, part_ld, ctr, x, s);
  return hub_launch<1, false, false>(p, L, B, ldb, F, C, ldc, e, workspace, part_ld, ctr, x, s);
}

}  // namespace gcnk
