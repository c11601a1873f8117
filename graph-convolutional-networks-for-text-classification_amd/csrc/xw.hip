// X W for operands with a few dense rows among rows that use only a few
// columns -- the reference's topic features X (trainer.py:226-238;
// layer.py:102 th.spmm(X, W1): R8 7,674 document rows over the 50 topic
// columns, 50 fully dense topic rows over 7,463 columns) and its transpose in
// the backward (X^T g: 7,413 feature rows over the 50 topic nodes, 50 dense
// rows).  Plan magic 'GNX1' ("split plan").
//
// One launch, two kinds of workgroups:
//   * light blocks: 32 light rows x a 256-column tile of W; W's rows at the
//     "hot" columns (the only columns light rows use) are staged in LDS once
//     per block, the rows' values are stored densely over the hot columns in
//     the plan; 32 x 256 x hot on fp32 MFMA (v_mfma_f32_16x16x4_f32: an exact
//     fp32 fmaf chain in column order, as CSR order sums them);
//   * heavy blocks (k chunk, column slice): the dense rows' partial product
//     over one chunk of K on MFMA, staged through LDS, stored write-through as
//     a float4 slab; the last blocks of each column slice sum the chunks in
//     order inside the launch (combine.h) -- no reduce launch, no slab round
//     trip through a kernel boundary.
// The heavy rows must form one contiguous range (row h0 .. h0 + nh - 1); the
// light rows are the others, in order (R8 X: h0 = 7674; X^T: h0 = 0).
#include "gcnk_common.h"
#include "combine.h"

#include <algorithm>
#include <climits>
#include <vector>

namespace gcnk {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kXwBlock = 256;          // 4 waves
constexpr int kLightRows = 32;         // light rows per light block (2 MFMA m-tiles)
constexpr int kLightCols = 256;        // W columns per light block (16 n-tiles)
constexpr int kMaxHot = 64;            // hot columns per plan
constexpr int kMaxHeavy = 128;         // heavy rows per plan (8 m-tiles)
constexpr int kHeavyCols = 32;         // W columns per heavy block (2 n-tiles)
constexpr int kHeavyTarget = 512;      // heavy blocks per launch (~two per CU)

// Plan layout (int32 words):
//   header[16]: 0 magic 'GNX1'  1 M  2 K  3 lane groups  4 nl (light rows)
//               5 nhot  6 nhp (nhot rounded up to 4)  7 nh (heavy rows)
//               8 h0 (first heavy row)  9 nnz  10 o_hot  11 o_xl  12 o_xh
//               13 ldxh (K rounded up to 4)  14 heavy threshold  15 0
//   hot columns int32[nhp] (padding: column 0 with value 0 below)
//   Xl float[nl x nhp]   light row l (row l < h0 ? l : l + nh) over the hot columns
//   Xh float[nh x ldxh]  heavy rows, dense
struct XwLayout {
  int64_t M, K, nl, nhot, nhp, nh, h0, o_hot, o_xl, o_xh, ldxh, total;
  explicit XwLayout(const int32_t* h) {
    M = h[1]; K = h[2]; nl = h[4]; nhot = h[5]; nhp = h[6]; nh = h[7]; h0 = h[8];
    o_hot = h[10]; o_xl = h[11]; o_xh = h[12]; ldxh = h[13];
    total = o_xh + nh * ldxh;
  }
};

struct XwArgs {
  const int32_t* plan;
  int32_t nl, nhot, nhp, nh, h0, ldxh, K;
  int32_t nlb;            // light blocks (row blocks x column tiles)
  int32_t nct;            // light column tiles
  int32_t nkc, kc_len;    // heavy k chunks and their length (multiple of 4)
  int32_t ncs, cs_len;    // heavy column slices and their width (multiple of 16)
  int32_t K_comb;         // combining workgroups per slice (combine.h)
  const float* W;
  int64_t ldw;
  int32_t F;
  float* C;
  int64_t ldc;
  float* slab;            // [nh][nkc][ldp] partials
  int64_t ldp;
  uint64_t* ctr;
};

// MFMA fragment maps (v_mfma_f32_16x16x4_f32): A lane l -> row l & 15, k l >> 4;
// B lane l -> col l & 15, k l >> 4; C register r -> row (l >> 4) * 4 + r, col l & 15.
template <int VEC>
__global__ void __launch_bounds__(kXwBlock) xw_kernel(XwArgs a, Epi epi) {
  using V = Vec<VEC>;
  using T = typename V::T;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  if ((int32_t)blockIdx.x < a.nlb) {
    // ---------------- light block: rows [r0, r0 + 32) x columns [n0, n0 + tn)
    const int32_t rb = blockIdx.x / a.nct, ct = blockIdx.x % a.nct;
    const int32_t l0 = rb * kLightRows;
    const int32_t n0 = ct * kLightCols, tn = min(kLightCols, a.F - n0);
    const int32_t ntile = (tn + 15) / 16, tnp = ntile * 16;
    const int32_t* hotc = a.plan + a.plan[10];
    const float* xl = reinterpret_cast<const float*>(a.plan + a.plan[11]);
    float* sW = sm;                       // [nhp][tnp]
    float* sX = sm + a.nhp * tnp;         // [32][nhp + 1]
    const int32_t ldx = a.nhp + 1;
    // W's hot rows (zero past tn and past nhot), then the block's X rows
    for (int32_t e = tid; e < a.nhp * tnp; e += kXwBlock) {
      const int32_t h = e / tnp, c = e - h * tnp;
      sW[e] = (c < tn && h < a.nhot) ? a.W[(int64_t)hotc[h] * a.ldw + n0 + c] : 0.f;
    }
    for (int32_t e = tid; e < kLightRows * a.nhp; e += kXwBlock) {
      const int32_t r = e / a.nhp, h = e - r * a.nhp;
      sX[r * ldx + h] = (l0 + r < a.nl) ? xl[(int64_t)(l0 + r) * a.nhp + h] : 0.f;
    }
    __syncthreads();
    // wave w: n-tiles w, w + 4, ... for both m-tiles
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int lr = lane & 15, lk = lane >> 4;
    for (int32_t k = 0; k < a.nhp; k += 4) {
      const float a0 = sX[lr * ldx + k + lk], a1 = sX[(16 + lr) * ldx + k + lk];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int32_t nt = wv + 4 * j;
        if (nt < ntile) {
          const float b = sW[(k + lk) * tnp + nt * 16 + lr];
          acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b, acc[0][j], 0, 0, 0);
          acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b, acc[1][j], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int32_t nt = wv + 4 * j;
      if (nt >= ntile) continue;
      const int64_t col = n0 + nt * 16 + lr;
      const float bv = (epi.bias && col < a.F) ? epi.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int32_t l = l0 + i * 16 + lk * 4 + r;
          if (l < a.nl && col < a.F) {
            const int64_t row = light_row(l, a.h0, a.nh);
            a.C[row * a.ldc + col] = apply_epi(epi, acc[i][j][r], bv, row, col);
          }
        }
    }
    return;
  }
  // ---------------- heavy block: k chunk kc x column slice cs
  const int32_t hb = blockIdx.x - a.nlb;
  const int32_t kc = hb % a.nkc, cs = hb / a.nkc;
  const int32_t k0 = kc * a.kc_len, kl = min(a.kc_len, a.K - k0);
  const int32_t c0 = cs * a.cs_len, cw = min(a.cs_len, a.F - c0);
  const int32_t mt = (a.nh + 15) / 16, nts = a.cs_len / 16;
  const float* xh = reinterpret_cast<const float*>(a.plan + a.plan[12]);
  const int32_t lda = a.kc_len + 1, ldb = a.cs_len + 4;
  float* sA = sm;                                  // [mt * 16][kc_len + 1]
  float* sB = sm + mt * 16 * lda;                  // [kc_len][cs_len + 4]
  for (int32_t e = tid; e < mt * 16 * a.kc_len; e += kXwBlock) {
    const int32_t r = e / a.kc_len, k = e - r * a.kc_len;
    sA[r * lda + k] = (r < a.nh && k < kl) ? xh[(int64_t)r * a.ldxh + k0 + k] : 0.f;
  }
  for (int32_t e = tid; e < a.kc_len * a.cs_len; e += kXwBlock) {
    const int32_t k = e / a.cs_len, c = e - k * a.cs_len;
    sB[k * ldb + c] = (k < kl && c < cw) ? a.W[(int64_t)(k0 + k) * a.ldw + c0 + c] : 0.f;
  }
  __syncthreads();
  // (m-tile, n-tile) pairs p = wv, wv + 4, ...  (mt <= 8, nts <= 4: <= 8 per wave)
  f32x4 acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lr = lane & 15, lk = lane >> 4;
  const int32_t npair = mt * nts;
  for (int32_t k = 0; k < a.kc_len; k += 4) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int32_t pr = wv + 4 * q;
      if (pr < npair) {
        const int32_t i = pr / nts, j = pr - i * nts;
        const float av = sA[(i * 16 + lr) * lda + k + lk];
        const float bv = sB[(k + lk) * ldb + j * 16 + lr];
        acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[q], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // sA / sB are reused: the partial tile [mt * 16][cs_len] goes through LDS
  float* sT = sm;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int32_t pr = wv + 4 * q;
    if (pr < npair) {
      const int32_t i = pr / nts, j = pr - i * nts;
#pragma unroll
      for (int r = 0; r < 4; ++r) sT[(i * 16 + lk * 4 + r) * a.cs_len + j * 16 + lr] = acc[q][r];
    }
  }
  __syncthreads();
  // partial rows (VEC-wide pieces), write-through, at slab[(h * nkc + kc) * ldp + c0 ..]
  const float* slab_u = uniform_ptr(a.slab);
  const int32_t wv4 = (cw + VEC - 1) / VEC;
  for (int32_t e = tid; e < a.nh * wv4; e += kXwBlock) {
    const int32_t h = e / wv4, q = e - h * wv4;
    const T v = *reinterpret_cast<const T*>(sT + h * a.cs_len + VEC * q);
    store_sc1(slab_u, ((int64_t)h * a.nkc + kc) * a.ldp + c0 + VEC * q, v);
  }
  // the chunks of this slice summed in order by its last workgroups
  HubExtra none{};
  hub_combine<kXwBlock, VEC, false>(a.ctr, a.K_comb, reinterpret_cast<int32_t*>(sm), a.nkc, cs, a.h0, a.nh, wv4,
                                    c0 / VEC, slab_u, a.ldp, a.C, a.ldc, epi, nullptr, nullptr, nullptr, none, tid);
}

}  // namespace

// ---------------------------------------------------------------------------
// Host plan: GCNK_OK with `img` filled, 1 when the operand does not have the
// structure (the caller builds another plan), or a negative error code.
int xw_plan_host(const int32_t* rp, const int32_t* ci, const float* vv, int32_t M, int32_t K, int64_t nnz,
                 int32_t groups, std::vector<int32_t>& img) {
  if (M <= 0 || K <= 0 || nnz <= 0 || groups <= 0) return 1;
  // heavy rows: more nonzeros than the hot-column limit; they must be one
  // contiguous range and few
  const int64_t hthr = kMaxHot;
  int64_t h0 = -1, h1 = -1;
  for (int32_t r = 0; r < M; ++r) {
    if ((int64_t)rp[r + 1] - rp[r] <= hthr) continue;
    if (h0 < 0) {
      h0 = r;
    } else if (r != h1) {
      return 1;
    }
    h1 = r + 1;
  }
  if (h0 < 0) h0 = h1 = M;
  const int64_t nh = h1 - h0, nl = (int64_t)M - nh;
  if (nh > kMaxHeavy) return 1;
  const int64_t ldxh = align4(K);
  if (nh * ldxh * 4 > ((int64_t)256 << 20)) return 1;
  // hot columns: every column a light row uses (<= kMaxHot)
  std::vector<int32_t> slot((size_t)K, -1), hotc;
  for (int64_t l = 0; l < nl; ++l) {
    const int64_t r = light_row_host(l, h0, nh);
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
      if (slot[(size_t)ci[k]] < 0) {
        if ((int64_t)hotc.size() == kMaxHot) return 1;
        slot[(size_t)ci[k]] = 0;
        hotc.push_back(ci[k]);
      }
    }
  }
  // light rows must be at least a quarter full over the hot columns (else the
  // dense staging wastes more than it saves), and there must be heavy or many light rows
  std::sort(hotc.begin(), hotc.end());
  for (size_t h = 0; h < hotc.size(); ++h) slot[(size_t)hotc[h]] = (int32_t)h;
  const int64_t nhot = (int64_t)hotc.size(), nhp = std::max<int64_t>(4, align4(nhot));
  const int64_t light_nnz = nnz - (nh > 0 ? (int64_t)rp[h1] - rp[h0] : 0);
  if (nl > 0 && light_nnz * 4 < nl * nhot) return 1;
  if (nh == 0 && nl < 1024) return 1;
  const int64_t o_hot = 16, o_xl = align4(o_hot + nhp), o_xh = align4(o_xl + nl * nhp);
  const int64_t words = o_xh + nh * ldxh;
  if (words >= INT32_MAX) return 1;
  img.assign((size_t)words, 0);
  const int32_t hdr[16] = {kXwMagic, M, K, groups, (int32_t)nl, (int32_t)nhot, (int32_t)nhp, (int32_t)nh,
                           (int32_t)h0, (int32_t)nnz, (int32_t)o_hot, (int32_t)o_xl, (int32_t)o_xh, (int32_t)ldxh,
                           (int32_t)hthr, 0};
  std::copy(hdr, hdr + 16, img.begin());
  for (int64_t h = 0; h < nhp; ++h) img[(size_t)(o_hot + h)] = h < nhot ? hotc[(size_t)h] : 0;
  float* xl = reinterpret_cast<float*>(img.data() + o_xl);
  float* xh = reinterpret_cast<float*>(img.data() + o_xh);
  // duplicates summed in CSR order (what th.spmm's coalesce computes)
  for (int64_t l = 0; l < nl; ++l) {
    const int64_t r = light_row_host(l, h0, nh);
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k) xl[l * nhp + slot[(size_t)ci[k]]] += vv ? vv[k] : 0.f;
  }
  for (int64_t h = 0; h < nh; ++h)
    for (int64_t k = rp[h0 + h]; k < rp[h0 + h + 1]; ++k) xh[h * ldxh + ci[k]] += vv ? vv[k] : 0.f;
  return GCNK_OK;
}

int64_t xw_plan_words(const int32_t* hdr) { return XwLayout(hdr).total; }

// launch geometry for width F
static void xw_geometry(const XwLayout& L, int32_t F, int32_t& nct, int32_t& nlb, int32_t& ncs, int32_t& cs_len,
                        int32_t& nkc, int32_t& kc_len) {
  nct = (F + kLightCols - 1) / kLightCols;
  nlb = (int32_t)((L.nl + kLightRows - 1) / kLightRows) * nct;
  cs_len = kHeavyCols * std::max<int32_t>(1, (F + kHeavyCols * kMaxSlices - 1) / (kHeavyCols * kMaxSlices));
  cs_len = std::min<int32_t>(cs_len, 64);
  ncs = (F + cs_len - 1) / cs_len;
  nkc = 0;
  kc_len = 4;
  if (L.nh > 0) {
    nkc = (int32_t)std::max<int64_t>(1, std::min<int64_t>(kHeavyTarget / std::max(ncs, 1), (L.K + 15) / 16));
    kc_len = (int32_t)align4((L.K + nkc - 1) / nkc);
    nkc = (int32_t)((L.K + kc_len - 1) / kc_len);
  }
}

int64_t xw_workspace_bytes(const int32_t* hdr, int32_t F) {
  const XwLayout L(hdr);
  int32_t nct, nlb, ncs, cs_len, nkc, kc_len;
  xw_geometry(L, F, nct, nlb, ncs, cs_len, nkc, kc_len);
  return ((L.nh * nkc * align4(F) * 4) + 255) & ~255LL;
}

int64_t xw_counter_bytes(const int32_t* hdr) { return XwLayout(hdr).nh > 0 ? combine_counter_bytes() : 0; }

template <int VEC>
static int xw_launch(const XwLayout& L, const void* plan, const float* B, int64_t ldb, int32_t F, float* C,
                     int64_t ldc, const Epi& e, float* workspace, int32_t* counters, hipStream_t s);

int xw_spmm(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F, float* C, int64_t ldc,
            const Epi& e, float* workspace, int32_t* counters, bool vec4, hipStream_t s) {
  const XwLayout L(hdr);
  if (e.code != GCNK_EPI_NONE) {
    set_error("gcnk_spmm (split plan): epilogue %d unsupported (the X W products of the reference have none)", e.code);
    return GCNK_EUNSUP;
  }
  if (vec4) return xw_launch<4>(L, plan, B, ldb, F, C, ldc, e, workspace, counters, s);
  return xw_launch<1>(L, plan, B, ldb, F, C, ldc, e, workspace, counters, s);
}

template <int VEC>
static int xw_launch(const XwLayout& L, const void* plan, const float* B, int64_t ldb, int32_t F, float* C,
                     int64_t ldc, const Epi& e, float* workspace, int32_t* counters, hipStream_t s) {
  int32_t nct, nlb, ncs, cs_len, nkc, kc_len;
  xw_geometry(L, F, nct, nlb, ncs, cs_len, nkc, kc_len);
  if (L.nh > 0 && (ncs > kMaxSlices || !counters || (reinterpret_cast<uintptr_t>(counters) & 7))) {
    set_error("gcnk_spmm (split plan): F = %d needs %d column slices / an 8-byte aligned counter region", F, ncs);
    return GCNK_EUNSUP;
  }
  const int64_t lds_light = (L.nhp * (int64_t)(((std::min(F, kLightCols) + 15) / 16) * 16) +
                             (int64_t)kLightRows * (L.nhp + 1)) * 4;
  const int64_t lds_heavy = L.nh > 0 ? ((L.nh + 15) / 16 * 16 * (int64_t)(kc_len + 1) +
                                        (int64_t)kc_len * (cs_len + 4)) * 4 : 0;
  const int64_t lds = std::max<int64_t>(std::max(lds_light, lds_heavy), (int64_t)kXwBlock * 16);
  if (lds > kLdsDyn) {
    set_error("gcnk_spmm (split plan): %lld B of LDS (k chunk %d)", (long long)lds, kc_len);
    return GCNK_EUNSUP;
  }
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&xw_kernel<VEC>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, kLdsDyn);
  if (attr != hipSuccess) return hip_check(attr, "xw_kernel LDS attribute");
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&xw_kernel<VEC>), kXwBlock,
                                                   (size_t)lds) != hipSuccess)
    per_cu = 0;
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 0;
    return n;
  }();
  const int64_t grid = (int64_t)nlb + (int64_t)nkc * ncs;
  if (grid == 0) return GCNK_OK;
  XwArgs a;
  a.plan = (const int32_t*)plan;
  a.nl = (int32_t)L.nl; a.nhot = (int32_t)L.nhot; a.nhp = (int32_t)L.nhp; a.nh = (int32_t)L.nh; a.h0 = (int32_t)L.h0;
  a.ldxh = (int32_t)L.ldxh; a.K = (int32_t)L.K;
  a.nlb = nlb; a.nct = nct; a.nkc = nkc; a.kc_len = kc_len; a.ncs = ncs; a.cs_len = cs_len;
  // waiting combiners only when every workgroup of the grid is resident at once
  a.K_comb = grid <= (int64_t)cus * std::max(per_cu, 0) ? std::min(kCombineChunks, std::max(nkc, 1)) : 1;
  a.W = B; a.ldw = ldb; a.F = F; a.C = C; a.ldc = ldc;
  a.slab = workspace; a.ldp = align4(F);
  a.ctr = reinterpret_cast<uint64_t*>(counters);
  hipLaunchKernelGGL((xw_kernel<VEC>), dim3((unsigned)grid), dim3(kXwBlock), (size_t)lds, s, a, e);
  return launch_check("xw_kernel");
}

}  // namespace gcnk
