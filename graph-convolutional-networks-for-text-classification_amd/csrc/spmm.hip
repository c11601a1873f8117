// CSR SpMM for gfx950:  C = epi(A_csr * B)
//
// Replaces th.spmm(adj, support) (reference layer.py:106) and th.spmm(X, W)
// with sparse X (layer.py:102), plus their autograd products A^T g / X^T g.
//
// A sparse operand is converted once (gcnk_spmm_plan_build) into a hybrid
// plan that splits its rows between two kernels writing disjoint rows of C:
//
//  * dense blocks -> spmm_tile_kernel (fp32 MFMA).  Rows are grouped in
//    blocks of RB = 64; a block whose nonzeros fill at least `dense_threshold`
//    of its condensed column set (the distinct columns its rows use) is stored
//    densely over those columns, in MFMA fragment order, in chunks of KC = 64
//    columns.  One workgroup per chunk stages the chunk's 64 B rows in LDS
//    ONCE and reuses them for all 64 rows (R8's X: every document row uses
//    the same 50 topic columns; the 50 topic rows are fully dense), instead
//    of gathering a B row per nonzero.  Blocks with several chunks write
//    partial slabs that spmm_tile_reduce_kernel sums in chunk order.
//
//  * the remaining rows -> spmm_path_kernel (gathers).  The nonzeros in row
//    order, each row closed by an end-of-row marker (col = -1, payload = row)
//    form one int2 item stream cut into workgroup windows of W = G*ipc items;
//    a row of at most W/2 items that would straddle a window is pushed to the
//    next with pad items (col = -2), so only heavy rows cross windows and the
//    kernel needs no search: window w is items [w*W, (w+1)*W), loaded in one
//    coalesced pass, then the B-row gathers issue.  Groups of LPR lanes walk
//    ipc items each, gathering U nonzeros at a time (U*VPL independent 16-B
//    loads in flight per lane) and flushing a row at its marker with
//    bias/ReLU/dropout fused into the store.  Lanes own VEC-wide column
//    vectors interleaved by LPR (one load instruction of a group covers
//    LPR*VEC contiguous floats of a B row).  Rows split between the groups of
//    a window meet in LDS; heavy rows crossing windows leave one partial per
//    window, and the last of those windows to finish (arrival counter in the
//    plan) sums them in path order -- one launch, no fix-up kernel.
//
// Every sum has a fixed order (no float atomics): results are bitwise
// reproducible run to run.
#include "gcnk_common.h"

#include <algorithm>
#include <climits>
#include <vector>

namespace gcnk {
namespace {

constexpr int32_t kMarker = -1;  // end of row; .y = row index
constexpr int32_t kPad = -2;     // no-op
constexpr int32_t kMagic = 0x474e4b34;  // "GNK4"
constexpr int kRB = 64;          // tile rows per dense block (4 waves x 16)
constexpr int kKC = 64;          // condensed columns per tile chunk (16 MFMA k-steps)
constexpr int kMaxNT = 14;
constexpr int kMaxColTiles = 64;  // path column tiles per launch (arrival counters per cross row)       // 16-column MFMA n-tiles per tile workgroup (B tile <= 57 KB LDS)

template <int VEC>
struct Vec;

template <>
struct Vec<4> {
  using T = float4;
  static __device__ __forceinline__ T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  static __device__ __forceinline__ T load(const float* p) { return *reinterpret_cast<const float4*>(p); }
  static __device__ __forceinline__ void store(float* p, const T& v) { *reinterpret_cast<float4*>(p) = v; }
  static __device__ __forceinline__ void fma(T& acc, float a, const T& b) {
    acc.x = fmaf(a, b.x, acc.x);
    acc.y = fmaf(a, b.y, acc.y);
    acc.z = fmaf(a, b.z, acc.z);
    acc.w = fmaf(a, b.w, acc.w);
  }
  static __device__ __forceinline__ void add(T& acc, const T& b) {
    acc.x += b.x; acc.y += b.y; acc.z += b.z; acc.w += b.w;
  }
  static __device__ __forceinline__ T epi(const Epi& e, const T& a, const T& b, int64_t row, int64_t col) {
    T r;
    r.x = apply_epi(e, a.x, b.x, row, col + 0);
    r.y = apply_epi(e, a.y, b.y, row, col + 1);
    r.z = apply_epi(e, a.z, b.z, row, col + 2);
    r.w = apply_epi(e, a.w, b.w, row, col + 3);
    return r;
  }
};

template <>
struct Vec<1> {
  using T = float;
  static __device__ __forceinline__ T zero() { return 0.f; }
  static __device__ __forceinline__ T load(const float* p) { return *p; }
  static __device__ __forceinline__ void store(float* p, const T& v) { *p = v; }
  static __device__ __forceinline__ void fma(T& acc, float a, const T& b) { acc = fmaf(a, b, acc); }
  static __device__ __forceinline__ void add(T& acc, const T& b) { acc += b; }
  static __device__ __forceinline__ T epi(const Epi& e, const T& a, const T& b, int64_t row, int64_t col) {
    return apply_epi(e, a, b, row, col);
  }
};

// ---------------------------------------------------------------------------
// Plan layout (int32 words).  Header (16 words, see gcnk.h):
//   0 magic  1 M  2 K  3 groups  4 ipc  5 W  6 nwin  7 nfix  8 nslots
//   9 ntile (chunks)  10 nred  11 nslabs  12 ntblk (tile blocks)  13 has_diag  14 heavy  15 0
struct Layout {
  int64_t nwin, W, nfix, ntile, nred, ntblk, has_diag, M;
  int64_t items, head, tail, hfix, tfix, fix, cnt, tdesc, tcols, tfrag, red, trows, dval, total;
  __host__ __device__ explicit Layout(const int32_t* h) {
    M = h[1]; nwin = h[6]; W = h[5]; nfix = h[7]; ntile = h[9]; nred = h[10]; ntblk = h[12]; has_diag = h[13];
    items = 16;
    head = items + 2 * nwin * W;
    tail = head + nwin;
    hfix = tail + nwin;
    tfix = hfix + nwin;
    fix = tfix + nwin;
    cnt = fix + 3 * nfix;
    tdesc = (cnt + (int64_t)kMaxColTiles * nfix + 3) & ~3LL;
    tcols = tdesc + 4 * ntile;
    tfrag = (tcols + (int64_t)kKC * ntile + 3) & ~3LL;
    red = tfrag + (int64_t)kRB * kKC * ntile;
    trows = red + 4 * nred;
    dval = trows + (int64_t)kRB * ntblk;
    total = dval + (has_diag ? M : 0);
  }
};

// ---------------------------------------------------------------------------
// Plan construction kernels.
__global__ void fill_pad_kernel(int2* __restrict__ items, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) items[i] = make_int2(kPad, 0);
}

// nonzero k of row r goes to start[r] + (k - rowptr[r]); the marker to start[r] + deg(r);
// rows handled by the tile path have start[r] < 0 and no items.
__global__ void scatter_items_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colind,
                                     const float* __restrict__ val, int32_t M, const int32_t* __restrict__ start,
                                     int2* __restrict__ items) {
  const int32_t r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= M) return;
  const int32_t s = start[r];
  if (s < 0) return;
  const int lane = threadIdx.x & 63;
  const int32_t b = rowptr[r], e = rowptr[r + 1];
  for (int32_t k = b + lane; k < e; k += 64) items[s + (k - b)] = make_int2(colind[k], __float_as_int(val[k]));
  if (lane == 0) items[s + (e - b)] = make_int2(kMarker, r);
}

// ---------------------------------------------------------------------------
// Fused dense projection of a finished row: C2[row, :P] = h[row, :F] * W[F, P]
// (the gc2 support H1 W2 of reference layer.py:102, computed while H1's row
// is still in registers).  Each lane holds W rows of its own columns; the
// group's partial sums meet by an xor butterfly over its LPR lanes.
struct ProjArgs {
  const float* W;  // [F x P] row-major; null = no projection
  int64_t ldw;
  int32_t P;
  float* C2;       // [M x P]
  int64_t ldc2;
  int32_t store_main;  // also store C (the SpMM output itself)
};

template <int NP, int LPR, int VPL, int VEC>
struct Proj {
  float w[VPL * VEC][NP > 0 ? NP : 1];
  __device__ __forceinline__ void load(const ProjArgs& pa, int32_t F, const int64_t* colv, const bool* colok) {
    if constexpr (NP > 0) {
#pragma unroll
      for (int v = 0; v < VPL; ++v)
#pragma unroll
        for (int i = 0; i < VEC; ++i)
#pragma unroll
          for (int c = 0; c < NP; ++c) {
            const int64_t col = colv[v] + i;
            w[v * VEC + i][c] = (colok[v] && col < F && c < pa.P) ? pa.W[col * pa.ldw + c] : 0.f;
          }
    }
  }
  template <typename T>
  __device__ __forceinline__ void apply(const ProjArgs& pa, const T* h, int64_t row, int lg) const {
    if constexpr (NP > 0) {
      float s[NP];
#pragma unroll
      for (int c = 0; c < NP; ++c) s[c] = 0.f;
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        const float* hv = reinterpret_cast<const float*>(&h[v]);
#pragma unroll
        for (int i = 0; i < VEC; ++i)
#pragma unroll
          for (int c = 0; c < NP; ++c) s[c] = fmaf(hv[i], w[v * VEC + i][c], s[c]);
      }
      // transpose-reduce: while channels remain to split, each xor step sends the
      // half of the channels the partner keeps (n/2 shuffles instead of n), so a
      // lane ends with NP/2^h channels summed over 2^h lanes; plain xor steps finish.
      int chan = 0;
      reduce_split<NP>(s, lg, chan);
      constexpr int H = ilog2(NP) < ilog2(LPR) ? ilog2(NP) : ilog2(LPR);
      constexpr int NR = NP >> H;          // channels left per lane
      constexpr int REST = LPR >> H;       // lanes still to sum over
#pragma unroll
      for (int off = REST / 2; off >= 1; off >>= 1)
#pragma unroll
        for (int c = 0; c < NR; ++c) s[c] += __shfl_xor(s[c], off, 64);
      if ((lg & (REST - 1)) == 0) {
#pragma unroll
        for (int c = 0; c < NR; ++c)
          if (chan + c < pa.P) pa.C2[row * pa.ldc2 + chan + c] = s[c];
      }
    }
  }

  static constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x >> 1); }

  // One halving step per recursion level, offsets LPR/2, LPR/4, ... while n > 1.
  template <int N, int OFF = LPR / 2>
  __device__ __forceinline__ static void reduce_split(float* s, int lg, int& chan) {
    if constexpr (N > 1 && OFF >= 1) {
      constexpr int Hn = N / 2;
      const bool up = (lg & OFF) != 0;
#pragma unroll
      for (int c = 0; c < Hn; ++c) {
        const float keep = up ? s[c + Hn] : s[c];
        const float send = up ? s[c] : s[c + Hn];
        s[c] = keep + __shfl_xor(send, OFF, 64);
      }
      if (up) chan += Hn;
      reduce_split<Hn, OFF / 2>(s, lg, chan);
    }
  }
};

// ---------------------------------------------------------------------------
// Path kernel (gathers).
struct PathPlan {
  const int2* items;
  const int32_t* head;  // per window: partial slot of the row ending here that began earlier (-1)
  const int32_t* tail;  // per window: partial slot of the row leaving the window (-1)
  const int32_t* hfix;  // per window: cross-row index of head / tail partial (-1)
  const int32_t* tfix;
  const int32_t* fix;   // per cross row: row, first slot, last slot
  int32_t* cnt;         // per cross row x column tile: arrival counters (zero between launches)
};

// Partial slots are written and read with agent-coherent accesses (relaxed
// agent-scope atomics: sc1, past the per-XCD L2), so publishing them needs no
// L2 write-back/invalidate: the writer waits for its stores to complete
// (s_waitcnt vmcnt(0)) before bumping the arrival counter.
template <typename T>
__device__ __forceinline__ void store_coherent(float* p, const T& v) {
  const float* f = reinterpret_cast<const float*>(&v);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) __hip_atomic_store(p + i, f[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T load_coherent(const float* p) {
  T v;
  float* f = reinterpret_cast<float*>(&v);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i)
    f[i] = __hip_atomic_load(const_cast<float*>(p + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return v;
}

// A group has just stored one partial of cross row `fi` (a heavy row spanning
// windows).  The last of the row's windows to arrive sums all its partial
// slots in slot (= path) order, applies the epilogue and stores the row, then
// re-arms the counter -- no fix-up launch; the sum order is fixed whichever
// window arrives last.
template <int LPR, int VPL, int VEC, typename T, typename ProjT>
__device__ __forceinline__ void finish_cross(const PathPlan& pp, int32_t fi, int lg, const int64_t* colv,
                                             const bool* colok, const T* bv, const float* part, int64_t part_ld,
                                             float* C, int64_t ldc, const Epi& epi, bool store_main,
                                             const ProjT& proj, const ProjArgs& pa) {
  using V = Vec<VEC>;
  __builtin_amdgcn_s_waitcnt(0);  // this group's partial stores have completed
  const int32_t r = pp.fix[3 * fi], sb = pp.fix[3 * fi + 1], se = pp.fix[3 * fi + 2];
  int32_t* ctr = pp.cnt + (int64_t)fi * kMaxColTiles + blockIdx.y;
  int last = 0;
  if (lg == 0) last = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == se - sb;
  last = __shfl(last, (int)(threadIdx.x & 63) - lg, 64);
  if (!last) return;
  T h[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    h[v] = V::zero();
    if (!colok[v]) continue;
    T acc = V::zero();
    const float* p = part + (int64_t)sb * part_ld + colv[v];
    int32_t q = sb;
    for (; q + 3 <= se; q += 4, p += 4 * part_ld) {
      const T p0 = load_coherent<T>(p), p1 = load_coherent<T>(p + part_ld), p2 = load_coherent<T>(p + 2 * part_ld),
              p3 = load_coherent<T>(p + 3 * part_ld);
      V::add(acc, p0); V::add(acc, p1); V::add(acc, p2); V::add(acc, p3);
    }
    for (; q <= se; ++q, p += part_ld) V::add(acc, load_coherent<T>(p));
    h[v] = V::epi(epi, acc, bv[v], r, colv[v]);
    if (store_main) V::store(C + (int64_t)r * ldc + colv[v], h[v]);
  }
  proj.apply(pa, h, r, lg);
  if (lg == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int BLOCK, int LPR, int VPL, int VEC, int U, int NP>
__global__ void __launch_bounds__(BLOCK)
spmm_path_kernel(PathPlan pp, int32_t ipc, const float* __restrict__ B, int64_t ldb, int32_t F,
                 float* __restrict__ C, int64_t ldc, Epi epi, float* __restrict__ part, int64_t part_ld,
                 ProjArgs pa) {
  const int2* __restrict__ items = pp.items;
  using V = Vec<VEC>;
  using T = typename V::T;
  constexpr int G = BLOCK / LPR;
  constexpr int FT = LPR * VPL * VEC;  // columns per tile
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];

  const int W = G * ipc;
  // LDS: item[W + 1] (index 0 = the item before the window) | per-group words | H, T partials
  int2* s_item = reinterpret_cast<int2*>(smem);
  int32_t* s_meta = smem + 2 * ((W + 2 + 1) & ~1);  // 4 words per group: has_marker, head_partial, tail, head_row
  float* s_H = reinterpret_cast<float*>(s_meta + ((4 * G + 3) & ~3));
  float* s_T = s_H + G * FT;

  const int tid = threadIdx.x;
  const int64_t w = blockIdx.x;
  const int64_t base = w * W;

  // ---- one coalesced pass: the window's items (+ the item before it)
  for (int i = tid; i < W; i += BLOCK) s_item[1 + i] = items[base + i];
  if (tid == 0) s_item[0] = w > 0 ? items[base - 1] : make_int2(kMarker, -1);
  stamp(epi, 0);
  const int32_t hslot = pp.head[w];
  const int32_t tslot = pp.tail[w];
  __syncthreads();
  stamp(epi, 1);

  const int g = tid / LPR;
  const int lg = tid % LPR;
  const int64_t col_base = (int64_t)blockIdx.y * FT;
  int64_t colv[VPL];
  bool colok[VPL];
  T bv[VPL];  // bias of this lane's columns, loaded once
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    colv[v] = col_base + (int64_t)(v * LPR + lg) * VEC;
    colok[v] = colv[v] < F;
    bv[v] = (epi.bias && colok[v]) ? V::load(epi.bias + colv[v]) : V::zero();
  }
  Proj<NP, LPR, VPL, VEC> proj;
  proj.load(pa, F, colv, colok);
  const bool store_main = NP == 0 || pa.store_main;
  float* myH = s_H + g * FT;
  float* myT = s_T + g * FT;

  const int i0 = 1 + g * ipc;                       // first item of this group's chunk in s_item
  const bool head_partial = s_item[i0 - 1].x >= 0;  // the chunk starts inside a row
  bool has_marker = false;
  int32_t head_row = -1;

  T acc[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) acc[v] = V::zero();

  for (int k0 = 0; k0 < ipc; k0 += U) {
    T gv[U][VPL];
    int2 it[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      it[u] = (k0 + u < ipc) ? s_item[i0 + k0 + u] : make_int2(kPad, 0);
      const float* brow = B + (int64_t)(it[u].x >= 0 ? it[u].x : 0) * ldb;
#pragma unroll
      for (int v = 0; v < VPL; ++v)
        gv[u][v] = (it[u].x >= 0 && colok[v]) ? V::load(brow + colv[v]) : V::zero();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (it[u].x >= 0) {
        const float a = __int_as_float(it[u].y);
#pragma unroll
        for (int v = 0; v < VPL; ++v) V::fma(acc[v], a, gv[u][v]);
      } else if (it[u].x == kMarker) {
        const int32_t r = it[u].y;
        if (!has_marker && head_partial) {
#pragma unroll
          for (int v = 0; v < VPL; ++v) V::store(myH + (v * LPR + lg) * VEC, acc[v]);
          head_row = r;
        } else {
          float* dst = C + (int64_t)r * ldc;
          T h[VPL];
#pragma unroll
          for (int v = 0; v < VPL; ++v) {
            h[v] = colok[v] ? V::epi(epi, acc[v], bv[v], r, colv[v]) : V::zero();
            if (colok[v] && store_main) V::store(dst + colv[v], h[v]);
          }
          proj.apply(pa, h, r, lg);
        }
        has_marker = true;
#pragma unroll
        for (int v = 0; v < VPL; ++v) acc[v] = V::zero();
      }
    }
  }
  const bool tail = s_item[i0 + ipc - 1].x >= 0;  // the chunk ends inside a row
  if (tail) {
#pragma unroll
    for (int v = 0; v < VPL; ++v) V::store(myT + (v * LPR + lg) * VEC, acc[v]);
  }
  stamp(epi, 2);
  if (lg == 0) {
    s_meta[4 * g + 0] = has_marker;
    s_meta[4 * g + 1] = head_partial;
    s_meta[4 * g + 2] = tail;
    s_meta[4 * g + 3] = head_row;
  }
  __syncthreads();

  // ---- rows split between groups of this window: the marker's group adds, in group order,
  //      T of the nearest earlier group holding a marker (the row's start) and T of the
  //      marker-free groups in between, then its own H.
  if (head_row >= 0) {
    int j = g - 1;
    while (j >= 0 && !s_meta[4 * j + 0]) --j;
    // the row starts in group j's tail if j ends inside a row, else at group j+1
    const int jf = (j >= 0 && s_meta[4 * j + 2]) ? j : j + 1;
    const bool from_before = j < 0 && s_meta[1];  // the row started in an earlier window
    T h[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int off = (v * LPR + lg) * VEC;
      T s = V::zero();
      for (int q = jf; q < g; ++q) V::add(s, V::load(s_T + q * FT + off));
      V::add(s, V::load(myH + off));
      h[v] = V::zero();
      if (!colok[v]) continue;
      if (from_before) {
        store_coherent(part + (int64_t)hslot * part_ld + colv[v], s);
      } else {
        h[v] = V::epi(epi, s, bv[v], head_row, colv[v]);
        if (store_main) V::store(C + (int64_t)head_row * ldc + colv[v], h[v]);
      }
    }
    if (!from_before) proj.apply(pa, h, head_row, lg);
    else finish_cross<LPR, VPL, VEC>(pp, pp.hfix[w], lg, colv, colok, bv, part, part_ld, C, ldc, epi, store_main,
                                     proj, pa);
  }
  // ---- a heavy row leaving the window: partial of its part in this window
  if (g == G - 1 && tail) {
    int j = g;
    while (j >= 0 && !s_meta[4 * j + 0]) --j;
    const int jf = (j >= 0 && s_meta[4 * j + 2]) ? j : j + 1;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int off = (v * LPR + lg) * VEC;
      T s = V::zero();
      for (int q = jf; q <= g; ++q) V::add(s, V::load(s_T + q * FT + off));
      if (colok[v]) store_coherent(part + (int64_t)tslot * part_ld + colv[v], s);
    }
    finish_cross<LPR, VPL, VEC>(pp, pp.tfix[w], lg, colv, colok, bv, part, part_ld, C, ldc, epi, store_main, proj,
                                pa);
  }
  stamp(epi, 3);
}

// ---------------------------------------------------------------------------
// Tile kernel (dense blocks, fp32 MFMA 16x16x4).  One workgroup = one chunk
// (64 rows x 64 condensed columns) x NT 16-column n-tiles; wave t owns rows
// 16t..16t+15.  The chunk's 64 B rows are staged once in LDS lane-major,
// [k][col & 15][nt] with NT4 = NT rounded up to 4 (+4 pad: 80-B lane rows
// put a 16-lane ds_read_b128 group on 16 disjoint bank quads), so each lane
// fetches the NT operands of a k-step with NT4/4 ds_read_b128.  Each wave's
// A fragments come pre-swizzled from the plan (16 floats per lane,
// contiguous).  acc[nt] += A(16x4) * B(4x16) over 16 k-steps.
//   A operand lane l: A[row l&15][k l>>4];  B operand: B[k l>>4][col l&15];
//   C/D reg j: row (l>>4)*4 + j, col l&15   (gfx950 16x16x4 f32 maps).
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool VEC4, int NT>
__global__ void __launch_bounds__(256)
spmm_tile_kernel(const int4* __restrict__ tdesc, const int32_t* __restrict__ tcols, const float* __restrict__ tfrag,
                 const int32_t* __restrict__ trows, const float* __restrict__ dval, int32_t F,
                 const float* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc, Epi epi,
                 float* __restrict__ slabs, int64_t slab_ld) {
  constexpr int NT4 = (NT + 3) & ~3;
  // floats per (k, lane column) row: an odd number of 16-B quads keeps the 16 lanes
  // of a ds_read_b128 group on disjoint bank quads
  constexpr int LR = ((NT4 / 4) & 1) ? NT4 : NT4 + 4;
  constexpr int stride = 16 * LR;       // floats per k
  __shared__ __attribute__((aligned(16))) float s_B[kKC * stride];
  __shared__ int32_t s_cols[kKC];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t item = blockIdx.x;
  stamp(epi, 0);
  const int4 d = tdesc[item];  // block, nrows, slab (-1: single chunk), 0
  constexpr int32_t col0 = 0;  // column slices are folded into the B/C pointers by the host

  if (tid < kKC) s_cols[tid] = tcols[item * kKC + tid];
  // A fragments of this wave: 16 consecutive floats per lane
  const float4* af = reinterpret_cast<const float4*>(tfrag + ((item * 4 + wave) * 64 + lane) * 16);
  const float4 a0 = af[0], a1 = af[1], a2 = af[2], a3 = af[3];
  __syncthreads();
  // ---- stage the chunk's B rows, columns [0, 16*NT): element (k, n) -> s_B[k][n&15][n>>4]
  // all of a thread's loads issue before any LDS store (one memory latency, not PT)
  constexpr int nq = NT * 4;  // float4 per staged row
  constexpr int PT = (kKC * nq + 255) / 256;
  float4 v[PT];
#pragma unroll
  for (int p = 0; p < PT; ++p) {
    const int q = tid + p * 256;
    const int k = q / nq, c4 = q % nq;
    const int32_t src = q < kKC * nq ? s_cols[k] : -1;
    const int64_t col = col0 + c4 * 4;
    v[p] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (src >= 0) {
      const float* bp = B + (int64_t)src * ldb + col;
      if (VEC4) {
        if (col < F) v[p] = *reinterpret_cast<const float4*>(bp);
      } else {
        if (col + 0 < F) v[p].x = bp[0];
        if (col + 1 < F) v[p].y = bp[1];
        if (col + 2 < F) v[p].z = bp[2];
        if (col + 3 < F) v[p].w = bp[3];
      }
    }
  }
#pragma unroll
  for (int p = 0; p < PT; ++p) {
    const int q = tid + p * 256;
    if (q >= kKC * nq) break;
    const int k = q / nq, c4 = q % nq;
    const int n = c4 * 4, nt = n >> 4, nc0 = n & 15;
    float* dst = s_B + k * stride + nc0 * LR + nt;
    dst[0] = v[p].x;
    dst[LR] = v[p].y;
    dst[2 * LR] = v[p].z;
    dst[3 * LR] = v[p].w;
  }
  __syncthreads();
  stamp(epi, 1);

  f32x4 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float a[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                       a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
  const int kr = lane >> 4, nc = lane & 15;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const float4* brow = reinterpret_cast<const float4*>(s_B + (4 * s + kr) * stride + nc * LR);
    float4 bq[NT4 / 4];
#pragma unroll
    for (int q = 0; q < NT4 / 4; ++q) bq[q] = brow[q];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const float4& b4 = bq[nt >> 2];
      const float bval = (nt & 3) == 0 ? b4.x : (nt & 3) == 1 ? b4.y : (nt & 3) == 2 ? b4.z : b4.w;
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bval, acc[nt], 0, 0, 0);
    }
  }

  stamp(epi, 2);
  // ---- output: block rows 16*wave + 4*(lane>>4) + j, cols col0 + 16*nt + (lane&15);
  //      single-chunk blocks finish here (+ extracted diagonal, epilogue), others
  //      leave a slab for spmm_tile_reduce_kernel
  int32_t orow[4];
  float dv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int32_t rl = 16 * wave + 4 * (lane >> 4) + j;
    orow[j] = rl < d.y ? trows[(int64_t)d.x * kRB + rl] : -1;
    dv[j] = (d.z < 0 && dval && orow[j] >= 0) ? dval[orow[j]] : 0.f;
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int64_t col = col0 + nt * 16 + nc;
    if (col >= F) continue;
    const float bcol = (d.z < 0 && epi.bias) ? epi.bias[col] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (orow[j] < 0) continue;
      if (d.z < 0) {
        float v = acc[nt][j];
        if (dv[j] != 0.f) v = fmaf(dv[j], B[(int64_t)orow[j] * ldb + col], v);
        C[(int64_t)orow[j] * ldc + col] = apply_epi(epi, v, bcol, orow[j], col);
      } else {
        const int32_t rl = 16 * wave + 4 * (lane >> 4) + j;
        slabs[((int64_t)d.z * kRB + rl) * slab_ld + col] = acc[nt][j];
      }
    }
  }
  stamp(epi, 3);
}

// Multi-chunk dense blocks: out[row, :] = epi(sum over the block's slabs, in
// chunk order).  256 threads = 16 slab lanes x 16 float4 column lanes; a
// workgroup covers one row x 64 columns; slab lanes take slabs strided by 16,
// then the 16 partial sums are added in lane order through LDS.
__global__ void __launch_bounds__(256)
spmm_tile_reduce_kernel(const int4* __restrict__ red, const int32_t* __restrict__ trows,
                        const float* __restrict__ dval, int32_t F, const float* __restrict__ slabs, int64_t slab_ld,
                        const float* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc, Epi epi) {
  __shared__ float4 s_acc[16][16];
  const int4 rb = red[blockIdx.x];  // block, nrows, first slab, nslabs
  const int32_t rl = blockIdx.y;    // row within block
  if (rl >= rb.y) return;
  const int sl = threadIdx.x >> 4, c4 = threadIdx.x & 15;
  const int64_t col = (int64_t)blockIdx.z * 64 + c4 * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  // slab rows are padded to 16 floats (slab_ld % 16 == 0): whole float4 reads stay
  // inside the row; lanes past F are never stored.  Four slabs in flight per lane.
  if (col < F) {
    const int64_t step = (int64_t)16 * kRB * slab_ld;
    const float* p = slabs + ((int64_t)(rb.z + sl) * kRB + rl) * slab_ld + col;
    int s = sl;
    for (; s + 48 < rb.w; s += 64, p += 4 * step) {
      const float4 u0 = *reinterpret_cast<const float4*>(p);
      const float4 u1 = *reinterpret_cast<const float4*>(p + step);
      const float4 u2 = *reinterpret_cast<const float4*>(p + 2 * step);
      const float4 u3 = *reinterpret_cast<const float4*>(p + 3 * step);
      acc.x += u0.x; acc.y += u0.y; acc.z += u0.z; acc.w += u0.w;
      acc.x += u1.x; acc.y += u1.y; acc.z += u1.z; acc.w += u1.w;
      acc.x += u2.x; acc.y += u2.y; acc.z += u2.z; acc.w += u2.w;
      acc.x += u3.x; acc.y += u3.y; acc.z += u3.z; acc.w += u3.w;
    }
    for (; s < rb.w; s += 16, p += step) {
      const float4 u = *reinterpret_cast<const float4*>(p);
      acc.x += u.x; acc.y += u.y; acc.z += u.z; acc.w += u.w;
    }
  }
  s_acc[sl][c4] = acc;
  __syncthreads();
  if (sl != 0 || col >= F) return;
  float4 t = s_acc[0][c4];
  for (int q = 1; q < 16; ++q) {
    const float4 u = s_acc[q][c4];
    t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
  }
  const int64_t row = trows[(int64_t)rb.x * kRB + rl];
  const float dv = dval ? dval[row] : 0.f;
  float vals[4] = {t.x, t.y, t.z, t.w};
  for (int i = 0; i < 4 && col + i < F; ++i) {
    if (dv != 0.f) vals[i] = fmaf(dv, B[row * ldb + col + i], vals[i]);
    const float b = epi.bias ? epi.bias[col + i] : 0.f;
    C[row * ldc + col + i] = apply_epi(epi, vals[i], b, row, col + i);
  }
}

// ---------------------------------------------------------------------------
// Dispatch

inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// Lanes per group from F alone (so a plan's G does not depend on pointer
// alignment, which only picks VEC/VPL at launch).
inline int choose_lpr(int32_t F, int lanes_hint) {
  if (lanes_hint > 0) return next_pow2(lanes_hint > 64 ? 64 : lanes_hint);
  const int Wv = (F % 4 == 0) ? F / 4 : F;
  return Wv <= 64 ? next_pow2(Wv < 1 ? 1 : Wv) : 64;
}

// Workgroup size: small groups use one wave so a window holds at most 32 groups
// (bounds the in-LDS chain walk of split rows).
inline int choose_block(int lpr) { return lpr >= 8 ? 256 : 64; }
inline int choose_groups(int32_t F, int lanes_hint) {
  const int lpr = choose_lpr(F, lanes_hint);
  return choose_block(lpr) / lpr;
}

struct Cfg {
  int lpr, vpl, vec, col_tiles, block;
};

inline Cfg choose_cfg(int32_t F, int vec, int lpr) {
  Cfg c;
  c.vec = vec;
  c.lpr = lpr;
  c.block = choose_block(lpr);
  const int Wv = (F + vec - 1) / vec;
  int vpl = (Wv + lpr - 1) / lpr;
  vpl = vpl <= 1 ? 1 : (vpl <= 2 ? 2 : 4);
  c.vpl = vpl;
  c.col_tiles = (Wv + lpr * vpl - 1) / (lpr * vpl);
  return c;
}

constexpr int kMaxLds = 65536;

inline size_t lds_bytes(int G, int ipc, int FT) {
  const int W = G * ipc;
  return (size_t)(2 * ((W + 2 + 1) & ~1) + ((4 * G + 3) & ~3) + 2 * G * FT) * 4;
}

struct Launch {
  const int32_t* plan;
  Layout L;
  int32_t ipc, nfix;
  const float* B;
  int64_t ldb;
  int32_t F;
  float* C;
  int64_t ldc;
  Epi epi;
  float* part;  // path partial slots
  int64_t part_ld;
  int col_tiles;
  ProjArgs pa;
  hipStream_t s;
};

template <int BLOCK, int LPR, int VPL, int VEC, int NP>
int launch_path(const Launch& a) {
  constexpr int G = BLOCK / LPR;
  constexpr int UB = NP > 0 ? 8 : 16;  // the projection holds W in registers: shorter batches
  constexpr int U = (UB / VPL) < 2 ? 2 : UB / VPL;
  const size_t lds = lds_bytes(G, a.ipc, LPR * VPL * VEC);
  if (lds > (size_t)kMaxLds) {
    set_error("gcnk_spmm_csr_f32: ipc %d needs %zu B of LDS (> %d) at %d groups", a.ipc, lds, kMaxLds, G);
    return GCNK_EUNSUP;
  }
  if (a.col_tiles > kMaxColTiles) {
    set_error("gcnk_spmm_csr_f32: F=%d needs %d column tiles (> %d)", a.F, a.col_tiles, kMaxColTiles);
    return GCNK_EUNSUP;
  }
  if (a.L.nwin == 0) return GCNK_OK;
  PathPlan pp{reinterpret_cast<const int2*>(a.plan + a.L.items), a.plan + a.L.head, a.plan + a.L.tail,
              a.plan + a.L.hfix, a.plan + a.L.tfix, a.plan + a.L.fix, const_cast<int32_t*>(a.plan + a.L.cnt)};
  hipLaunchKernelGGL((spmm_path_kernel<BLOCK, LPR, VPL, VEC, U, NP>), dim3((unsigned)a.L.nwin, a.col_tiles),
                     dim3(BLOCK), lds, a.s, pp, a.ipc, a.B, a.ldb, a.F, a.C, a.ldc, a.epi, a.part, a.part_ld, a.pa);
  return launch_check("spmm_path_kernel");
}

template <int VEC>
int dispatch_path(const Cfg& c, const Launch& a) {
#define GCNK_CASE(BL, L, P) \
  if (c.block == BL && c.lpr == L && c.vpl == P) return launch_path<BL, L, P, VEC, 0>(a);
  GCNK_CASE(64, 1, 1) GCNK_CASE(64, 2, 1) GCNK_CASE(64, 4, 1) GCNK_CASE(256, 8, 1) GCNK_CASE(256, 16, 1)
  GCNK_CASE(256, 32, 1) GCNK_CASE(256, 64, 1) GCNK_CASE(64, 1, 2) GCNK_CASE(64, 2, 2) GCNK_CASE(64, 4, 2)
  GCNK_CASE(256, 8, 2) GCNK_CASE(256, 16, 2) GCNK_CASE(256, 32, 2) GCNK_CASE(256, 64, 2) GCNK_CASE(64, 1, 4)
  GCNK_CASE(64, 2, 4) GCNK_CASE(64, 4, 4) GCNK_CASE(256, 8, 4) GCNK_CASE(256, 16, 4) GCNK_CASE(256, 32, 4)
  GCNK_CASE(256, 64, 4)
#undef GCNK_CASE
  set_error("gcnk_spmm_csr_f32: unsupported lanes/vectors config (%d,%d)", c.lpr, c.vpl);
  return GCNK_EUNSUP;
}

// Fused projection variants: float4 columns, one column tile, groups of >= 16 lanes.
template <int NP>
int dispatch_path_proj(const Cfg& c, const Launch& a) {
#define GCNK_CASE(L, P) \
  if (c.block == 256 && c.lpr == L && c.vpl == P) return launch_path<256, L, P, 4, NP>(a);
  GCNK_CASE(16, 1) GCNK_CASE(32, 1) GCNK_CASE(64, 1) GCNK_CASE(16, 2) GCNK_CASE(32, 2) GCNK_CASE(64, 2)
  GCNK_CASE(16, 4) GCNK_CASE(32, 4) GCNK_CASE(64, 4)
#undef GCNK_CASE
  set_error("gcnk_spmm_proj_f32: no fused-projection kernel for lanes/vectors (%d,%d)", c.lpr, c.vpl);
  return GCNK_EUNSUP;
}

struct TileArgs {
  const int4* tdesc;
  const int32_t* tcols;
  const float* tfrag;
  const int32_t* trows;
  const float* dval;
  int32_t F;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  Epi epi;
  float* slabs;
  int64_t slab_ld;
};

template <bool V4, int NT>
int launch_tile_nt(unsigned nitems, const TileArgs& t, hipStream_t s) {
  hipLaunchKernelGGL((spmm_tile_kernel<V4, NT>), dim3(nitems), dim3(256), 0, s, t.tdesc, t.tcols, t.tfrag, t.trows, t.dval, t.F, t.B,
                     t.ldb, t.C, t.ldc, t.epi, t.slabs, t.slab_ld);
  return launch_check("spmm_tile_kernel");
}

template <bool V4>
int launch_tile_v(int nt_need, unsigned nitems, const TileArgs& t, hipStream_t s) {
  if (nt_need <= 1) return launch_tile_nt<V4, 1>(nitems, t, s);
  if (nt_need <= 2) return launch_tile_nt<V4, 2>(nitems, t, s);
  if (nt_need <= 4) return launch_tile_nt<V4, 4>(nitems, t, s);
  if (nt_need <= 8) return launch_tile_nt<V4, 8>(nitems, t, s);
  if (nt_need <= 13) return launch_tile_nt<V4, 13>(nitems, t, s);
  if (nt_need <= kMaxNT) return launch_tile_nt<V4, kMaxNT>(nitems, t, s);
  set_error("spmm_tile_kernel: %d n-tiles exceed %d", nt_need, kMaxNT);
  return GCNK_EUNSUP;
}

inline int launch_tile(bool v4, int nt_need, unsigned nitems, const TileArgs& t, hipStream_t s) {
  return v4 ? launch_tile_v<true>(nt_need, nitems, t, s) : launch_tile_v<false>(nt_need, nitems, t, s);
}

// ---------------------------------------------------------------------------
// Host side of the plan.
struct HostPlan {
  int32_t hdr[16];
  std::vector<int32_t> start;   // item position of each path row, -1 for tile rows
  std::vector<int32_t> head, tail, hfix, tfix, fix;
  std::vector<int32_t> tdesc, tcols, red, trows;
  std::vector<float> tfrag, dval;  // dval: extracted diagonal of tile rows (M, or empty)
};

int host_plan(const int32_t* rowptr_dev, const int32_t* colind_dev, const float* val_dev, int32_t M, int32_t K,
              int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold, bool want_values, hipStream_t s,
              HostPlan& hp) {
  std::vector<int32_t> rp((size_t)M + 1), ci((size_t)nnz);
  std::vector<float> vv(want_values ? (size_t)nnz : 0);
  int rc = hip_check(hipMemcpyAsync(rp.data(), rowptr_dev, ((size_t)M + 1) * 4, hipMemcpyDeviceToHost, s),
                     "plan rowptr copy");
  if (!rc && nnz > 0)
    rc = hip_check(hipMemcpyAsync(ci.data(), colind_dev, (size_t)nnz * 4, hipMemcpyDeviceToHost, s), "plan colind copy");
  if (!rc && want_values && nnz > 0)
    rc = hip_check(hipMemcpyAsync(vv.data(), val_dev, (size_t)nnz * 4, hipMemcpyDeviceToHost, s), "plan val copy");
  if (rc) return rc;
  if ((rc = hip_check(hipStreamSynchronize(s), "plan copy sync"))) return rc;
  if ((int64_t)rp[M] != nnz || rp[0] != 0) {
    set_error("gcnk_spmm_plan: rowptr[0]=%d rowptr[M]=%d inconsistent with nnz=%lld", rp[0], rp[M], (long long)nnz);
    return GCNK_EARG;
  }
  for (int32_t r = 0; r < M; ++r)
    if (rp[r + 1] < rp[r]) {
      set_error("gcnk_spmm_plan: rowptr decreases at row %d", r);
      return GCNK_EARG;
    }
  for (int64_t k = 0; k < nnz; ++k)
    if (ci[(size_t)k] < 0 || ci[(size_t)k] >= K) {
      set_error("gcnk_spmm_plan: column index %d out of range [0, %d) at nonzero %lld", ci[(size_t)k], K, (long long)k);
      return GCNK_EARG;
    }

  // ---- dense blocks (tile path).  Rows are grouped by degree class (factor-8
  //      buckets of the off-diagonal degree), in row order within a class, 64 per
  //      block, so rows of one shape share blocks (R8: document rows vs topic rows).
  //      A block goes to the MFMA tile path when its nonzeros fill at least
  //      dense_threshold of its condensed column set and each condensed column is
  //      used at least twice on average; its rows' diagonal entries (r < K) are
  //      taken out of the column set and added in the epilogue (dval[r] * B[r,:]).
  std::vector<char> tile_row((size_t)M, 0);
  int32_t ntile = 0, nred = 0, nslabs = 0, ntblk = 0;
  bool any_diag = false;
  hp.dval.clear();
  auto is_diag = [&](int32_t r, int64_t k) { return r < K && ci[(size_t)k] == r; };
  if (dense_threshold <= 1.0f && M > 0) {
    std::vector<std::vector<int32_t>> cls(33);
    for (int32_t r = 0; r < M; ++r) {
      int64_t deg = 0;
      for (int64_t k = rp[r]; k < rp[r + 1]; ++k) deg += !is_diag(r, k);
      int bw = 0;
      while (bw < 63 && (deg >> bw) != 0) ++bw;
      cls[(size_t)(bw / 3)].push_back(r);
    }
    std::vector<int32_t> cmap((size_t)K, -1);
    std::vector<int32_t> cols;
    std::vector<float> dv((size_t)M, 0.f);
    for (const std::vector<int32_t>& rows : cls) {
      for (size_t i0 = 0; i0 < rows.size(); i0 += kRB) {
        const size_t i1 = std::min(rows.size(), i0 + kRB);
        cols.clear();
        int64_t bnnz = 0;
        for (size_t i = i0; i < i1; ++i) {
          const int32_t r = rows[i];
          for (int64_t k = rp[r]; k < rp[r + 1]; ++k)
            if (!is_diag(r, k)) {
              cols.push_back(ci[(size_t)k]);
              ++bnnz;
            }
        }
        if (bnnz == 0) continue;
        std::sort(cols.begin(), cols.end());
        cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
        const int64_t ncols = (int64_t)cols.size();
        const int64_t nrows = (int64_t)(i1 - i0);
        if ((double)bnnz < (double)dense_threshold * (double)nrows * (double)ncols || bnnz < 2 * ncols) continue;
        const int32_t nch = (int32_t)((ncols + kKC - 1) / kKC);
        const int32_t first_slab = nch > 1 ? nslabs : -1;
        const int32_t blk = ntblk++;
        for (int64_t c = 0; c < ncols; ++c) cmap[(size_t)cols[(size_t)c]] = (int32_t)c;
        const size_t base_item = (size_t)ntile;
        for (int32_t ch = 0; ch < nch; ++ch) {
          hp.tdesc.insert(hp.tdesc.end(), {blk, (int32_t)nrows, nch > 1 ? first_slab + ch : -1, 0});
          for (int k = 0; k < kKC; ++k) {
            const int64_t cc = (int64_t)ch * kKC + k;
            hp.tcols.push_back(cc < ncols ? cols[(size_t)cc] : -1);
          }
        }
        for (int64_t rl = 0; rl < kRB; ++rl) hp.trows.push_back(rl < nrows ? rows[i0 + (size_t)rl] : -1);
        hp.tfrag.resize(hp.tfrag.size() + (size_t)nch * kRB * kKC, 0.f);
        for (size_t i = i0; i < i1; ++i) {
          const int32_t r = rows[i];
          const int32_t rl = (int32_t)(i - i0), t = rl / 16, lr = rl % 16;
          tile_row[(size_t)r] = 1;
          for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
            if (is_diag(r, k)) {
              any_diag = true;
              if (want_values) dv[(size_t)r] += vv[(size_t)k];
              continue;
            }
            if (!want_values) continue;
            const int32_t cc = cmap[(size_t)ci[(size_t)k]];
            const int32_t ch = cc / kKC, kk = cc % kKC;
            const int32_t st = kk / 4, kq = kk % 4;
            const int32_t ln = kq * 16 + lr;
            hp.tfrag[(((base_item + ch) * 4 + t) * 64 + ln) * 16 + st] += vv[(size_t)k];
          }
        }
        for (int64_t c = 0; c < ncols; ++c) cmap[(size_t)cols[(size_t)c]] = -1;
        if (nch > 1) {
          hp.red.insert(hp.red.end(), {blk, (int32_t)nrows, first_slab, nch});
          ++nred;
          nslabs += nch;
        }
        ntile += nch;
      }
    }
    if (any_diag) hp.dval = std::move(dv);
  }

  // ---- path windows over the other rows
  const int64_t W = (int64_t)groups * ipc;
  const int64_t heavy = W / 2;
  hp.start.assign((size_t)M, -1);
  int64_t pos = 0;
  for (int32_t r = 0; r < M; ++r) {
    if (tile_row[(size_t)r]) continue;
    const int64_t len = (int64_t)rp[r + 1] - rp[r] + 1;
    const int64_t off = pos % W;
    if (len <= heavy && off + len > W) pos += W - off;
    hp.start[(size_t)r] = (int32_t)pos;
    pos += len;
    if (pos >= (int64_t)INT32_MAX) {
      set_error("gcnk_spmm_plan: item stream exceeds 2^31 items");
      return GCNK_EUNSUP;
    }
  }
  const int64_t nwin = (pos + W - 1) / W;
  hp.head.assign((size_t)nwin, -1);
  hp.tail.assign((size_t)nwin, -1);
  // heavy rows crossing window boundaries: tail slot in every window they leave,
  // head slot in the window of their marker; slots numbered in window order,
  // a window's head before its tail (contiguous per row).
  struct Cross { int32_t row; int64_t wa, wb; };
  std::vector<Cross> cross;
  for (int32_t r = 0; r < M; ++r) {
    if (hp.start[(size_t)r] < 0) continue;
    const int64_t a0 = hp.start[(size_t)r], e = a0 + (rp[r + 1] - rp[r]);  // e = marker position
    const int64_t wa = a0 / W, wb = e / W;
    if (wa < wb) cross.push_back({r, wa, wb});
  }
  for (const Cross& c : cross) {
    for (int64_t x = c.wa; x < c.wb; ++x) hp.tail[(size_t)x] = 1;
    hp.head[(size_t)c.wb] = 1;
  }
  int32_t slot = 0;
  for (int64_t x = 0; x < nwin; ++x) {
    if (hp.head[(size_t)x] >= 0) hp.head[(size_t)x] = slot++;
    if (hp.tail[(size_t)x] >= 0) hp.tail[(size_t)x] = slot++;
  }
  hp.hfix.assign((size_t)nwin, -1);
  hp.tfix.assign((size_t)nwin, -1);
  for (size_t i = 0; i < cross.size(); ++i) {
    const Cross& c = cross[i];
    hp.fix.insert(hp.fix.end(), {c.row, hp.tail[(size_t)c.wa], hp.head[(size_t)c.wb]});
    for (int64_t x = c.wa; x < c.wb; ++x) hp.tfix[(size_t)x] = (int32_t)i;
    hp.hfix[(size_t)c.wb] = (int32_t)i;
  }
  const int32_t h[16] = {kMagic, M, K, groups, ipc, (int32_t)W, (int32_t)nwin, (int32_t)cross.size(), slot,
                         ntile, nred, nslabs, ntblk, any_diag ? 1 : 0, (int32_t)heavy, 0};
  std::copy(h, h + 16, hp.hdr);
  return GCNK_OK;
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

static unsigned long long* g_stamps = nullptr;
extern "C" void gcnk_debug_set_stamps(void* buf) { g_stamps = (unsigned long long*)buf; }

extern "C" int32_t gcnk_spmm_groups(int32_t F, int32_t lanes_hint) { return choose_groups(F, lanes_hint); }

extern "C" int32_t gcnk_spmm_default_ipc(int32_t M, int64_t nnz, int32_t F, int32_t lanes_hint) {
  (void)M;
  (void)nnz;
  const int lpr = choose_lpr(F, lanes_hint);
  const int G = choose_block(lpr) / lpr;
  const Cfg c = choose_cfg(F, F % 4 == 0 ? 4 : 1, lpr);
  int ipc = lpr >= 16 ? 16 : 8;
  while (ipc > 2 && lds_bytes(G, ipc, lpr * c.vpl * c.vec) > (size_t)kMaxLds) ipc /= 2;
  return ipc;
}

extern "C" int64_t gcnk_spmm_plan_bytes(const int32_t* rowptr, const int32_t* colind, int32_t M, int32_t K,
                                        int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold,
                                        void* stream) {
  if (!rowptr || M < 0 || K < 0 || nnz < 0 || ipc <= 0 || groups <= 0 || (nnz > 0 && !colind)) {
    set_error("gcnk_spmm_plan_bytes: bad argument");
    return GCNK_EARG;
  }
  HostPlan hp;
  const int rc = host_plan(rowptr, colind, nullptr, M, K, nnz, ipc, groups, dense_threshold, false,
                           (hipStream_t)stream, hp);
  if (rc) return rc;
  // + M words of scratch (path row start positions) used while building
  return (Layout(hp.hdr).total + M) * 4;
}

extern "C" int gcnk_spmm_plan_build(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                                    int32_t K, int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold,
                                    void* plan, int64_t plan_bytes, void* stream) {
  if (!rowptr || !plan || M < 0 || K < 0 || nnz < 0 || ipc <= 0 || groups <= 0 || (nnz > 0 && (!colind || !val))) {
    set_error("gcnk_spmm_plan_build: bad argument (M=%d nnz=%lld ipc=%d groups=%d)", M, (long long)nnz, ipc, groups);
    return GCNK_EARG;
  }
  hipStream_t s = (hipStream_t)stream;
  HostPlan hp;
  int rc = host_plan(rowptr, colind, val, M, K, nnz, ipc, groups, dense_threshold, true, s, hp);
  if (rc) return rc;
  const Layout L(hp.hdr);
  if (plan_bytes < (L.total + M) * 4) {
    set_error("gcnk_spmm_plan_build: plan buffer %lld B < %lld B", (long long)plan_bytes,
              (long long)((L.total + M) * 4));
    return GCNK_EARG;
  }
  int32_t* p = (int32_t*)plan;
  int32_t* d_start = p + L.total;  // scratch words after the plan proper
  auto up = [&](int64_t off, const void* src, size_t bytes, const char* what) {
    if (!rc && bytes > 0) rc = hip_check(hipMemcpyAsync(p + off, src, bytes, hipMemcpyHostToDevice, s), what);
  };
  up(0, hp.hdr, sizeof(hp.hdr), "plan header");
  up(L.head, hp.head.data(), hp.head.size() * 4, "plan head");
  up(L.tail, hp.tail.data(), hp.tail.size() * 4, "plan tail");
  up(L.hfix, hp.hfix.data(), hp.hfix.size() * 4, "plan head rows");
  up(L.tfix, hp.tfix.data(), hp.tfix.size() * 4, "plan tail rows");
  up(L.fix, hp.fix.data(), hp.fix.size() * 4, "plan fix");
  if (!rc && L.nfix > 0)
    rc = hip_check(hipMemsetAsync(p + L.cnt, 0, (size_t)L.nfix * kMaxColTiles * 4, s), "plan counters");
  up(L.tdesc, hp.tdesc.data(), hp.tdesc.size() * 4, "plan tile desc");
  up(L.tcols, hp.tcols.data(), hp.tcols.size() * 4, "plan tile cols");
  up(L.tfrag, hp.tfrag.data(), hp.tfrag.size() * 4, "plan tile frags");
  up(L.red, hp.red.data(), hp.red.size() * 4, "plan tile reduce");
  up(L.trows, hp.trows.data(), hp.trows.size() * 4, "plan tile rows");
  up(L.dval, hp.dval.data(), hp.dval.size() * 4, "plan diagonal");
  up(L.total, hp.start.data(), hp.start.size() * 4, "plan start");
  const int64_t nitems = L.nwin * L.W;
  int2* items = reinterpret_cast<int2*>(p + L.items);
  if (!rc && nitems > 0) {
    hipLaunchKernelGGL(fill_pad_kernel, dim3((unsigned)((nitems + 255) / 256)), dim3(256), 0, s, items, nitems);
    rc = launch_check("fill_pad_kernel");
  }
  if (!rc && M > 0 && nitems > 0) {
    hipLaunchKernelGGL(scatter_items_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, rowptr, colind, val, M,
                       d_start, items);
    rc = launch_check("scatter_items_kernel");
  }
  // the host vectors must outlive the async copies
  const int rc2 = hip_check(hipStreamSynchronize(s), "plan build sync");
  return rc ? rc : rc2;
}

extern "C" int gcnk_spmm_plan_query(const void* plan, int32_t* out16, void* stream) {
  if (!plan || !out16) {
    set_error("gcnk_spmm_plan_query: null pointer");
    return GCNK_EARG;
  }
  hipStream_t s = (hipStream_t)stream;
  int rc = hip_check(hipMemcpyAsync(out16, plan, 64, hipMemcpyDeviceToHost, s), "plan query copy");
  if (rc) return rc;
  rc = hip_check(hipStreamSynchronize(s), "plan query sync");
  if (!rc && out16[0] != kMagic) {
    set_error("gcnk_spmm_plan_query: not a gcnk plan");
    return GCNK_EARG;
  }
  return rc;
}

static int64_t tile_fpad(int32_t F) { return ((int64_t)F + 15) & ~15LL; }

extern "C" int64_t gcnk_spmm_workspace_bytes(const int32_t* hdr, int32_t F) {
  if (!hdr || hdr[0] != kMagic || F < 0) return GCNK_EARG;
  const int64_t ld = ((int64_t)F + 3) & ~3LL;
  const int64_t path = (int64_t)hdr[8] * ld * 4;
  const int64_t slabs = (int64_t)hdr[11] * kRB * tile_fpad(F) * 4;
  return ((path + 255) & ~255LL) + slabs;
}

static int spmm_impl(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F, float* C,
                     int64_t ldc, const float* bias, int32_t epilogue, const uint8_t* drop_mask, int64_t ldm,
                     float drop_scale, float keep_prob, uint64_t seed, uint64_t offset, float* workspace,
                     int64_t workspace_bytes, int32_t lanes_hint, const ProjArgs& pa, void* stream) {
  if (!plan || !hdr || hdr[0] != kMagic || F < 0) {
    set_error("gcnk_spmm_csr_f32: bad argument (plan/header missing or not a gcnk plan, F=%d)", F);
    return GCNK_EARG;
  }
  const int32_t M = hdr[1], K = hdr[2], groups = hdr[3], ipc = hdr[4];
  if (M == 0 || F == 0) return GCNK_OK;
  const bool proj = pa.W != nullptr;
  if (proj && (!pa.C2 || pa.P <= 0 || pa.ldw < pa.P || pa.ldc2 < pa.P)) {
    set_error("gcnk_spmm_proj_f32: bad projection (P=%d)", pa.P);
    return GCNK_EARG;
  }
  if ((!C && (!proj || pa.store_main)) || (K > 0 && !B)) {
    set_error("gcnk_spmm_csr_f32: null pointer");
    return GCNK_EARG;
  }
  if (ldb < F || ldc < F) {
    set_error("gcnk_spmm_csr_f32: leading dimension smaller than F (ldb=%lld ldc=%lld F=%d)", (long long)ldb,
              (long long)ldc, F);
    return GCNK_EARG;
  }
  if (epilogue < GCNK_EPI_NONE || epilogue > GCNK_EPI_BIAS_RELU_HASH) {
    set_error("gcnk_spmm_csr_f32: unknown epilogue %d", epilogue);
    return GCNK_EARG;
  }
  if (epilogue == GCNK_EPI_BIAS_RELU_DROP && (!drop_mask || ldm < F)) {
    set_error("gcnk_spmm_csr_f32: dropout epilogue needs a mask with ldm >= F");
    return GCNK_EARG;
  }
  const int lpr = choose_lpr(F, lanes_hint);
  if (groups != choose_block(lpr) / lpr) {
    set_error("gcnk_spmm_csr_f32: plan built for %d groups, this F/lanes uses %d (gcnk_spmm_groups)", groups,
              choose_block(lpr) / lpr);
    return GCNK_EARG;
  }
  const int64_t need = gcnk_spmm_workspace_bytes(hdr, F);
  if (need > 0 && (!workspace || workspace_bytes < need)) {
    set_error("gcnk_spmm_csr_f32: plan needs %lld B of workspace, got %lld", (long long)need,
              (long long)workspace_bytes);
    return GCNK_EARG;
  }
  Epi e;
  e.bias = bias;
  e.mask = drop_mask;
  e.ldm = epilogue == GCNK_EPI_BIAS_RELU_HASH ? (ldm > 0 ? ldm : F) : ldm;
  e.scale = drop_scale;
  e.keep_prob = keep_prob;
  e.seed_lo = (uint32_t)seed;
  e.seed_hi = (uint32_t)(seed >> 32);
  e.offset = offset;
  e.code = epilogue;
  e.stamps = g_stamps;
  const bool vec4 = (F % 4 == 0) && (ldb % 4 == 0) && (ldc % 4 == 0) && aligned16(B) && aligned16(C) &&
                    (!workspace || aligned16(workspace)) && (!bias || aligned16(bias));
  if (proj) {
    // the projection needs whole rows in one group: path rows only, float4, one column tile
    const Cfg c = choose_cfg(F, 4, lpr);
    if (hdr[9] > 0 || !vec4 || c.col_tiles != 1 || pa.P > 32 || lpr < 16) {
      set_error("gcnk_spmm_proj_f32: fused projection unsupported here (tile rows=%d vec4=%d col_tiles=%d P=%d lanes=%d)",
                hdr[9], (int)vec4, c.col_tiles, pa.P, lpr);
      return GCNK_EUNSUP;
    }
  }
  hipStream_t s = (hipStream_t)stream;
  const int32_t* p = (const int32_t*)plan;
  const Layout L(hdr);
  const int64_t part_ld = ((int64_t)F + 3) & ~3LL;
  const int64_t path_ws = ((int64_t)hdr[8] * part_ld * 4 + 255) & ~255LL;
  float* slabs = workspace ? reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + path_ws) : nullptr;
  const int64_t slab_ld = tile_fpad(F);

  // ---- dense blocks: tile kernel (+ slab reduce)
  const float* dval = L.has_diag ? reinterpret_cast<const float*>(p + L.dval) : nullptr;
  if (L.ntile > 0) {
    const int32_t nt_total = (int32_t)(slab_ld / 16);
    // F <= 16*kMaxNT: one launch over all columns; wider: 128-column slices with the
    // slice offset folded into the B/C/bias/mask pointers (multiples of 4: alignment kept)
    const int32_t slice = nt_total <= kMaxNT ? (int32_t)(nt_total * 16) : 128;
    const int4* td = reinterpret_cast<const int4*>(p + L.tdesc);
    for (int64_t c0 = 0; c0 < F; c0 += slice) {
      const int32_t Fs = (int32_t)std::min<int64_t>(slice, F - c0);
      Epi es = e;
      es.bias = bias ? bias + c0 : nullptr;
      es.mask = drop_mask ? drop_mask + c0 : nullptr;
      es.offset = e.offset + (uint64_t)c0;  // hash index shifts with the column
      TileArgs ta{td,      p + L.tcols, reinterpret_cast<const float*>(p + L.tfrag), p + L.trows, dval, Fs, B + c0,
                  ldb,     C + c0,      ldc, es, slabs ? slabs + c0 : nullptr, slab_ld};
      const int rc = launch_tile(vec4, (Fs + 15) / 16, (unsigned)L.ntile, ta, s);
      if (rc) return rc;
    }
    if (L.nred > 0) {
      hipLaunchKernelGGL(spmm_tile_reduce_kernel, dim3((unsigned)L.nred, kRB, (unsigned)((F + 63) / 64)), dim3(256),
                         0, s, reinterpret_cast<const int4*>(p + L.red), p + L.trows, dval, F, slabs, slab_ld, B, ldb,
                         C, ldc, e);
      int rc = launch_check("spmm_tile_reduce_kernel");
      if (rc) return rc;
    }
  }
  // ---- remaining rows: path kernel (+ fix-up)
  if (L.nwin > 0) {
    const Cfg c = choose_cfg(F, vec4 ? 4 : 1, lpr);
    Launch a{p, L, ipc, (int32_t)L.nfix, B, ldb, F, C, ldc, e, workspace, part_ld, c.col_tiles, pa, s};
    if (proj) return pa.P <= 8 ? dispatch_path_proj<8>(c, a) : dispatch_path_proj<32>(c, a);
    return vec4 ? dispatch_path<4>(c, a) : dispatch_path<1>(c, a);
  }
  return GCNK_OK;
}

extern "C" int gcnk_spmm_csr_f32(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F,
                                 float* C, int64_t ldc, const float* bias, int32_t epilogue, const uint8_t* drop_mask,
                                 int64_t ldm, float drop_scale, float keep_prob, uint64_t seed, uint64_t offset,
                                 float* workspace, int64_t workspace_bytes, int32_t lanes_hint, void* stream) {
  const ProjArgs none{nullptr, 0, 0, nullptr, 0, 1};
  return spmm_impl(plan, hdr, B, ldb, F, C, ldc, bias, epilogue, drop_mask, ldm, drop_scale, keep_prob, seed, offset,
                   workspace, workspace_bytes, lanes_hint, none, stream);
}

extern "C" int gcnk_spmm_proj_f32(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F,
                                  float* C, int64_t ldc, const float* bias, int32_t epilogue,
                                  const uint8_t* drop_mask, int64_t ldm, float drop_scale, float keep_prob,
                                  uint64_t seed, uint64_t offset, const float* W, int64_t ldw, int32_t P, float* C2,
                                  int64_t ldc2, float* workspace, int64_t workspace_bytes, int32_t lanes_hint,
                                  void* stream) {
  if (!W) {
    set_error("gcnk_spmm_proj_f32: null projection matrix");
    return GCNK_EARG;
  }
  const ProjArgs pa{W, ldw, P, C2, ldc2, C != nullptr};
  return spmm_impl(plan, hdr, B, ldb, F, C, ldc, bias, epilogue, drop_mask, ldm, drop_scale, keep_prob, seed, offset,
                   workspace, workspace_bytes, lanes_hint, pa, stream);
}
