// CSR SpMM for gfx950:  C = epi(A_csr * B)
//
// Replaces th.spmm(adj, support) (reference layer.py:106) and th.spmm(X, W)
// with sparse X (layer.py:102), plus their autograd products A^T g / X^T g.
//
// Schedule: merge-path over the sequence of (row ends + nonzeros) cut into
// chunks of `ipc` items (built once per sparsity pattern by
// gcnk_spmm_plan_build).  A boundary landing inside a row shorter than `ipc`
// is snapped back to the start of that row, so light rows are never split;
// heavy rows (e.g. the 50 topic rows of R8, up to 1.8k nonzeros vs a median
// of 5) are split over several chunks and summed in fixed chunk order by a
// fix-up pass: no float atomics, bitwise reproducible.
//
// Kernel shape: 256-thread workgroups.  A workgroup owns G = 256/LPR
// consecutive chunks; it stages their row pointers, column indices, values
// and a per-nonzero row id in LDS with coalesced loads, then each group of
// LPR lanes walks one chunk: batches of U nonzeros are gathered together
// (U*VPL independent 16-B loads in flight per lane), accumulated in fp32
// registers and flushed when the row changes, with bias/ReLU/dropout fused
// into the store.  Each lane owns VEC-wide column vectors interleaved by LPR,
// so one load instruction of a group covers LPR*VEC contiguous floats of a
// B row (coalesced).  F wider than LPR*VPL*VEC is tiled over gridDim.y.
#include "gcnk_common.h"

#include <climits>

namespace gcnk {
namespace {

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
  static __device__ __forceinline__ T epi(const Epi& e, const T& a, int64_t row, int64_t col) {
    T r;
    r.x = apply_epi(e, a.x, row, col + 0);
    r.y = apply_epi(e, a.y, row, col + 1);
    r.z = apply_epi(e, a.z, row, col + 2);
    r.w = apply_epi(e, a.w, row, col + 3);
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
  static __device__ __forceinline__ T epi(const Epi& e, const T& a, int64_t row, int64_t col) {
    return apply_epi(e, a, row, col);
  }
};

// ---------------------------------------------------------------------------
// Plan construction (one-time per sparsity pattern and ipc).

// Merge-path split point of diagonal d over A = row ends (rowptr[1..M]) and
// B = nonzero indices; then snap to the row start when the row is light.
__global__ void plan_coords_kernel(const int32_t* __restrict__ rowptr, int32_t M, int64_t nnz,
                                   int32_t ipc, int64_t nchunks, Coord* __restrict__ coords) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > nchunks) return;
  const int64_t total = (int64_t)M + nnz;
  const int64_t d = min(t * (int64_t)ipc, total);
  int64_t lo = max<int64_t>(0, d - nnz), hi = min<int64_t>(d, M);
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)rowptr[mid + 1] <= d - mid - 1) lo = mid + 1;
    else hi = mid;
  }
  int32_t x = (int32_t)lo;
  int32_t y = (int32_t)(d - lo);
  if (x < M && y > rowptr[x] && (rowptr[x + 1] - rowptr[x]) < ipc) y = rowptr[x];
  coords[t] = Coord{x, y};
}

// Per chunk: does it finish a row it did not start (head partial) and does it
// start a row it does not finish (tail partial)?  Flags are stored in the
// slot arrays and turned into slot numbers by plan_scan_kernel.
__global__ void plan_flags_kernel(const int32_t* __restrict__ rowptr, int32_t M, int64_t nchunks,
                                  const Coord* __restrict__ coords, int32_t* __restrict__ head,
                                  int32_t* __restrict__ tail) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nchunks) return;
  const Coord a = coords[t], b = coords[t + 1];
  head[t] = (a.x < b.x && a.y > rowptr[a.x]) ? 1 : 0;
  tail[t] = (b.x < M && b.y > max(a.y, rowptr[b.x])) ? 1 : 0;
}

// Single-workgroup ordered scan: slots are numbered in chunk order with a
// chunk's head before its tail, so the partials of one split row occupy a
// contiguous slot range ending at the finishing chunk's head slot.
__global__ void __launch_bounds__(1024) plan_scan_kernel(int64_t nchunks, int32_t ipc,
                                                         int32_t* __restrict__ head,
                                                         int32_t* __restrict__ tail,
                                                         int32_t* __restrict__ fix_index,
                                                         int32_t* __restrict__ header) {
  __shared__ int32_t s_slot[16], s_fix[16];
  __shared__ int32_t s_base[2];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  if (tid == 0) { s_base[0] = 0; s_base[1] = 0; }
  __syncthreads();
  for (int64_t base = 0; base < nchunks; base += 1024) {
    const int64_t t = base + tid;
    const int hf = t < nchunks ? head[t] : 0;
    const int tf = t < nchunks ? tail[t] : 0;
    int cs = hf + tf, cf = hf;
    // inclusive wave scans
    for (int o = 1; o < 64; o <<= 1) {
      const int a = __shfl_up(cs, o, 64), b = __shfl_up(cf, o, 64);
      if (lane >= o) { cs += a; cf += b; }
    }
    if (lane == 63) { s_slot[wv] = cs; s_fix[wv] = cf; }
    __syncthreads();
    int ws = 0, wf = 0, ts = 0, tfx = 0;
    for (int w = 0; w < 16; ++w) {
      if (w < wv) { ws += s_slot[w]; wf += s_fix[w]; }
      ts += s_slot[w]; tfx += s_fix[w];
    }
    const int slot0 = s_base[0] + ws + cs - (hf + tf);
    const int fix0 = s_base[1] + wf + cf - hf;
    if (t < nchunks) {
      head[t] = hf ? slot0 : -1;
      tail[t] = tf ? slot0 + hf : -1;
      fix_index[t] = hf ? fix0 : -1;
    }
    __syncthreads();
    if (tid == 0) { s_base[0] += ts; s_base[1] += tfx; }
    __syncthreads();
  }
  if (tid == 0) {
    header[0] = s_base[0];
    header[1] = s_base[1];
    header[2] = ipc;
    header[3] = (int32_t)(nchunks & 0x7fffffff);
  }
}

// Fix-up list entry i = (finishing chunk t, first partial slot of the row).
__global__ void plan_fix_kernel(const int32_t* __restrict__ rowptr, int64_t nchunks,
                                const Coord* __restrict__ coords, const int32_t* __restrict__ head,
                                const int32_t* __restrict__ tail, const int32_t* __restrict__ fix_index,
                                int32_t* __restrict__ fix) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nchunks || fix_index[t] < 0) return;
  const int32_t r = coords[t].x;
  const int64_t dr = (int64_t)r + rowptr[r];  // diagonal where row r starts
  // largest u <= t with diag(coords[u]) <= dr
  int64_t lo = 0, hi = t;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    const Coord c = coords[mid];
    if ((int64_t)c.x + c.y <= dr) lo = mid;
    else hi = mid - 1;
  }
  int32_t sb = head[t];
  for (int64_t w = lo; w < t; ++w) {
    if (tail[w] >= 0) { sb = tail[w]; break; }
  }
  const int32_t i = fix_index[t];
  fix[2 * i] = (int32_t)t;
  fix[2 * i + 1] = sb;
}

// ---------------------------------------------------------------------------
// Main SpMM kernel.
template <int LPR, int VPL, int VEC, int U>
__global__ void __launch_bounds__(256)
spmm_merge_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colind,
                  const float* __restrict__ val, int32_t M, const int32_t* __restrict__ plan,
                  int64_t nchunks, int32_t ipc, const float* __restrict__ B, int64_t ldb, int32_t F,
                  float* __restrict__ C, int64_t ldc, Epi epi, float* __restrict__ part,
                  int64_t part_ld) {
  using V = Vec<VEC>;
  using T = typename V::T;
  constexpr int G = 256 / LPR;
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];

  const PlanLayout L(nchunks);
  const Coord* __restrict__ coords = reinterpret_cast<const Coord*>(plan + L.coords);
  const int32_t* __restrict__ head_slot = plan + L.head;
  const int32_t* __restrict__ tail_slot = plan + L.tail;

  const int rows_cap = G * ipc + 2;
  const int nnz_cap = G * ipc + ipc;
  int32_t* s_rp = smem;
  int32_t* s_col = s_rp + rows_cap;
  float* s_val = reinterpret_cast<float*>(s_col + nnz_cap);
  int32_t* s_row = reinterpret_cast<int32_t*>(s_val + nnz_cap);

  const int tid = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * G;
  const int64_t tE = min<int64_t>(t0 + G, nchunks);
  const Coord c0 = coords[t0], c1 = coords[tE];
  const int32_t X0 = c0.x, Y0 = c0.y;
  const int nrows = min(c1.x + 1, M) - X0 + 1;
  const int nnzs = c1.y - Y0;

  // ---- stage the workgroup's slice of the CSR in LDS (coalesced)
  for (int i = tid; i < nrows; i += 256) s_rp[i] = rowptr[X0 + i];
  for (int i = tid; i < nnzs; i += 256) {
    s_col[i] = colind[Y0 + i];
    s_val[i] = val[Y0 + i];
  }
  __syncthreads();
  for (int i = tid; i < nnzs; i += 256) {
    const int32_t k = Y0 + i;
    int lo = 0, hi = nrows - 1;  // s_rp[lo] <= k < s_rp[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (s_rp[mid] <= k) lo = mid;
      else hi = mid;
    }
    s_row[i] = lo;
  }
  __syncthreads();

  // ---- one chunk per group of LPR lanes
  const int g = tid / LPR;
  const int lg = tid % LPR;
  const int64_t t = t0 + g;
  if (t >= nchunks) return;
  const Coord a = coords[t], b = coords[t + 1];
  const int32_t x0 = a.x, y0 = a.y, x1 = b.x, y1 = b.y;

  const int64_t col_base = (int64_t)blockIdx.y * (LPR * VPL * VEC);
  int64_t colv[VPL];
  bool colok[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    colv[v] = col_base + (int64_t)(v * LPR + lg) * VEC;
    colok[v] = colv[v] < F;
  }

  const bool head_partial = (x0 < x1) && (y0 > s_rp[x0 - X0]);
  const int32_t hslot = head_partial ? head_slot[t] : -1;

  T acc[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) acc[v] = V::zero();

  int32_t cur = x0;
  auto flush = [&](int32_t r) {
    if (r == x0 && head_partial) {
      float* dst = part + (int64_t)hslot * part_ld;
#pragma unroll
      for (int v = 0; v < VPL; ++v)
        if (colok[v]) V::store(dst + colv[v], acc[v]);
    } else {
      float* dst = C + (int64_t)r * ldc;
#pragma unroll
      for (int v = 0; v < VPL; ++v)
        if (colok[v]) V::store(dst + colv[v], V::epi(epi, acc[v], r, colv[v]));
    }
#pragma unroll
    for (int v = 0; v < VPL; ++v) acc[v] = V::zero();
  };

  for (int32_t base = y0; base < y1; base += U) {
    T gv[U][VPL];
    float vv[U];
    int32_t rr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int32_t k = base + u;
      const bool ok = k < y1;
      const int li = k - Y0;
      const int32_t c = ok ? s_col[li] : 0;
      vv[u] = ok ? s_val[li] : 0.f;
      rr[u] = ok ? s_row[li] + X0 : INT_MAX;
      const float* brow = B + (int64_t)c * ldb;
#pragma unroll
      for (int v = 0; v < VPL; ++v) gv[u][v] = (ok && colok[v]) ? V::load(brow + colv[v]) : V::zero();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (rr[u] != INT_MAX) {
        while (cur < rr[u]) {
          flush(cur);
          ++cur;
        }
#pragma unroll
        for (int v = 0; v < VPL; ++v) V::fma(acc[v], vv[u], gv[u][v]);
      }
    }
  }
  while (cur < x1) {
    flush(cur);
    ++cur;
  }
  if (x1 < M && y1 > max(y0, s_rp[x1 - X0])) {
    float* dst = part + (int64_t)tail_slot[t] * part_ld;
#pragma unroll
    for (int v = 0; v < VPL; ++v)
      if (colok[v]) V::store(dst + colv[v], acc[v]);
  }
}

// Sum the contiguous partial slots of every split row in slot (= chunk)
// order, apply the epilogue, store the row.
template <int LPR, int VPL, int VEC>
__global__ void __launch_bounds__(256)
spmm_fixup_kernel(const int32_t* __restrict__ plan, int64_t nchunks, int32_t nfix_host, int32_t F,
                  const float* __restrict__ part, int64_t part_ld, float* __restrict__ C,
                  int64_t ldc, Epi epi) {
  using V = Vec<VEC>;
  using T = typename V::T;
  constexpr int G = 256 / LPR;
  const PlanLayout L(nchunks);
  const Coord* __restrict__ coords = reinterpret_cast<const Coord*>(plan + L.coords);
  const int32_t* __restrict__ head_slot = plan + L.head;
  const int32_t* __restrict__ fix = plan + L.fix;
  const int32_t nfix = nfix_host >= 0 ? nfix_host : plan[1];
  const int64_t i = (int64_t)blockIdx.x * G + threadIdx.x / LPR;
  if (i >= nfix) return;
  const int lg = threadIdx.x % LPR;
  const int32_t t = fix[2 * i];
  const int32_t sb = fix[2 * i + 1];
  const int32_t se = head_slot[t];
  const int32_t r = coords[t].x;
  const int64_t col_base = (int64_t)blockIdx.y * (LPR * VPL * VEC);
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int64_t col = col_base + (int64_t)(v * LPR + lg) * VEC;
    if (col >= F) continue;
    T acc = V::zero();
    int32_t s = sb;
    for (; s + 3 <= se; s += 4) {
      const T p0 = V::load(part + (int64_t)(s + 0) * part_ld + col);
      const T p1 = V::load(part + (int64_t)(s + 1) * part_ld + col);
      const T p2 = V::load(part + (int64_t)(s + 2) * part_ld + col);
      const T p3 = V::load(part + (int64_t)(s + 3) * part_ld + col);
      V::add(acc, p0); V::add(acc, p1); V::add(acc, p2); V::add(acc, p3);
    }
    for (; s <= se; ++s) V::add(acc, V::load(part + (int64_t)s * part_ld + col));
    V::store(C + (int64_t)r * ldc + col, V::epi(epi, acc, r, col));
  }
}

// ---------------------------------------------------------------------------
// Dispatch

struct Cfg {
  int lpr, vpl, vec, col_tiles;
};

inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

inline Cfg choose_cfg(int32_t F, int vec, int lanes_hint) {
  Cfg c;
  c.vec = vec;
  const int W = (F + vec - 1) / vec;
  if (lanes_hint > 0) c.lpr = next_pow2(lanes_hint > 64 ? 64 : lanes_hint);
  else c.lpr = W <= 64 ? next_pow2(W) : 64;
  int vpl = (W + c.lpr - 1) / c.lpr;
  vpl = vpl <= 1 ? 1 : (vpl <= 2 ? 2 : 4);
  c.vpl = vpl;
  c.col_tiles = (W + c.lpr * c.vpl - 1) / (c.lpr * c.vpl);
  return c;
}

template <int LPR, int VPL, int VEC>
int launch_cfg(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
               const int32_t* plan, int64_t nchunks, int32_t ipc, int32_t nfix, const float* B,
               int64_t ldb, int32_t F, float* C, int64_t ldc, const Epi& epi, float* part,
               int64_t part_ld, int col_tiles, hipStream_t stream) {
  constexpr int G = 256 / LPR;
  constexpr int U = 8 / VPL;
  const int64_t nwg = (nchunks + G - 1) / G;
  const size_t lds = (size_t)((G * ipc + 2) + 3 * (G * ipc + ipc)) * 4;
  if (nwg > 0) {
    hipLaunchKernelGGL((spmm_merge_kernel<LPR, VPL, VEC, U>), dim3((unsigned)nwg, col_tiles), dim3(256),
                       lds, stream, rowptr, colind, val, M, plan, nchunks, ipc, B, ldb, F, C, ldc, epi,
                       part, part_ld);
    int rc = launch_check("spmm_merge_kernel");
    if (rc) return rc;
  }
  if (nfix != 0) {
    const int64_t nf = nfix > 0 ? nfix : nchunks;
    const int64_t nwf = (nf + G - 1) / G;
    hipLaunchKernelGGL((spmm_fixup_kernel<LPR, VPL, VEC>), dim3((unsigned)nwf, col_tiles), dim3(256), 0,
                       stream, plan, nchunks, nfix, F, part, part_ld, C, ldc, epi);
    return launch_check("spmm_fixup_kernel");
  }
  return GCNK_OK;
}

template <int VEC>
int dispatch_vec(const Cfg& c, const int32_t* rowptr, const int32_t* colind, const float* val,
                 int32_t M, const int32_t* plan, int64_t nchunks, int32_t ipc, int32_t nfix,
                 const float* B, int64_t ldb, int32_t F, float* C, int64_t ldc, const Epi& epi,
                 float* part, int64_t part_ld, hipStream_t s) {
#define GCNK_CASE(L, P)                                                                         \
  if (c.lpr == L && c.vpl == P)                                                                 \
    return launch_cfg<L, P, VEC>(rowptr, colind, val, M, plan, nchunks, ipc, nfix, B, ldb, F, C, \
                                 ldc, epi, part, part_ld, c.col_tiles, s);
  GCNK_CASE(1, 1) GCNK_CASE(2, 1) GCNK_CASE(4, 1) GCNK_CASE(8, 1) GCNK_CASE(16, 1) GCNK_CASE(32, 1)
  GCNK_CASE(64, 1) GCNK_CASE(16, 2) GCNK_CASE(16, 4) GCNK_CASE(32, 2) GCNK_CASE(32, 4)
  GCNK_CASE(64, 2) GCNK_CASE(64, 4)
#undef GCNK_CASE
  set_error("gcnk_spmm_csr_f32: unsupported lanes/vectors config (%d,%d)", c.lpr, c.vpl);
  return GCNK_EUNSUP;
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int32_t gcnk_spmm_default_ipc(int32_t M, int64_t nnz, int32_t F) {
  const int vec = (F % 4 == 0) ? 4 : 1;
  const Cfg c = choose_cfg(F, vec, 0);
  const int G = 256 / c.lpr;
  const int64_t items = (int64_t)M + nnz;
  int64_t ipc = items / ((int64_t)G * 1024);
  if (ipc < 4) ipc = 4;
  if (ipc > 64) ipc = 64;
  ipc = (ipc + 3) & ~3LL;
  while (G * ipc > 2048) ipc >>= 1;
  return (int32_t)ipc;
}

extern "C" int64_t gcnk_spmm_plan_chunks(int32_t M, int64_t nnz, int32_t ipc) {
  if (ipc <= 0 || M < 0 || nnz < 0) return -1;
  return plan_nchunks(M, nnz, ipc);
}

extern "C" int64_t gcnk_spmm_plan_bytes(int32_t M, int64_t nnz, int32_t ipc) {
  const int64_t nc = gcnk_spmm_plan_chunks(M, nnz, ipc);
  if (nc < 0) return -1;
  // + nchunks words of scratch for the fix index (kept after the fix list)
  return (PlanLayout(nc).total + nc) * 4;
}

extern "C" int gcnk_spmm_plan_build(const int32_t* rowptr, int32_t M, int64_t nnz, int32_t ipc,
                                    void* plan, int64_t plan_bytes, void* stream) {
  if (!rowptr || !plan || M < 0 || nnz < 0 || ipc <= 0 || ipc > 4096) {
    set_error("gcnk_spmm_plan_build: bad argument (M=%d nnz=%lld ipc=%d)", M, (long long)nnz, ipc);
    return GCNK_EARG;
  }
  if ((int64_t)M + nnz >= (int64_t)INT32_MAX) {
    set_error("gcnk_spmm_plan_build: M + nnz must be < 2^31");
    return GCNK_EUNSUP;
  }
  const int64_t need = gcnk_spmm_plan_bytes(M, nnz, ipc);
  if (plan_bytes < need) {
    set_error("gcnk_spmm_plan_build: plan buffer %lld B < %lld B", (long long)plan_bytes, (long long)need);
    return GCNK_EARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t nc = plan_nchunks(M, nnz, ipc);
  const PlanLayout L(nc);
  int32_t* p = (int32_t*)plan;
  Coord* coords = reinterpret_cast<Coord*>(p + L.coords);
  int32_t* fix_index = p + L.total;
  int rc;
  hipLaunchKernelGGL(plan_coords_kernel, dim3((unsigned)((nc + 1 + 255) / 256)), dim3(256), 0, s, rowptr, M,
                     nnz, ipc, nc, coords);
  if ((rc = launch_check("plan_coords_kernel"))) return rc;
  if (nc > 0) {
    hipLaunchKernelGGL(plan_flags_kernel, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, rowptr, M, nc,
                       coords, p + L.head, p + L.tail);
    if ((rc = launch_check("plan_flags_kernel"))) return rc;
  }
  hipLaunchKernelGGL(plan_scan_kernel, dim3(1), dim3(1024), 0, s, nc, ipc, p + L.head, p + L.tail, fix_index, p);
  if ((rc = launch_check("plan_scan_kernel"))) return rc;
  if (nc > 0) {
    hipLaunchKernelGGL(plan_fix_kernel, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, rowptr, nc, coords,
                       p + L.head, p + L.tail, fix_index, p + L.fix);
    if ((rc = launch_check("plan_fix_kernel"))) return rc;
  }
  return GCNK_OK;
}

extern "C" int gcnk_spmm_plan_query(const void* plan, int32_t* out4, void* stream) {
  if (!plan || !out4) {
    set_error("gcnk_spmm_plan_query: null pointer");
    return GCNK_EARG;
  }
  hipStream_t s = (hipStream_t)stream;
  int rc = hip_check(hipMemcpyAsync(out4, plan, 16, hipMemcpyDeviceToHost, s), "plan query copy");
  if (rc) return rc;
  return hip_check(hipStreamSynchronize(s), "plan query sync");
}

extern "C" int64_t gcnk_spmm_workspace_bytes(int32_t nslots, int32_t F) {
  const int64_t ld = ((int64_t)F + 3) & ~3LL;
  return (int64_t)(nslots > 0 ? nslots : 0) * ld * 4;
}

extern "C" int gcnk_spmm_csr_f32(const int32_t* rowptr, const int32_t* colind, const float* val,
                                 int32_t M, int32_t K, int64_t nnz, const void* plan, int32_t ipc,
                                 int32_t nfix, const float* B, int64_t ldb, int32_t F, float* C,
                                 int64_t ldc, const float* bias, int32_t epilogue,
                                 const uint8_t* drop_mask, int64_t ldm, float drop_scale,
                                 float keep_prob, uint64_t seed, uint64_t offset, float* workspace,
                                 int64_t workspace_bytes, int32_t lanes_hint, void* stream) {
  if (M < 0 || K < 0 || nnz < 0 || F < 0 || ipc <= 0 || !plan) {
    set_error("gcnk_spmm_csr_f32: bad argument (M=%d K=%d nnz=%lld F=%d ipc=%d)", M, K, (long long)nnz, F, ipc);
    return GCNK_EARG;
  }
  if (M == 0 || F == 0) return GCNK_OK;
  if (!rowptr || !C || (nnz > 0 && (!colind || !val || !B))) {
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
  const int64_t nc = plan_nchunks(M, nnz, ipc);
  const int64_t part_ld = ((int64_t)F + 3) & ~3LL;
  if (nfix != 0 && !workspace) {
    set_error("gcnk_spmm_csr_f32: plan has split rows but no workspace was given");
    return GCNK_EARG;
  }
  (void)workspace_bytes;
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
  const bool vec4 = (F % 4 == 0) && (ldb % 4 == 0) && (ldc % 4 == 0) && aligned16(B) && aligned16(C) &&
                    (!workspace || aligned16(workspace)) && (!bias || aligned16(bias));
  const Cfg c = choose_cfg(F, vec4 ? 4 : 1, lanes_hint);
  const int G = 256 / c.lpr;
  if ((int64_t)G * ipc > 2048) {
    set_error("gcnk_spmm_csr_f32: ipc %d too large for %d groups per workgroup", ipc, G);
    return GCNK_EUNSUP;
  }
  hipStream_t s = (hipStream_t)stream;
  const int32_t* p = (const int32_t*)plan;
  if (vec4)
    return dispatch_vec<4>(c, rowptr, colind, val, M, p, nc, ipc, nfix, B, ldb, F, C, ldc, e, workspace,
                           part_ld, s);
  return dispatch_vec<1>(c, rowptr, colind, val, M, p, nc, ipc, nfix, B, ldb, F, C, ldc, e, workspace,
                         part_ld, s);
}
