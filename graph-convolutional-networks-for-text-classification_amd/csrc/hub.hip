// Hub-split CSR SpMM for gfx950:  C = epi(A_csr * B)  for graphs with a few
// very heavy rows ("hubs") among many light ones -- the reference's doc-topic
// adjacency (layer.py:106 th.spmm(adj, support); R8: 50 topic rows of
// 191..1807 nonzeros beside 7,674 document rows of 2..14).
//
// Why a separate schedule.  Gathering row by row moves one B row per nonzero
// from L2 into the CUs: R8 A-hat at F = 200 gathers 69k x 800 B = 55 MB for a
// product whose compulsory traffic is 12.9 MB, and the per-CU L2->CU rate, not
// HBM, bounds the launch.  Two facts remove most of that volume:
//   * the light rows of one block reference few distinct B rows (after sorting
//     them by the hub columns they reference, a 30-row R8 block references its
//     own 30 rows and ~23 topic rows): each distinct B row is staged in LDS
//     ONCE per block and every nonzero reads it from LDS;
//   * a hub row h sums A[h, j] * B[j] over thousands of j, and B[j] is exactly
//     what the block owning light row j has just staged.  So the hub rows are
//     computed TRANSPOSED: block b adds up A[h, j] * B[j] over its own j for
//     every hub h it touches (one partial row per (block, hub) pair), and a
//     small second kernel sums each hub's partials in block order.  Each B row
//     is read once for its own row and all hub rows at the same time.
// Nonzeros of hub rows whose column no block owns (hub x hub entries, columns
// >= M) are gathered by the finishing kernel ("leftover" items).
//
// Two launches, no arrival counters, no atomics: the kernel boundary is the
// only hand-off (partials are plain stores), so concurrent calls on different
// streams with different workspaces never interact, and every sum has a fixed
// order (bitwise reproducible).
#include "gcnk_common.h"

#include <algorithm>
#include <climits>
#include <mutex>
#include <numeric>
#include <vector>

namespace gcnk {
namespace {

constexpr int kHubSmax = 64;            // B rows staged per block (F = 200: 51 KB of LDS)
#ifndef GCNK_HUB_BLOCK
#define GCNK_HUB_BLOCK 1024
#endif
constexpr int kHubBlock = GCNK_HUB_BLOCK;  // threads per light-block workgroup (16 waves)
constexpr int kHubRecMaxWords = 24576;  // record cap (96 KB of LDS)
constexpr int kHubTargetBlocks = 256;   // light blocks per launch: one per CU (256 CUs)
// finishing kernel: 1024 threads = 64 partial lanes x 16 column lanes at F >= 64,
// so a hub's ~100-250 partials are all in flight in one round of loads
constexpr int kHubFinishBlock = 1024;
constexpr int kLdsMax = 163840;         // gfx950: 160 KiB per workgroup

__host__ __device__ inline int64_t align4(int64_t x) { return (x + 3) & ~3LL; }

// ---------------------------------------------------------------------------
// Plan layout (int32 words):
//   header[16]:  0 magic 'GNH1'  1 M  2 K  3 groups  4 nblocks  5 R (record
//                stride, words)  6 nhub  7 npart (partial rows)  8 max staged
//                rows per block  9 nnz  10 nleft  11 light rows  12 rows per
//                block  13 hub degree threshold  14 stage slots  15 0
//   records[nblocks][R]: one per block of light rows (below)
//   hubs int4[nhub + 1]: {row, first partial, partial count, first leftover}
//                        (entry nhub: sentinel, .w = nleft)
//   left int2[nleft]:    {col, value bits} leftover nonzeros of the hub rows
// Record of block b (offsets in words; o_out = align4(4 + nstage),
// o_it = align4(o_out + 2 * nout)):
//   0 nstage  1 nlight  2 ngroups  3 nitems
//   4..      staged B row indices [nstage] (slot s holds B[scol[s]])
//   o_out..  outputs {dest, item end}[nout]: first the block's light rows
//            (dest = row of C), then one per hub it touches, hub order
//            (dest = -(partial row + 1))
//   o_it..   items {slot, value bits}[nitems]: an output's items run from the
//            previous output's end, padded to a multiple of 4 with {nstage, 0}
//            (slot nstage is a zero row); every item reads its B row from the
//            block's stage in LDS (blocks are cut so that all the rows they
//            reference fit: no LDS-or-global select in the inner loop, which
//            would turn the LDS reads into FLAT loads ordered behind the
//            block's global stores)
struct HubLayout {
  int64_t nblocks, R, nhub, npart, nleft, max_stage;
  int64_t recs, hubs, left, total;
  explicit HubLayout(const int32_t* h) {
    nblocks = h[4]; R = h[5]; nhub = h[6]; npart = h[7]; max_stage = h[8]; nleft = h[10];
    recs = 16;
    hubs = recs + nblocks * R;
    left = hubs + 4 * (nhub + 1);
    total = left + 2 * nleft;
  }
};

// ---------------------------------------------------------------------------
// Light blocks + hub partials.  Grid (nblocks, column tiles of LPR * VEC).
//  1. the block's record -> LDS (one coalesced pass);
//  2. its staged B rows (this column tile) -> LDS, all loads of a thread in
//     flight before the first LDS store;
//  3. lane group g (LPR lanes, one VEC-wide column vector each) takes outputs
//     g, g + SG, ...: sum of value * staged row over the output's items in
//     order; a light row gets the epilogue and goes to C, a hub partial goes
//     to the workspace.
template <int BLOCK, int LPR, int VEC>
__global__ void __launch_bounds__(BLOCK)
hub_light_kernel(const int32_t* __restrict__ recs, int32_t R, const float* __restrict__ B, int64_t ldb, int32_t F,
                 float* __restrict__ C, int64_t ldc, Epi epi, float* __restrict__ part, int64_t part_ld) {
  using V = Vec<VEC>;
  using T = typename V::T;
  constexpr int SG = BLOCK / LPR;  // lane groups per workgroup
  // staging loads per thread: kHubSmax rows + the zero row of a 64-vector tile
  constexpr int SU = ((kHubSmax + 1) * 64 + BLOCK - 1) / BLOCK;
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];
  int32_t* s_rec = smem;
  float* s_stage = reinterpret_cast<float*>(smem + R);
  const int tid = threadIdx.x;
  const int64_t c0 = (int64_t)blockIdx.y * (LPR * VEC);
  const int32_t Fw = (int32_t)min((int64_t)(LPR * VEC), (int64_t)F - c0);  // this tile's width

  stamp(epi, 0);
  const int4* rec = reinterpret_cast<const int4*>(recs + (int64_t)blockIdx.x * R);
  for (int i = tid; i < R / 4; i += BLOCK) reinterpret_cast<int4*>(s_rec)[i] = rec[i];
  __syncthreads();
  stamp(epi, 1);
  const int32_t nstage = s_rec[0], nlight = s_rec[1], ngroups = s_rec[2];
  const int32_t nout = nlight + ngroups;
  const int32_t o_out = (int32_t)align4(4 + nstage), o_it = (int32_t)align4(o_out + 2 * nout);

  // the bias is loaded here, ahead of the staging loads, so the waits that land
  // those also cover it: loaded later, its first use inside the output loop gets
  // an s_waitcnt vmcnt(0) in EVERY iteration, which also waits for all the
  // stores issued so far (measured: ~1 us per output row)
  const int lg = tid % LPR, g = tid / LPR;
  const int32_t lcol = lg * VEC;
  const int64_t colv = c0 + lcol;
  const bool colok = lcol < Fw;
  const T bv = (epi.bias && colok) ? V::load(epi.bias + colv) : V::zero();

  // ---- stage: row s of the tile at s_stage[s * SW] (SW = LPR * VEC floats, a
  //      power of two: an item's row address is one shift-add), element e =
  //      s * nq + q (VEC floats each); thread tid takes e = tid + j * BLOCK
  //      (slot / column stepped, no division per element), all of its loads in
  //      flight before the LDS stores.  Row nstage is all zeros: the padding
  //      items of the plan point at it.
  constexpr int SW = LPR * VEC;
  constexpr int SWL = __builtin_ctz(SW);
  const int32_t nq = (Fw + VEC - 1) / VEC;
  {
    const int32_t ds = BLOCK / nq, dq = BLOCK - ds * nq;
    int32_t s0 = tid / nq, q0 = tid - s0 * nq;
    T v[SU];
#pragma unroll
    for (int j = 0; j < SU; ++j) {
      v[j] = V::zero();
#if defined(GCNK_HUB_EXP) && GCNK_HUB_EXP >= 8  // ablation: no staging loads
      (void)ldb;
#else
      if (s0 < nstage) v[j] = V::load(B + (int64_t)s_rec[4 + s0] * ldb + c0 + (int64_t)q0 * VEC);
#endif
      s0 += ds;
      q0 += dq;
      if (q0 >= nq) {
        q0 -= nq;
        ++s0;
      }
    }
    s0 = tid / nq;
    q0 = tid - s0 * nq;
#pragma unroll
    for (int j = 0; j < SU; ++j) {
      if (s0 <= nstage) V::store(s_stage + (s0 << SWL) + q0 * VEC, v[j]);  // s0 == nstage: the zero row
      s0 += ds;
      q0 += dq;
      if (q0 >= nq) {
        q0 -= nq;
        ++s0;
      }
    }
  }
  __syncthreads();
  stamp(epi, 2);

  // ---- outputs.  Lane group g (a whole wavefront at LPR = 64, which takes a
  //      contiguous range of outputs) walks its outputs' items in groups of 4
  //      (the plan pads every output to a multiple of 4 with {zero row, 0}):
  //      two 16-B reads bring 4 {slot, value} items (the same address for the
  //      whole group: a broadcast), four row reads, eight packed FMAs -- no
  //      guards, no selects, no per-item scalar work.  Idle lanes (columns past
  //      the tile) read inside their row, keeping the read conflict-free.
  const int4* s_items4 = reinterpret_cast<const int4*>(s_rec + o_it);
  const bool fast_epi = VEC == 4 && epi.code <= GCNK_EPI_BIAS_RELU;
  if constexpr (LPR == 64 && VEC == 4) {
    // Two outputs per wavefront: half-wave group h (32 lanes) owns a contiguous
    // range of outputs; lane hl holds columns 4 hl and 128 + 4 hl of the tile,
    // so each of its two row reads is contiguous across the half (conflict-free)
    // and every instruction of the walk and the epilogue serves two outputs.
    constexpr int HG = BLOCK / 32;
    const int hl = tid & 31, h = tid >> 5;
    const int32_t ca = 4 * hl, cb = 128 + 4 * hl;
    const bool oka = ca < Fw, okb = cb < Fw;
    const float4 ba = (epi.bias && oka) ? *reinterpret_cast<const float4*>(epi.bias + c0 + ca) : V::zero();
    const float4 bb = (epi.bias && okb) ? *reinterpret_cast<const float4*>(epi.bias + c0 + cb) : V::zero();
    const int32_t og0 = (int32_t)((int64_t)nout * h / HG), og1 = (int32_t)((int64_t)nout * (h + 1) / HG);
    const float* sa = s_stage + ca;
    const float* sb = s_stage + cb;
    int32_t ib = og0 == 0 ? 0 : s_rec[o_out + 2 * og0 - 1];
    for (int32_t o = og0; o < og1; ++o) {
      const int32_t dest = s_rec[o_out + 2 * o], ie = s_rec[o_out + 2 * o + 1];
      float4 xa = V::zero(), xb = V::zero();
      for (int32_t k = ib; k < ie; k += 4) {
        const int4 p0 = s_items4[k >> 1], p1 = s_items4[(k >> 1) + 1];  // items k .. k + 3
        const int32_t r0 = p0.x << 8, r1 = p0.z << 8, r2 = p1.x << 8, r3 = p1.z << 8;
        const float4 a0 = V::load(sa + r0), a1 = V::load(sa + r1), a2 = V::load(sa + r2), a3 = V::load(sa + r3);
        const float4 b0 = V::load(sb + r0), b1 = V::load(sb + r1), b2 = V::load(sb + r2), b3 = V::load(sb + r3);
        V::fma(xa, __int_as_float(p0.y), a0);
        V::fma(xb, __int_as_float(p0.y), b0);
        V::fma(xa, __int_as_float(p0.w), a1);
        V::fma(xb, __int_as_float(p0.w), b1);
        V::fma(xa, __int_as_float(p1.y), a2);
        V::fma(xb, __int_as_float(p1.y), b2);
        V::fma(xa, __int_as_float(p1.w), a3);
        V::fma(xb, __int_as_float(p1.w), b3);
      }
      ib = ie;
#ifdef GCNK_HUB_EXP
      if (((GCNK_HUB_EXP & 1) && dest < 0) || ((GCNK_HUB_EXP & 2) && dest >= 0)) {
        if (xa.x == 1234.5f) V::store(C, xb);  // keeps the sums live
        continue;
      }
#endif
      if (dest >= 0) {
        if (fast_epi) {
          if (epi.code != GCNK_EPI_NONE) {
            V::add(xa, ba);
            V::add(xb, bb);
            if (epi.code == GCNK_EPI_BIAS_RELU) {
              xa.x = fmaxf(xa.x, 0.f); xa.y = fmaxf(xa.y, 0.f); xa.z = fmaxf(xa.z, 0.f); xa.w = fmaxf(xa.w, 0.f);
              xb.x = fmaxf(xb.x, 0.f); xb.y = fmaxf(xb.y, 0.f); xb.z = fmaxf(xb.z, 0.f); xb.w = fmaxf(xb.w, 0.f);
            }
          }
        } else {
          xa = V::epi(epi, xa, ba, dest, c0 + ca);
          xb = V::epi(epi, xb, bb, dest, c0 + cb);
        }
      }
      float* dst = dest >= 0 ? C + (int64_t)dest * ldc + c0 : part + (int64_t)(-dest - 1) * part_ld + c0;
      if (oka) V::store_aligned(dst + ca, xa);
      if (okb) V::store_aligned(dst + cb, xb);
    }
#ifdef GCNK_STAMPS
    __syncthreads();
    stamp(epi, 3);
#endif
    return;
  }
  constexpr int NW = BLOCK / 64;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (the compiler cannot tell)
  const int32_t ow0 = LPR == 64 ? (int32_t)((int64_t)nout * w / NW) : g;
  const int32_t ow1 = LPR == 64 ? (int32_t)((int64_t)nout * (w + 1) / NW) : nout;
  const float* srow = s_stage + lcol;
  int32_t ib = ow0 == 0 ? 0 : s_rec[o_out + 2 * ow0 - 1];
  if (LPR == 64) ib = __builtin_amdgcn_readfirstlane(ib);
  for (int32_t o = ow0; o < ow1; o += (LPR == 64 ? 1 : SG)) {
    int32_t dest = s_rec[o_out + 2 * o], ie = s_rec[o_out + 2 * o + 1];
    if (LPR == 64) {
      dest = __builtin_amdgcn_readfirstlane(dest);
      ie = __builtin_amdgcn_readfirstlane(ie);
    } else {
      ib = o == 0 ? 0 : s_rec[o_out + 2 * o - 1];
    }
    T acc = V::zero();
#if defined(GCNK_HUB_EXP) && (GCNK_HUB_EXP & 16)  // ablation: no item loop
    ib = ie;
#endif
    for (int32_t k = ib; k < ie; k += 4) {
      const int4 p0 = s_items4[k >> 1], p1 = s_items4[(k >> 1) + 1];  // items k .. k + 3
      const T g0 = V::load(srow + (p0.x << SWL)), g1 = V::load(srow + (p0.z << SWL));
      const T g2 = V::load(srow + (p1.x << SWL)), g3 = V::load(srow + (p1.z << SWL));
      V::fma(acc, __int_as_float(p0.y), g0);
      V::fma(acc, __int_as_float(p0.w), g1);
      V::fma(acc, __int_as_float(p1.y), g2);
      V::fma(acc, __int_as_float(p1.w), g3);
    }
    ib = ie;
    if (!colok) continue;
#ifdef GCNK_HUB_EXP  // ablation builds (scripts/hub_probe.py): 1 no partial stores, 2 no C stores, 4 neither
    if (((GCNK_HUB_EXP & 1) && dest < 0) || ((GCNK_HUB_EXP & 2) && dest >= 0)) {
      if (reinterpret_cast<const float*>(&acc)[0] == 1234.5f) V::store(C, acc);  // keeps the sum live
      continue;
    }
#endif
    // value and destination first, then ONE store (separate store sites get sunk
    // into a common one that the backend splits into dword + dwordx3)
    T val = acc;
    if (dest >= 0) {
      if (fast_epi) {
        float* a = reinterpret_cast<float*>(&val);
        const float* bb = reinterpret_cast<const float*>(&bv);
        if (epi.code != GCNK_EPI_NONE)
#pragma unroll
          for (int i = 0; i < VEC; ++i) {
            a[i] += bb[i];
            if (epi.code == GCNK_EPI_BIAS_RELU) a[i] = a[i] > 0.f ? a[i] : 0.f;
          }
      } else {
        val = V::epi(epi, acc, bv, dest, colv);
      }
    }
    float* dst = dest >= 0 ? C + (int64_t)dest * ldc + colv : part + (int64_t)(-dest - 1) * part_ld + colv;
    V::store_aligned(dst, val);
  }
#ifdef GCNK_STAMPS
  __syncthreads();
  stamp(epi, 3);
#endif
}

// Hub rows: C[row] = epi(sum of the hub's partials in block order + its leftover
// nonzeros).  Grid (nhub, column tiles of LPR * VEC); BLOCK threads = PL partial
// lanes x LPR column lanes; partial lane p takes partials p, p + PL, ... and
// leftovers p, p + PL, ... (U loads in flight), then a fixed-order LDS tree.
template <int BLOCK, int LPR, int VEC>
__global__ void __launch_bounds__(BLOCK)
hub_finish_kernel(const int4* __restrict__ hubs, const int2* __restrict__ left, const float* __restrict__ part,
                  int64_t part_ld, const float* __restrict__ B, int64_t ldb, int32_t F, float* __restrict__ C,
                  int64_t ldc, Epi epi) {
  using V = Vec<VEC>;
  using T = typename V::T;
  constexpr int PL = BLOCK / LPR;
  constexpr int U = 8;
  __shared__ T s_red[PL][LPR];
  stamp(epi, 0);
  const int4 hb = hubs[blockIdx.x];
  const int32_t le = hubs[blockIdx.x + 1].w;
  const int tid = threadIdx.x, pl = tid / LPR, lg = tid % LPR;
  const int64_t colv = (int64_t)blockIdx.y * (LPR * VEC) + (int64_t)lg * VEC;
  const bool ok = colv < F;
  const T bv = (epi.bias && ok) ? V::load(epi.bias + colv) : V::zero();  // first: no wait behind the partials
  T acc = V::zero();
  // indices clamped into range and out-of-range terms dropped by a select, so
  // each batch's U loads issue back to back (no load under a branch)
  const int64_t cv = ok ? colv : 0;
  const float* p0 = part + (int64_t)hb.y * part_ld + cv;
  for (int32_t s0 = pl; s0 < hb.z; s0 += PL * U) {
    T pv[U];
#pragma unroll
    for (int j = 0; j < U; ++j) pv[j] = V::load(p0 + (int64_t)min(s0 + PL * j, hb.z - 1) * part_ld);
#pragma unroll
    for (int j = 0; j < U; ++j) {
      T t = acc;
      V::add(t, pv[j]);
      if (s0 + PL * j < hb.z) acc = t;
    }
  }
  for (int32_t k0 = hb.w + pl; k0 < le; k0 += PL * U) {
    int2 it[U];
#pragma unroll
    for (int j = 0; j < U; ++j) it[j] = left[min(k0 + PL * j, le - 1)];
    T gv[U];
#pragma unroll
    for (int j = 0; j < U; ++j) gv[j] = V::load(B + (int64_t)it[j].x * ldb + cv);
#pragma unroll
    for (int j = 0; j < U; ++j) {
      T t = acc;
      V::fma(t, __int_as_float(it[j].y), gv[j]);
      if (k0 + PL * j < le) acc = t;
    }
  }
  s_red[pl][lg] = acc;
  __syncthreads();
  stamp(epi, 1);
#pragma unroll
  for (int w = PL / 2; w >= 1; w >>= 1) {
    if (pl < w) V::add(s_red[pl][lg], s_red[pl + w][lg]);
    __syncthreads();
  }
  if (pl == 0 && ok) {
    V::store(C + (int64_t)hb.x * ldc + colv, V::epi(epi, s_red[0][lg], bv, hb.x, colv));
  }
  stamp(epi, 2);
}

struct HubArgs {
  const int32_t* plan;
  HubLayout L;
  const float* B;
  int64_t ldb;
  int32_t F;
  float* C;
  int64_t ldc;
  Epi epi;
  float* part;
  int64_t part_ld;
  hipStream_t s;
};

template <int LPR, int VEC>
int hub_launch(const HubArgs& a) {
  const int64_t tile = (int64_t)LPR * VEC;
  const int64_t ntiles = (a.F + tile - 1) / tile;
  const int64_t TW = std::min<int64_t>(a.F, tile);
  // staged rows at a stride of one tile (LPR * VEC floats) + the zero row
  (void)TW;
  const int64_t lds = a.L.R * 4 + (a.L.max_stage + 1) * tile * 4;
  if (lds > kLdsMax || ntiles > 65535) {
    set_error("gcnk_spmm (hub plan): %lld B of LDS / %lld column tiles exceed the launch limits", (long long)lds,
              (long long)ntiles);
    return GCNK_EUNSUP;
  }
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hub_light_kernel<kHubBlock, LPR, VEC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax);
  });
  if (a.L.nblocks > 0) {
    hipLaunchKernelGGL((hub_light_kernel<kHubBlock, LPR, VEC>), dim3((unsigned)a.L.nblocks, (unsigned)ntiles),
                       dim3(kHubBlock), (size_t)lds, a.s, a.plan + a.L.recs, (int32_t)a.L.R, a.B, a.ldb, a.F, a.C,
                       a.ldc, a.epi, a.part, a.part_ld);
    const int rc = launch_check("hub_light_kernel");
    if (rc) return rc;
  }
  constexpr int LB = LPR < 16 ? LPR : 16;
  const int64_t tb = (a.F + LB * VEC - 1) / (LB * VEC);
  Epi eb = a.epi;  // debug stamps of the finishing kernel follow the light kernel's
  if (eb.stamps) eb.stamps += 4 * a.L.nblocks * ntiles;
  hipLaunchKernelGGL((hub_finish_kernel<kHubFinishBlock, LB, VEC>), dim3((unsigned)a.L.nhub, (unsigned)tb),
                     dim3(kHubFinishBlock), 0, a.s,
                     reinterpret_cast<const int4*>(a.plan + a.L.hubs), reinterpret_cast<const int2*>(a.plan + a.L.left),
                     a.part, a.part_ld, a.B, a.ldb, a.F, a.C, a.ldc, eb);
  return launch_check("hub_finish_kernel");
}

template <int VEC>
int hub_dispatch(int lpr, const HubArgs& a) {
  switch (lpr) {
    case 1: return hub_launch<1, VEC>(a);
    case 2: return hub_launch<2, VEC>(a);
    case 4: return hub_launch<4, VEC>(a);
    case 8: return hub_launch<8, VEC>(a);
    case 16: return hub_launch<16, VEC>(a);
    case 32: return hub_launch<32, VEC>(a);
    case 64: return hub_launch<64, VEC>(a);
  }
  set_error("gcnk_spmm (hub plan): unsupported lanes per group %d", lpr);
  return GCNK_EUNSUP;
}

}  // namespace

// ---------------------------------------------------------------------------
// Host plan.  Returns GCNK_OK with `img` filled, 1 when the operand has no hub
// structure worth the schedule (auto mode; the caller builds the row plan), or
// a negative error code.
int hub_plan_host(const int32_t* rp, const int32_t* ci, const float* vv, int32_t M, int32_t K, int64_t nnz,
                  int32_t groups, int32_t hub_min, int32_t block_rows, std::vector<int32_t>& img) {
  if (M <= 0 || nnz <= 0 || hub_min < 0) return 1;
  const bool auto_mode = hub_min == 0;
  // automatic: wide operands only (whole-wavefront groups, F > 128); at narrow
  // widths the row plan's gathers are cheap (R8 F = 8: 32-B rows) and measured faster
  if (auto_mode && groups != 1) return 1;
  // hub threshold: 8x the mean degree, at least 64 nonzeros (R8 A-hat: mean 9,
  // threshold 72: the 50 topic rows, 191..1807 nonzeros; uniform 1M/20M: mean
  // 20, threshold 160, max degree ~45: no hubs)
  const int64_t hmin = auto_mode ? std::max<int64_t>(64, 8 * ((nnz + M - 1) / M)) : hub_min;
  std::vector<int32_t> hubs, light;
  int64_t hub_nnz = 0;
  for (int32_t r = 0; r < M; ++r) {
    const int64_t d = (int64_t)rp[r + 1] - rp[r];
    if (d >= hmin) {
      hubs.push_back(r);
      hub_nnz += d;
    } else {
      light.push_back(r);
    }
  }
  const int64_t nhub = (int64_t)hubs.size(), nlight = (int64_t)light.size();
  if (nhub == 0 || nlight == 0 || nhub >= (1 << 24)) return 1;
  if (auto_mode && hub_nnz * 4 < nnz) return 1;  // hubs hold under a quarter of the nonzeros

  // light rows sorted by the hub columns they reference (columns referenced by
  // >= hmin light rows), so the rows of a block share their staged B rows
  std::vector<int32_t> colref((size_t)K, 0);
  for (int32_t r : light)
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k) ++colref[(size_t)ci[k]];
  std::vector<int64_t> so((size_t)nlight + 1, 0);
  std::vector<int32_t> sc;
  for (int64_t i = 0; i < nlight; ++i) {
    const int32_t r = light[(size_t)i];
    const size_t b = sc.size();
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k)
      if (colref[(size_t)ci[k]] >= hmin) sc.push_back(ci[k]);
    std::sort(sc.begin() + (int64_t)b, sc.end());
    so[(size_t)i + 1] = (int64_t)sc.size();
  }
  std::vector<int32_t> ord((size_t)nlight);
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(), [&](int32_t x, int32_t y) {
    return std::lexicographical_compare(sc.begin() + so[(size_t)x], sc.begin() + so[(size_t)x + 1],
                                        sc.begin() + so[(size_t)y], sc.begin() + so[(size_t)y + 1]);
  });
  std::vector<char> hubref((size_t)K, 0);
  for (int32_t r : hubs)
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k) hubref[(size_t)ci[k]] = 1;
  std::vector<int64_t> bstart;
  std::vector<int32_t> mark((size_t)K, -1), rowmark((size_t)K, -1);
  int64_t stamp_base = 0;
  // greedy cut at <= br rows; false when a single row alone overflows the stage
  auto partition = [&](int64_t br) {
    bstart.clear();
    std::fill(mark.begin(), mark.end(), -1);
    int64_t rows = 0, stage = 0;
    int32_t blk = -1;
    auto fresh = [&](int32_t r) {  // distinct columns row r adds to block blk
      const int32_t id = (int32_t)(stamp_base++ & 0x3fffffff);
      int64_t n = 0;
      auto see = [&](int32_t c) {
        if (rowmark[(size_t)c] != id && mark[(size_t)c] != blk) ++n;
        rowmark[(size_t)c] = id;
      };
      for (int64_t k = rp[r]; k < rp[r + 1]; ++k) see(ci[k]);
      if (r < K && hubref[(size_t)r]) see(r);
      return n;
    };
    for (int64_t i = 0; i < nlight; ++i) {
      const int32_t r = light[(size_t)ord[(size_t)i]];
      int64_t n = blk >= 0 ? fresh(r) : 0;
      if (blk < 0 || rows == br || stage + n > kHubSmax) {
        ++blk;
        bstart.push_back(i);
        rows = stage = 0;
        n = fresh(r);
        if (n > kHubSmax) {
          set_error("gcnk_spmm_plan (hub): light row %d references %lld rows, more than the %d stage slots", r,
                    (long long)n, kHubSmax);
          return false;
        }
      }
      for (int64_t k = rp[r]; k < rp[r + 1]; ++k) mark[(size_t)ci[k]] = blk;
      if (r < K && hubref[(size_t)r]) mark[(size_t)r] = blk;
      stage += n;
      ++rows;
    }
    bstart.push_back(nlight);
    return true;
  };
  // blocks of consecutive sorted rows, cut early where the B rows a block
  // references (its rows' columns + its own columns that hub rows reference)
  // would exceed the kHubSmax stage slots.  Automatic size: the smallest
  // row cap (>= 4) whose blocks number at most kHubTargetBlocks, so every
  // block is resident at once (one per CU)
  int64_t br = block_rows > 0 ? block_rows : std::max<int64_t>(4, (nlight + kHubTargetBlocks - 1) / kHubTargetBlocks);
  for (;;) {
    if (!partition(br)) return auto_mode ? 1 : GCNK_EUNSUP;
    if (block_rows > 0 || (int64_t)bstart.size() - 1 <= kHubTargetBlocks || br >= 64) break;
    ++br;
  }
  const int64_t nblocks = (int64_t)bstart.size() - 1;
  std::vector<int32_t> owner((size_t)K, -1);  // column j -> block of light row j
  for (int64_t b = 0; b < nblocks; ++b)
    for (int64_t i = bstart[(size_t)b]; i < bstart[(size_t)b + 1]; ++i) {
      const int32_t r = light[(size_t)ord[(size_t)i]];
      if (r < K) owner[(size_t)r] = (int32_t)b;
    }

  // hub nonzeros: owned column -> that block's group for the hub, else leftover
  struct Group {
    int32_t h;
    int64_t b, e;  // entries [b, e) of the block's entry list
  };
  std::vector<std::vector<Group>> bg((size_t)nblocks);
  std::vector<std::vector<int32_t>> ecol((size_t)nblocks);
  std::vector<std::vector<float>> eval((size_t)nblocks);
  std::vector<int32_t> lcol;
  std::vector<float> lval;
  std::vector<int64_t> left_off((size_t)nhub + 1, 0);
  int64_t owned = 0;
  for (int64_t h = 0; h < nhub; ++h) {
    const int32_t r = hubs[(size_t)h];
    left_off[(size_t)h] = (int64_t)lcol.size();
    for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
      const int32_t j = ci[k];
      const float v = vv ? vv[k] : 0.f;
      const int32_t b = owner[(size_t)j];
      if (b < 0) {
        lcol.push_back(j);
        lval.push_back(v);
        continue;
      }
      ++owned;
      std::vector<Group>& gs = bg[(size_t)b];
      if (gs.empty() || gs.back().h != (int32_t)h) gs.push_back({(int32_t)h, (int64_t)ecol[(size_t)b].size(), (int64_t)ecol[(size_t)b].size()});
      ecol[(size_t)b].push_back(j);
      eval[(size_t)b].push_back(v);
      ++gs.back().e;
    }
  }
  left_off[(size_t)nhub] = (int64_t)lcol.size();
  if (auto_mode && owned * 2 < hub_nnz) return 1;  // hubs mostly over unowned columns: nothing to share

  // partial rows: hub h's partials are contiguous, in block order
  std::vector<int64_t> part_off((size_t)nhub + 1, 0), seen((size_t)nhub, 0);
  for (const auto& gs : bg)
    for (const Group& g : gs) ++part_off[(size_t)g.h + 1];
  for (int64_t h = 0; h < nhub; ++h) part_off[(size_t)h + 1] += part_off[(size_t)h];
  const int64_t npart = part_off[(size_t)nhub];
  if (npart >= INT32_MAX || (int64_t)lcol.size() >= INT32_MAX) return GCNK_EUNSUP;

  // records
  std::vector<std::vector<int32_t>> recs((size_t)nblocks);
  std::vector<int32_t> cnt((size_t)K, 0), slot((size_t)K, -1), touched, staged;
  int64_t R = 4, max_stage = 0;
  for (int64_t b = 0; b < nblocks; ++b) {
    const int64_t i0 = bstart[(size_t)b], i1 = bstart[(size_t)b + 1];
    touched.clear();
    auto touch = [&](int32_t c) {
      if (cnt[(size_t)c]++ == 0) touched.push_back(c);
    };
    int64_t nit = 0;
    for (int64_t i = i0; i < i1; ++i) {
      const int32_t r = light[(size_t)ord[(size_t)i]];
      for (int64_t k = rp[r]; k < rp[r + 1]; ++k) touch(ci[k]);
      nit += (int64_t)rp[r + 1] - rp[r];
    }
    for (int32_t c : ecol[(size_t)b]) touch(c);
    nit += (int64_t)ecol[(size_t)b].size();
    // stage every referenced column (the partition guarantees <= kHubSmax), in column order
    staged = touched;
    if ((int64_t)staged.size() > kHubSmax) {
      set_error("gcnk_spmm_plan (hub): block %lld stages %zu rows", (long long)b, staged.size());
      return GCNK_EUNSUP;
    }
    std::sort(staged.begin(), staged.end());
    for (size_t s = 0; s < staged.size(); ++s) slot[(size_t)staged[s]] = (int32_t)s;
    const int64_t nstage = (int64_t)staged.size(), nl = i1 - i0, ng = (int64_t)bg[(size_t)b].size();
    const int64_t o_out = align4(4 + nstage), o_it = align4(o_out + 2 * (nl + ng));
    nit += 3 * (nl + ng);  // room for the padding of every output to a multiple of 4 items
    std::vector<int32_t>& w = recs[(size_t)b];
    w.assign((size_t)(o_it + 2 * nit), 0);
    w[0] = (int32_t)nstage;
    w[1] = (int32_t)nl;
    w[2] = (int32_t)ng;
    std::copy(staged.begin(), staged.end(), w.begin() + 4);
    int64_t it = 0, o = 0;
    auto item = [&](int32_t c, float v) {
      w[(size_t)(o_it + 2 * it)] = slot[(size_t)c];
      w[(size_t)(o_it + 2 * it + 1)] = __builtin_bit_cast(int32_t, v);
      ++it;
    };
    // every output's items padded to a multiple of 4 with {zero row (slot nstage), 0}
    auto pad = [&]() {
      while (it % 4) {
        w[(size_t)(o_it + 2 * it)] = (int32_t)nstage;
        w[(size_t)(o_it + 2 * it + 1)] = 0;
        ++it;
      }
    };
    for (int64_t i = i0; i < i1; ++i, ++o) {
      const int32_t r = light[(size_t)ord[(size_t)i]];
      for (int64_t k = rp[r]; k < rp[r + 1]; ++k) item(ci[k], vv ? vv[k] : 0.f);
      pad();
      w[(size_t)(o_out + 2 * o)] = r;
      w[(size_t)(o_out + 2 * o + 1)] = (int32_t)it;
    }
    for (const Group& g : bg[(size_t)b]) {
      for (int64_t e = g.b; e < g.e; ++e) item(ecol[(size_t)b][(size_t)e], eval[(size_t)b][(size_t)e]);
      pad();
      const int64_t p = part_off[(size_t)g.h] + seen[(size_t)g.h]++;
      w[(size_t)(o_out + 2 * o)] = (int32_t)(-p - 1);
      w[(size_t)(o_out + 2 * o + 1)] = (int32_t)it;
      ++o;
    }
    w[3] = (int32_t)it;
    w.resize((size_t)(o_it + 2 * it));
    for (int32_t c : touched) {
      cnt[(size_t)c] = 0;
      slot[(size_t)c] = -1;
    }
    R = std::max<int64_t>(R, align4((int64_t)w.size()));
    max_stage = std::max(max_stage, nstage);
  }
  if (R > kHubRecMaxWords) {
    if (auto_mode) return 1;
    set_error("gcnk_spmm_plan (hub): a block record of %lld words exceeds %d", (long long)R, kHubRecMaxWords);
    return GCNK_EUNSUP;
  }
  const int64_t nleft = (int64_t)lcol.size();
  const int64_t words = 16 + nblocks * R + 4 * (nhub + 1) + 2 * nleft;
  if (words >= INT32_MAX) return GCNK_EUNSUP;
  img.assign((size_t)words, 0);
  const int32_t hdr[16] = {kHubMagic, M, K, groups, (int32_t)nblocks, (int32_t)R, (int32_t)nhub, (int32_t)npart,
                           (int32_t)max_stage, (int32_t)nnz, (int32_t)nleft, (int32_t)nlight, (int32_t)br,
                           (int32_t)hmin, kHubSmax, 0};
  std::copy(hdr, hdr + 16, img.begin());
  for (int64_t b = 0; b < nblocks; ++b)
    std::copy(recs[(size_t)b].begin(), recs[(size_t)b].end(), img.begin() + 16 + b * R);
  const HubLayout L(img.data());
  for (int64_t h = 0; h <= nhub; ++h) {
    int32_t* e = img.data() + L.hubs + 4 * h;
    if (h < nhub) {
      e[0] = hubs[(size_t)h];
      e[1] = (int32_t)part_off[(size_t)h];
      e[2] = (int32_t)(part_off[(size_t)h + 1] - part_off[(size_t)h]);
      e[3] = (int32_t)left_off[(size_t)h];
    } else {
      e[0] = -1;
      e[1] = (int32_t)npart;
      e[2] = 0;
      e[3] = (int32_t)nleft;
    }
  }
  for (int64_t k = 0; k < nleft; ++k) {
    img[(size_t)(L.left + 2 * k)] = lcol[(size_t)k];
    img[(size_t)(L.left + 2 * k + 1)] = __builtin_bit_cast(int32_t, lval[(size_t)k]);
  }
  return GCNK_OK;
}

int64_t hub_plan_words(const int32_t* hdr) { return HubLayout(hdr).total; }

int64_t hub_workspace_bytes(const int32_t* hdr, int32_t F) {
  const int64_t ld = ((int64_t)F + 3) & ~3LL;
  return (((int64_t)hdr[7] * ld * 4) + 255) & ~255LL;
}

int hub_spmm(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F, float* C, int64_t ldc,
             const Epi& e, float* workspace, int lpr, bool vec4, hipStream_t s) {
  const HubLayout L(hdr);
  if (L.nhub <= 0) {
    set_error("gcnk_spmm (hub plan): empty hub table");
    return GCNK_EARG;
  }
  const int64_t part_ld = ((int64_t)F + 3) & ~3LL;
  HubArgs a{(const int32_t*)plan, L, B, ldb, F, C, ldc, e, workspace, part_ld, s};
  if (vec4) return hub_dispatch<4>(lpr, a);
  return hub_dispatch<1>(lpr, a);
}

}  // namespace gcnk
