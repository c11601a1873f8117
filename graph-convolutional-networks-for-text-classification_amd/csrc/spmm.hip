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
//  * the remaining rows -> spmm_row_kernel (gathers), one launch.  The plan
//    lists "units": a light row (at most `ipc` nonzeros) is one unit owned by
//    one lane group (LPR lanes, each lane one VEC-wide column vector of the
//    row: one load instruction of a group covers LPR*VEC contiguous floats of
//    a B row); a heavier row is cut into segments, each owned by a whole
//    wavefront whose 64/LPR lane groups take interleaved nonzeros and meet in
//    a fixed xor butterfly.  A row of one segment is stored directly; a row
//    of several leaves one partial per segment, and the last segment to
//    finish (arrival counter in the plan) sums them in segment order and
//    stores the row -- no fix-up launch.  With whole-wavefront groups (F >
//    128) a wavefront takes two light rows at once (their items in one vector
//    load, their gathers in one batch stream).  Every lane issues the U gathers of
//    a batch before its first FMA (U independent 16-B loads in flight), and a
//    unit's one store follows all of its loads, so no gather waits behind a
//    store.  Heavy segments come first in the grid (the longest work is
//    dispatched first); light rows follow in row order.  bias/ReLU/dropout
//    (and optionally a dense projection) are fused into the store.
//
// Every sum has a fixed order (no float atomics): results are bitwise
// reproducible run to run.
#include "gcnk_common.h"

#include <algorithm>
#include <climits>
#include <type_traits>
#include <vector>

namespace gcnk {
namespace {

constexpr int32_t kMagic = 0x474e4b35;  // "GNK5"
constexpr int kRB = 64;                 // tile rows per dense block (4 waves x 16)
constexpr int kKC = 64;                 // condensed columns per tile chunk (16 MFMA k-steps)
#ifndef GCNK_TILE_MAXNT
#define GCNK_TILE_MAXNT 4
#endif
// 16-column MFMA n-tiles per tile workgroup.  4 (R8 F = 200: 4 slices, 484
// workgroups for X_hubs W1): tile 6.8 us against 7.3 with 8 and 7.5 with 1, the
// forward 0.5-1 us shorter, factored or not (profiles/r03_tile_nt.log)
constexpr int kMaxNT = GCNK_TILE_MAXNT;
constexpr int kMaxColTiles = 64;        // row-kernel column tiles per launch (arrival counters per heavy row)
constexpr int kMaxSeg = 64;             // slots per heavy entry (bounds a last arriver's combine)
constexpr int kMaxSegRow = kMaxSeg * kMaxSeg;  // segments per heavy row (two combine levels)
// Schedule knobs of the whole-wavefront (F > 128) row kernel, overridable at
// compile time for experiments (scripts/variants.sh times prebuilt variants).
// Measured on R8 A-hat F = 200 / 20ng-shaped (profiles/r01_variants.log):
// 2 light rows per wavefront 10.6 / 18.2-19.0 us vs 1: 10.4 / 18.8 (the launch
// then fits one residency round); 4 rows: 13.9 / 25.4; heavy U = 16: 11.5 (120
// VGPRs, 4 waves/SIMD); 512-thread workgroups (8 waves per heavy segment): 10.7.
// Write-through (sc1) output stores: the launch leaves no dirty output lines
// in the XCD L2s for the kernel boundary to write back (R8 X W1: tile kernel
// 13.2 -> 11.4 us in the forward, forward 36.4 -> 34.7 us).  2: nontemporal
// stores instead (experiment).
#ifndef GCNK_TILE_SC1
#define GCNK_TILE_SC1 1
#endif
// Tile kernel: LDS writes / MFMA k-steps in this many phases (tile_body)
#ifndef GCNK_TILE_PHASES
#define GCNK_TILE_PHASES 2
#endif
// Nontemporal (streaming) output stores of the row kernel's finished rows: the
// launch leaves no dirty output lines in the XCD L2s for the end-of-kernel
// write-back.  R8 A-hat S1, F = 200, cold (HIP events per call,
// profiles/r04_probe_nt.log): 9.46 -> 8.16 us, document rows alone 8.16 ->
// 6.95, topic rows alone 9.05 -> 7.78 (a cold 12.4 MB copy: 4.35 -> 3.25 us,
// scripts/micro/ns_micro.hip).  Write-through (sc1) stores measured 9.06 us
// there (removed).
#ifndef GCNK_ROW_NT
#define GCNK_ROW_NT 1
#endif
// Light rows per wavefront (whole-wavefront groups).  Round 4, with the
// nontemporal stores and the gather-wait fix, cold R8 A-hat F = 200
// (profiles/r04_sweep2_*.log): one row per wavefront takes the document rows
// alone from 6.95 to 5.27 us and the launch from 8.30 to 8.14 (the topic rows,
// 7.76 alone, now bound it); two rows had measured even in round 1.
#ifndef GCNK_LIGHT_RPW
#define GCNK_LIGHT_RPW 1
#endif
// Gathers in flight per lane in a heavy segment.  With one light row per
// wavefront the kernel holds 6 under its 64-VGPR cap (8 spills 16 B/lane, 12
// spills 148): a 12-item segment is two batches of 6 instead of three of 4.
// Cold R8 A-hat F = 200 (scripts/r04_step19.sh, four runs each, the last in
// profiles/r04_sweep3_*.log): 8.10-8.15 -> 7.90-7.97 us; R8 F = 8
// unchanged (5.47-5.50), the 20ng-shaped graph at F = 200 12.6 -> 12.8
// (profiles/r04_hu_*.log).
#ifndef GCNK_HEAVY_U
#define GCNK_HEAVY_U 6
#endif
#ifndef GCNK_WAVE_BLOCK
#define GCNK_WAVE_BLOCK 256
#endif
constexpr int kHeavyU = GCNK_HEAVY_U;        // gathers in flight per lane in a heavy segment
#ifndef GCNK_ROW_U
#define GCNK_ROW_U 8
#endif
constexpr int kRowU = GCNK_ROW_U;            // gathers in flight per lane for light rows
#ifndef GCNK_NARROW_WG
#define GCNK_NARROW_WG 1
#endif
// Lane groups of 8-32 lanes (256-thread workgroups): a heavy segment spans the
// whole 4-wavefront workgroup (4x the nonzeros per segment, 4x fewer partials)
// instead of one wavefront.  R8 A-hat at F = 64: 7.30 -> 6.69 us, F = 32 even.
// Round 1-4 kept 1-4 lanes on one-wave workgroups (256-thread ones measured
// 5.64 -> 6.14 us at F = 8); with round 5's padded heavy items the 256-thread
// ones win from 2 lanes on (kNarrowMin below: F = 8 5.41 -> 4.73 us).
constexpr bool kNarrowWG = GCNK_NARROW_WG != 0;
// smallest group width (lanes) that takes 256-thread workgroups with
// workgroup-wide heavy segments (experiment knob; narrower groups run one-wave
// workgroups)
#ifndef GCNK_NARROW_MIN_LPR
#define GCNK_NARROW_MIN_LPR 2
#endif
constexpr int kNarrowMin = GCNK_NARROW_MIN_LPR;
// Heavy segments of whole-wavefront plans keep a padded copy of their items
// (segment u's at u * segp, col -1 past its end), so a heavy workgroup loads
// its items at an address it knows from its index, in flight with its unit
// word -- no unit -> items dependency before the gathers.
#ifndef GCNK_HEAVY_DIRECT
#define GCNK_HEAVY_DIRECT 1
#endif
constexpr int kWaveBlock = GCNK_WAVE_BLOCK;  // workgroup size for whole-wavefront groups
constexpr int kLightRPW = GCNK_LIGHT_RPW;    // light rows per wavefront with whole-wavefront groups
constexpr int kLightMax64 = 64 / kLightRPW;  // their nonzero limit (kLightRPW rows' items fill one 64-lane load)

// ---------------------------------------------------------------------------
// Plan layout (int32 words).  Header (16 words, see gcnk.h):
//   0 magic  1 M  2 K  3 lane groups per wavefront (64 / LPR)  4 ipc (light-row limit)
//   5 nunits  6 nhunits (heavy region, padded)  7 nheavy (rows of > 1 segment)
//   8 ntile (chunks)  9 nred  10 nslabs  11 ntblk (tile blocks)  12 has_diag | segp << 1 | tops << 30  13 nnz
//   14 nslots (partial slots)  15 nsingle (chunk items of single-chunk blocks, listed first)
// Body: items int2[nnz] {col, value bits} in CSR order | units int4[nunits]
//   {row (-1: empty), nz begin, nz end, heavy entry * 64 + slot or -1}: the
//   heavy region first, then light rows, each laid out so that the units of
//   workgroup b belong to XCD class b % 8 (below) | heavy int4[nheavy]
//   {row, first partial slot, slots, -1 (a row of <= kMaxSeg segments), or for
//   a row of more (bit 30 of header word 12 set): one entry per group of <=
//   kMaxSeg segments with .w = the top entry's slot for the group's sum, and
//   the top entry, .w = -2} | tile part (descriptors,
//   condensed columns, A fragments, reduce rows int4[64 * nred] {row (-1:
//   none), first slab, slabs, diagonal value bits}, row lists, extracted
//   diagonal float[64 * ntblk] in block order) | (segp > 0) the heavy units'
//   items, padded: int2[nhunits][segp], col -1 past a unit's end.
struct Layout {
  int64_t M, nnz, nunits, nhunits, nheavy, nslots, ntile, nred, ntblk, has_diag, segp, tops;
  int64_t items, units, heavy, tdesc, tcols, tfrag, red, trows, dval, hitems, total;
  __host__ __device__ explicit Layout(const int32_t* h) {
    M = h[1]; nunits = h[5]; nhunits = h[6]; nheavy = h[7]; ntile = h[8]; nred = h[9]; ntblk = h[11];
    has_diag = h[12] & 1; segp = ((uint32_t)h[12] >> 1) & ((1u << 29) - 1); tops = ((uint32_t)h[12] >> 30) & 1;
    nnz = h[13]; nslots = h[14];
    items = 16;
    units = (items + 2 * nnz + 3) & ~3LL;
    heavy = units + 4 * nunits;
    tdesc = (heavy + 4 * nheavy + 3) & ~3LL;
    tcols = tdesc + 4 * ntile;
    tfrag = (tcols + (int64_t)kKC * ntile + 3) & ~3LL;
    red = tfrag + (int64_t)kRB * kKC * ntile;
    trows = red + 4 * nred * kRB;
    dval = trows + (int64_t)kRB * ntblk;
    hitems = (dval + (has_diag ? (int64_t)kRB * ntblk : 0) + 3) & ~3LL;
    total = hitems + 2 * nhunits * segp;   // padded heavy items int2[nhunits][segp]
  }
};

// Coherent (sc1) raw-buffer accesses from a wave-uniform base (see RowPlan).
typedef float f32v4 __attribute__((ext_vector_type(4)));
constexpr int kBufSc1 = 16;               // cache-policy aux bit sc1 (gfx94x/gfx950)
constexpr int kBufDword3 = 0x00020000;    // raw buffer resource word 3 (gfx9)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const float* base_uniform) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base_uniform), (short)0, 0x7fffffff, kBufDword3);
}
__device__ __forceinline__ void store_coherent_v(const float* base_uniform, int64_t off, const float4& v) {
  const f32v4 x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, row_rsrc(base_uniform), (int)(off * 4), 0, kBufSc1);
}
__device__ __forceinline__ void store_coherent_v(const float* base_uniform, int64_t off, const float& v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), row_rsrc(base_uniform), (int)(off * 4), 0, kBufSc1);
}
template <typename T>
__device__ __forceinline__ T load_coherent_v(const float* base_uniform, int64_t off);
template <>
__device__ __forceinline__ float4 load_coherent_v<float4>(const float* base_uniform, int64_t off) {
  const f32v4 x = __builtin_amdgcn_raw_buffer_load_b128(row_rsrc(base_uniform), (int)(off * 4), 0, kBufSc1);
  return make_float4(x.x, x.y, x.z, x.w);
}
template <>
__device__ __forceinline__ float load_coherent_v<float>(const float* base_uniform, int64_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(row_rsrc(base_uniform), (int)(off * 4), 0, kBufSc1));
}
__device__ __forceinline__ const float* uniform_ptr(const float* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return reinterpret_cast<const float*>(((uint64_t)hi << 32) | lo);
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

// v from lane ^ OFF, by the cheapest exchange for the offset: DPP quad
// permutes (VALU rate) for 1 and 2, ds_swizzle's xor mode (no address VGPR)
// inside 32 lanes, ds_bpermute across the halves.
template <int OFF>
__device__ __forceinline__ float xor_lane(float v) {
  if constexpr (OFF == 1)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
  else if constexpr (OFF == 2)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  else if constexpr (OFF < 32)
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), (OFF << 10) | 0x1F));
  else
    return __shfl_xor(v, OFF, 64);
}

template <int NP, int LPR, int VPL, int VEC>
struct Proj {
  static constexpr int kMaxF = LPR * VPL * VEC;  // one column tile holds the whole row
  // W [F x P] is staged in LDS once per workgroup with coalesced loads and read
  // back per finished row (a lane's own W rows straight from global memory
  // would make every wave-instruction touch 64 cache lines; held in registers
  // they cost 32 VGPRs for the whole kernel -- 99 VGPRs, 4 waves per SIMD).
  __device__ __forceinline__ static float* lds() {
    __shared__ __attribute__((aligned(16))) float s_w[NP > 0 ? kMaxF * NP : 1];
    return s_w;
  }
  int64_t colv;
  bool colok;
  __device__ __forceinline__ void init(const int64_t* colv_, const bool* colok_) {
    colv = *colv_;
    colok = *colok_;
  }
  // W into LDS in two halves, so its loads can be in flight with others:
  // fetch() loads this thread's share (coalesced) into registers, put() writes
  // it to LDS; visible to the workgroup after sync().
  template <int NTHR>
  static constexpr int per_thread() { return NP > 0 ? (kMaxF * NP + NTHR - 1) / NTHR : 1; }
  template <int NTHR>
  __device__ __forceinline__ void fetch(const ProjArgs& pa, int32_t F, float* wv) const {
    if constexpr (NP > 0) {
#pragma unroll
      for (int j = 0; j < per_thread<NTHR>(); ++j) {
        const int e = (int)threadIdx.x + j * NTHR;
        const int r = e / NP, c = e % NP;
        wv[j] = (e < kMaxF * NP && r < F && c < pa.P) ? pa.W[(int64_t)r * pa.ldw + c] : 0.f;
      }
    }
  }
  template <int NTHR>
  __device__ __forceinline__ void put(const float* wv) const {
    if constexpr (NP > 0) {
      float* s_w = lds();
#pragma unroll
      for (int j = 0; j < per_thread<NTHR>(); ++j) {
        const int e = (int)threadIdx.x + j * NTHR;
        if (e < kMaxF * NP) s_w[e] = wv[j];
      }
    }
  }
  template <int NTHR>
  __device__ __forceinline__ void stage(const ProjArgs& pa, int32_t F) {
    float wv[per_thread<NTHR>()];
    fetch<NTHR>(pa, F, wv);
    put<NTHR>(wv);
    sync();
  }
  __device__ __forceinline__ void sync() {
    if constexpr (NP > 0) __syncthreads();
  }
  // W [F x NP] dense and 16-B aligned (the common case: P == NP): the whole
  // workgroup copies it straight into LDS with global_load_lds (no VGPRs, no
  // wait until sync(), which drains it), 1 KiB per wave-instruction.
  __device__ __forceinline__ static bool dma_ok(const ProjArgs& pa) {
    return NP > 0 && pa.P == NP && pa.ldw == NP && ((uintptr_t)pa.W & 15) == 0;
  }
  template <int NTHR>
  __device__ __forceinline__ void issue_dma(const ProjArgs& pa, int32_t F) const {
    if constexpr (NP > 0) {
      float* s_w = lds();
      const int32_t n = F * NP;                   // floats to copy (<= kMaxF * NP)
      const int w = (int)threadIdx.x >> 6, l = (int)threadIdx.x & 63;
#pragma unroll
      for (int j = 0; j < (kMaxF * NP + NTHR * 4 - 1) / (NTHR * 4); ++j) {
        const int32_t b = (j * (NTHR / 64) + w) * 256;  // this wave's 1 KiB piece (uniform)
        if (b < n) {
          // lanes past the end re-read the first float4 (they land in rows >= F, never read)
          const int32_t src = b + 4 * l < n ? b + 4 * l : 0;
          __builtin_amdgcn_global_load_lds(pa.W + src, (__attribute__((address_space(3))) void*)(s_w + b), 16, 0, 0);
        }
      }
    }
  }
  template <int NTHR>
  __device__ __forceinline__ void begin(const ProjArgs& pa, int32_t F) const {
    if (dma_ok(pa)) issue_dma<NTHR>(pa, F);
  }
  template <int NTHR>
  __device__ __forceinline__ void finish_stage(const ProjArgs& pa, int32_t F) {
    if (dma_ok(pa)) sync();
    else stage<NTHR>(pa, F);
  }
  template <typename T>
  __device__ __forceinline__ void apply(const ProjArgs& pa, const T* h, int64_t row, int lg) const {
    if constexpr (NP > 0) {
      static_assert(NP % 4 == 0, "W rows are read as float4");
      const float* s_w = lds();
      float s[NP];
#pragma unroll
      for (int c = 0; c < NP; ++c) s[c] = 0.f;
      // lanes past F hold h = 0 and read W row 0 (any finite row would do)
      const int64_t c0 = colok ? colv : 0;
#pragma unroll
      for (int v = 0; v < VPL; ++v) {
        const float* hv = reinterpret_cast<const float*>(&h[v]);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float4* wr = reinterpret_cast<const float4*>(s_w + (c0 + v * LPR * VEC + i) * NP);
#pragma unroll
          for (int c4 = 0; c4 < NP / 4; ++c4) {
            const float4 w4 = wr[c4];
            s[4 * c4 + 0] = fmaf(hv[i], w4.x, s[4 * c4 + 0]);
            s[4 * c4 + 1] = fmaf(hv[i], w4.y, s[4 * c4 + 1]);
            s[4 * c4 + 2] = fmaf(hv[i], w4.z, s[4 * c4 + 2]);
            s[4 * c4 + 3] = fmaf(hv[i], w4.w, s[4 * c4 + 3]);
          }
        }
      }
      // transpose-reduce: while channels remain to split, each xor step sends the
      // half of the channels the partner keeps (n/2 exchanges instead of n), so a
      // lane ends with NP/2^H channels summed over 2^H lanes; plain xor steps
      // finish.  Offsets ascend, so the costly cross-half exchange (32) comes
      // last, on the fewest channels.
      int chan = 0;
      reduce_split<NP, 1>(s, lg, chan);
      constexpr int H = ilog2(NP) < ilog2(LPR) ? ilog2(NP) : ilog2(LPR);
      constexpr int NR = NP >> H;          // channels left per lane
      tail_sum<NR, (1 << H)>(s);
      if ((lg >> H) == 0) {
#pragma unroll
        for (int c = 0; c < NR; ++c)
          if (chan + c < pa.P) {
            pa.C2[row * pa.ldc2 + chan + c] = s[c];
          }
      }
    }
  }

  static constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x >> 1); }

  // plain xor steps OFF, 2 OFF, ..., LPR/2 over the NR channels left per lane
  template <int NR, int OFF>
  __device__ __forceinline__ static void tail_sum(float* s) {
    if constexpr (OFF < LPR) {
#pragma unroll
      for (int c = 0; c < NR; ++c) s[c] += xor_lane<OFF>(s[c]);
      tail_sum<NR, OFF * 2>(s);
    }
  }

  // One halving step per recursion level, offsets 1, 2, 4, ... while n > 1.
  template <int N, int OFF>
  __device__ __forceinline__ static void reduce_split(float* s, int lg, int& chan) {
    if constexpr (N > 1 && OFF < LPR) {
      constexpr int Hn = N / 2;
      const bool up = (lg & OFF) != 0;
#pragma unroll
      for (int c = 0; c < Hn; ++c) {
        const float keep = up ? s[c + Hn] : s[c];
        const float send = up ? s[c] : s[c + Hn];
        s[c] = keep + xor_lane<OFF>(send);
      }
      if (up) chan += Hn;
      reduce_split<Hn, OFF * 2>(s, lg, chan);
    }
  }
};

// ---------------------------------------------------------------------------
// Row kernel (gathers).
struct RowPlan {
  const int2* items;   // {col, value bits} per nonzero, CSR order
  const int4* units;   // {row (-1: empty), nz begin, nz end, heavy row * 64 + segment or -1}
  const int4* heavy;   // {row, first partial slot, slots, parent * 64 + group or -1}
  int32_t* cnt;        // per heavy row x column tile: arrival counters, in the caller's
                       // counter region (zero on entry, re-armed by each row's last arriver)
  int32_t nunits, nhunits;
  const int2* hitems;  // heavy units' items, padded to segp each (null: none)
  int32_t segp;
};

// Partial slots are written and read with agent-coherent accesses (the sc1
// cache-policy bit, what relaxed agent-scope atomics get, past the per-XCD L2),
// so publishing them needs no L2 write-back/invalidate: the writing wave waits
// for its stores to complete (s_waitcnt vmcnt(0)) before bumping the arrival
// counter, and the last arriver is told so by the value its own add returns.
// This is the hand-off MI355X_MICROARCH.md lists under "Valid forms" (every
// store and load of the handed-off bytes sc1, each storing wave drained before
// ONE lane of its workgroup adds to an agent-scope counter, the last adder
// reading only after its add returned) in place of an agent release/acquire
// pair, which would cost a full L2 write-back (~1.7 us) per segment.  The
// counters live in a per-call region of the caller (gcnk.h): concurrent calls
// with distinct regions never share them.
// Whole-wavefront groups use raw-buffer instructions (a wave-uniform row base,
// per-lane byte offsets below 2^31, checked on the host): one 16-B access per
// lane where per-dword atomics take four (R8 A-hat F = 200: 10.6 -> 9.4 us).
// Narrow groups keep the per-dword atomics (measured faster there: R8 F = 8
// 5.2 us vs 6.1 with buffer accesses).
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

// B[c, col..] (VEC floats).  O32: through a 32-bit byte offset from the
// uniform base -- one scalar multiply and one vector add per row piece, the
// load taking the SGPR base -- where the 64-bit index costs ~7 scalar
// instructions per gathered row (the CU's one scalar unit was the row kernel's
// limiter: ~8k SALU per CU per R8 launch).  Needs K * ldb * 4 + F * 4 < 2^32
// (checked at launch).  col4 = the lane's column offset in bytes.
template <int VEC, bool O32>
__device__ __forceinline__ typename Vec<VEC>::T load_row(const float* __restrict__ B, int64_t ldb, uint32_t ldb4,
                                                       int32_t c, int64_t colv, uint32_t col4) {
  if constexpr (O32)
    return Vec<VEC>::load(
        reinterpret_cast<const float*>(reinterpret_cast<const char*>(B) + ((uint32_t)c * ldb4 + col4)));
  else
    return Vec<VEC>::load(B + (int64_t)c * ldb + colv);
}

// acc += sum of val * B[col, colv..] over items k = b + q + S*i, i ascending,
// U gathers in flight per batch (all issued before the first FMA).
template <int VEC, int U, int S, bool O32>
__device__ __forceinline__ void gather_rows(const int2* __restrict__ items, int32_t b, int32_t e, int q,
                                            const float* __restrict__ B, int64_t ldb, int64_t colv, bool colok,
                                            typename Vec<VEC>::T& acc) {
  const uint32_t ldb4 = (uint32_t)ldb * 4u, col4 = colok ? (uint32_t)colv * 4u : 0u;
  using V = Vec<VEC>;
  using T = typename V::T;
  for (int32_t k0 = b + q; k0 < e; k0 += S * U) {
    int2 it[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int32_t k = k0 + S * j;
      it[j] = k < e ? items[k] : make_int2(-1, 0);
    }
    T g[U];
#pragma unroll
    for (int j = 0; j < U; ++j)
      g[j] = it[j].x >= 0 ? load_row<VEC, O32>(B, ldb, ldb4, it[j].x, colok ? colv : 0, col4) : V::zero();
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (it[j].x >= 0) V::fma(acc, __int_as_float(it[j].y), g[j]);
  }
}

// Whole-wavefront groups (LPR == 64; b, e, q wave-uniform): the same sum, but
// the items come in with ONE vector load per 64 of them (lane l holds item
// b + q + S*l) and are broadcast with v_readlane, so a batch of U gathers
// waits for one latency instead of an item load and then the gathers (a heavy
// segment's 4 batches: 5 latencies instead of 8).
template <int VEC, int U, int S, bool O32>
__device__ __forceinline__ void gather_rows_wave(const int2* __restrict__ items, int32_t b, int32_t e, int q,
                                                 const float* __restrict__ B, int64_t ldb, int64_t colv, bool colok,
                                                 typename Vec<VEC>::T& acc) {
  using V = Vec<VEC>;
  using T = typename V::T;
  const int lane = threadIdx.x & 63;
  const uint32_t ldb4 = (uint32_t)ldb * 4u, col4 = colok ? (uint32_t)colv * 4u : 0u;
  const int64_t colc = colok ? colv : 0;  // idle lanes read inside the row (no branch around the load)
  for (int32_t base = b + q; base < e; base += 64 * S) {
    const int32_t k = base + S * lane;
    const int2 mine = k < e ? items[k] : make_int2(-1, 0);
    // wait for the item words HERE, with the builtin the wait-count pass sees:
    // otherwise it cannot prove on the paths that skip a conditional gather
    // below that `mine` has landed, and puts a vmcnt(0) in front of EVERY
    // readlane -- which also waits for the gathers already issued, so the
    // batch of U gathers ran one at a time (ISA of round 3's kernel)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
    const int32_t cnt = min(64, (e - base + S - 1) / S);  // wave-uniform
    for (int32_t j0 = 0; j0 < cnt; j0 += U) {
      T g[U];
      float a[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        g[j] = V::zero();
        a[j] = 0.f;
        if (j0 + j < cnt) {
          const int32_t c = __builtin_amdgcn_readlane(mine.x, j0 + j);
          a[j] = __int_as_float(__builtin_amdgcn_readlane(mine.y, j0 + j));
          g[j] = load_row<VEC, O32>(B, ldb, ldb4, c, colc, col4);
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (j0 + j < cnt) V::fma(acc, a[j], g[j]);
    }
  }
}

// gather_rows_wave over a heavy unit's padded item copy (its items at
// hi[0 .. segp), col -1 past the end): the item load's address is known from
// the unit index alone, so it flies with the unit word's load.
template <int VEC, int U, int S, bool O32>
__device__ __forceinline__ void gather_rows_wave_direct(const int2* __restrict__ hi, int32_t segp, int q,
                                                        const float* __restrict__ B, int64_t ldb, int64_t colv,
                                                        bool colok, typename Vec<VEC>::T& acc) {
  using V = Vec<VEC>;
  using T = typename V::T;
  const int lane = threadIdx.x & 63;
  const uint32_t ldb4 = (uint32_t)ldb * 4u, col4 = colok ? (uint32_t)colv * 4u : 0u;
  const int64_t colc = colok ? colv : 0;
  for (int32_t base = q; base < segp; base += 64 * S) {
    const int32_t k = base + S * lane;
    const int2 mine = k < segp ? hi[k] : make_int2(-1, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the item words (and the unit word) have landed
    // the segment's items are packed at the front: the valid lanes are a prefix
    const int32_t cnt = __builtin_popcountll(__ballot(mine.x >= 0));  // wave-uniform
    for (int32_t j0 = 0; j0 < cnt; j0 += U) {
      T g[U];
      float a[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        g[j] = V::zero();
        a[j] = 0.f;
        if (j0 + j < cnt) {
          const int32_t c = __builtin_amdgcn_readlane(mine.x, j0 + j);
          a[j] = __int_as_float(__builtin_amdgcn_readlane(mine.y, j0 + j));
          g[j] = load_row<VEC, O32>(B, ldb, ldb4, c, colc, col4);
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (j0 + j < cnt) V::fma(acc, a[j], g[j]);
    }
    if (cnt < 64) break;
  }
}

// Sum over the 64/LPR lane groups of a wave (xor butterfly: every lane ends
// with bitwise the same sum, since each level adds the same two operands).
template <int LPR, typename T>
__device__ __forceinline__ void wave_group_sum(T& acc) {
  if constexpr (LPR < 64) {
    float* f = reinterpret_cast<float*>(&acc);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) f[i] += xor_lane<LPR>(f[i]);
    wave_group_sum<LPR * 2>(acc);
  }
}

__device__ __forceinline__ void store_nt(float* p, const float4& v) {
  typedef float f4a __attribute__((ext_vector_type(4), aligned(16)));
  __builtin_nontemporal_store(f4a{v.x, v.y, v.z, v.w}, reinterpret_cast<f4a*>(p));
}
__device__ __forceinline__ void store_nt(float* p, const float& v) { __builtin_nontemporal_store(v, p); }

// Epilogue + store (+ fused projection) of one finished row by lane group
// q == 0 of the calling lanes.
template <int LPR, int VEC, int NP>
__device__ __forceinline__ void finish_row(const typename Vec<VEC>::T& acc, int32_t r, int64_t colv, bool colok,
                                           const typename Vec<VEC>::T& bv, int lg, float* __restrict__ C,
                                           int64_t ldc, const Epi& epi, bool store_main,
                                           const Proj<NP, LPR, 1, VEC>& proj, const ProjArgs& pa) {
  using V = Vec<VEC>;
  using T = typename V::T;
  const T h = colok ? V::epi(epi, acc, bv, r, colv) : V::zero();
#if GCNK_ROW_NT
  if (colok && store_main) store_nt(C + (int64_t)r * ldc + colv, h);
#else
  if (colok && store_main) V::store(C + (int64_t)r * ldc + colv, h);
#endif
  proj.apply(pa, &h, r, lg);
}

// grid.x: [0, nhb) heavy blocks, one heavy segment per wavefront (per
// workgroup for 64-lane groups); then light blocks, one light row per lane
// group.  grid.y: column tiles of LPR*VEC.
#ifndef GCNK_ROW_WPE
#define GCNK_ROW_WPE 8
#endif
// Whole-wave groups at 8 waves per SIMD (<= 64 VGPRs, no spills there; the
// narrower groups would spill): R8's 1832 workgroups then fit one residency
// round (at 66 VGPRs, 7 per SIMD, 40 of them waited for a second round)
template <int BLOCK, int LPR, int VEC, int U, int NP, bool O32>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(LPR == 64 && NP <= 8 ? GCNK_ROW_WPE : 1)))
spmm_row_kernel(RowPlan rp, int32_t nhb, const float* __restrict__ B, int64_t ldb, int32_t F,
                float* __restrict__ C, int64_t ldc, Epi epi, float* __restrict__ part, int64_t part_ld,
                ProjArgs pa) {
  resolve_rng(epi);
  using V = Vec<VEC>;
  using T = typename V::T;
  constexpr int SG = BLOCK / LPR;  // lane groups per workgroup
  constexpr int SW = 64 / LPR;     // lane groups per wavefront
  constexpr int WPB = BLOCK / 64;  // wavefronts per workgroup
  const int tid = threadIdx.x;
  const int lg = tid % LPR;
  const int64_t colv = (int64_t)blockIdx.y * (LPR * VEC) + (int64_t)lg * VEC;
  const bool colok = colv < F;
  stamp(epi, 0);
  T bv = (epi.bias && colok) ? V::load(epi.bias + colv) : V::zero();
  Proj<NP, LPR, 1, VEC> proj;
  proj.init(&colv, &colok);
  // W for the fused projection: narrow groups stage it up front; whole-wavefront
  // groups only where a row is finished, after the gathers (a heavy segment's
  // workgroup only if it finishes the row: most store a partial and leave; the
  // last arriver's W loads fly with its partial loads)
  if constexpr (LPR < 64) proj.template stage<BLOCK>(pa, F);
  else if ((int32_t)blockIdx.x >= nhb) proj.template begin<BLOCK>(pa, F);
  const bool store_main = NP == 0 || pa.store_main;
  T acc = V::zero();

  if ((int32_t)blockIdx.x >= nhb) {
    if constexpr (LPR == 64) {
      // ---- light rows, whole-wavefront groups: kLightRPW units per wavefront,
      //      their items in one vector load (row r's after rows < r's), their
      //      gathers in one stream of U-wide batches (light rows are at most
      //      kLightMax64 nonzeros each, so kLightRPW of them fill 64 lanes): the
      //      light part of the grid is kLightRPW times fewer wavefronts and the
      //      whole launch fits one residency round.
      constexpr int R = kLightRPW;
      const int32_t u0 = __builtin_amdgcn_readfirstlane(rp.nhunits + ((int32_t)blockIdx.x - nhb) * SG * R +
                                                        (tid / 64) * R);
      // (with a projection every wavefront reaches its barrier: past the end all
      // R units are empty and nothing is gathered or stored)
      if (NP == 0 && u0 >= rp.nunits) return;
      int4 un[R];
      int32_t nb[R + 1];  // item prefix offsets of the R rows (wave-uniform)
      nb[0] = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        un[r] = u0 + r < rp.nunits ? rp.units[u0 + r] : make_int4(-1, 0, 0, -1);
        nb[r + 1] = nb[r] + (un[r].x >= 0 ? un[r].z - un[r].y : 0);
      }
      stamp(epi, 1);
      const int lane = tid & 63;
      int32_t k = -1;
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (lane >= nb[r] && lane < nb[r + 1]) k = un[r].y + lane - nb[r];
      const int2 mine = k >= 0 ? rp.items[k] : make_int2(-1, 0);
      const uint32_t ldb4 = (uint32_t)ldb * 4u, col4 = colok ? (uint32_t)colv * 4u : 0u;
      const int64_t colc = colok ? colv : 0;  // idle lanes read inside the row (no branch around the load)
      T accs[R];
#pragma unroll
      for (int r = 0; r < R; ++r) accs[r] = V::zero();
      const int32_t cnt = nb[R];
      for (int32_t j0 = 0; j0 < cnt; j0 += U) {
        T g[U];
        float a[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
          g[j] = V::zero();
          a[j] = 0.f;
          if (j0 + j < cnt) {
            const int32_t c = __builtin_amdgcn_readlane(mine.x, j0 + j);
            a[j] = __int_as_float(__builtin_amdgcn_readlane(mine.y, j0 + j));
            g[j] = load_row<VEC, O32>(B, ldb, ldb4, c, colc, col4);
          }
        }
#pragma unroll
        for (int j = 0; j < U; ++j)
#pragma unroll
          for (int r = 0; r < R; ++r)
            if (j0 + j >= nb[r] && j0 + j < nb[r + 1]) V::fma(accs[r], a[j], g[j]);
      }
      stamp(epi, 2);
      proj.template finish_stage<BLOCK>(pa, F);
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (un[r].x >= 0)
          finish_row<LPR, VEC, NP>(accs[r], un[r].x, colv, colok, bv, lg, C, ldc, epi, store_main, proj, pa);
      stamp(epi, 3);
      return;
    }
    // ---- light rows: one unit per lane group
    int32_t u = rp.nhunits + ((int32_t)blockIdx.x - nhb) * SG + tid / LPR;
    if (LPR == 64) u = __builtin_amdgcn_readfirstlane(u);
    if (u >= rp.nunits) return;
    const int4 un = rp.units[u];
    if (un.x < 0) return;  // padding of the XCD-class layout
    stamp(epi, 1);
    gather_rows<VEC, U, 1, O32>(rp.items, un.y, un.z, 0, B, ldb, colv, colok, acc);
    stamp(epi, 2);
    finish_row<LPR, VEC, NP>(acc, un.x, colv, colok, bv, lg, C, ldc, epi, store_main, proj, pa);
    stamp(epi, 3);
    return;
  }

  // ---- heavy segment.  One unit per wavefront whose SW lane groups take nonzeros
  //      q, q + SW, ... (LPR < 64); with whole-wavefront groups (LPR == 64) one
  //      unit per workgroup, its WPB wavefronts interleaving the nonzeros and
  //      meeting in LDS.  Either way GS = SW * (LPR == 64 ? WPB : 1) groups
  //      share the segment and every sum has a fixed order.
  constexpr bool WG = WPB > 1 && (LPR == 64 || (kNarrowWG && LPR >= kNarrowMin));
  constexpr int GS = WG ? SW * WPB : SW;
  __shared__ T s_red[WG ? WPB : 1][64];
  __shared__ int32_t s_last;
  const int lane = tid & 63;
  const int w = tid / 64;
  const int q = WG ? w * SW + lane / LPR : lane / LPR;
  const int32_t u = WG ? (int32_t)blockIdx.x : __builtin_amdgcn_readfirstlane((int32_t)blockIdx.x * WPB + w);
  if (u >= rp.nhunits) return;  // WG: uniform over the workgroup
  const int4 un = rp.units[u];
  if (LPR == 64 && GCNK_HEAVY_DIRECT && rp.segp > 0) {
    // the unit word and the padded items load together (a padding unit's items are all -1)
    gather_rows_wave_direct<VEC, kHeavyU, GS, O32>(rp.hitems + (int64_t)u * rp.segp, rp.segp, q, B, ldb, colv, colok,
                                                   acc);
    if (un.x < 0) return;           // padding of the XCD-class layout (workgroup-uniform)
  } else {
    if (un.x < 0) return;           // padding of the XCD-class layout
    stamp(epi, 1);
    if constexpr (LPR == 64) gather_rows_wave<VEC, kHeavyU, GS, O32>(rp.items, un.y, un.z, q, B, ldb, colv, colok, acc);
    else gather_rows<VEC, U, GS, O32>(rp.items, un.y, un.z, q, B, ldb, colv, colok, acc);
  }
  wave_group_sum<LPR>(acc);  // the wave's SW groups (no-op at LPR = 64)
  if constexpr (WG) {
    if (w > 0) s_red[w][lane] = acc;
    __syncthreads();
#pragma unroll
    for (int v = 1; v < WPB; ++v) V::add(acc, s_red[v][lane]);  // every wave: same order, same bits
  }
  stamp(epi, 2);
  if (un.w < 0) {  // the row's only segment
    if constexpr (LPR == 64) {  // (workgroup-uniform here)
      proj.template begin<BLOCK>(pa, F);
      proj.template finish_stage<BLOCK>(pa, F);
    }
    if (q == 0) finish_row<LPR, VEC, NP>(acc, un.x, colv, colok, bv, lg, C, ldc, epi, store_main, proj, pa);
    stamp(epi, 3);
    return;
  }
  // publish this segment's partial, then count in; the last arriver sums all of
  // the entry's partials in segment order.  A row of more than kMaxSeg segments
  // has one entry per group of at most kMaxSeg of them (.w = the row's slot for
  // the group's sum) and a top entry (.w = -2) whose slots spmm_heavy_top_kernel
  // sums after this launch: segments stay ipc-sized on power-law rows and no
  // combine reads more than kMaxSeg partials
  const int32_t hid = un.w >> 6;  // heavy entry, segment un.w & 63
  const int4 hv = rp.heavy[hid];
  int32_t* ctr = rp.cnt + (int64_t)hid * kMaxColTiles + blockIdx.y;
  int32_t last = 0;
  // (the unit, hence the slot row, is wave-uniform; lane group 0 stores)
  if constexpr (LPR == 64) {
    if (q == 0 && colok) store_coherent_v(uniform_ptr(part + (int64_t)(hv.y + (un.w & 63)) * part_ld), colv, acc);
  } else {
    if (q == 0 && colok) store_coherent(part + (int64_t)(hv.y + (un.w & 63)) * part_ld + colv, acc);
  }
  if (!WG || w == 0) {  // the wavefront that stored counts in, after its stores completed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int32_t arrived = 0;
    if (lane == 0) arrived = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = __builtin_amdgcn_readfirstlane(arrived) == hv.z - 1;
  }
  if constexpr (WG) {
    if (tid == 0) s_last = last;
    __syncthreads();
    last = s_last;
  }
  stamp(epi, 3);
  if (!last) return;
  // group q sums slots q, q + GS, ... (U loads in flight), then the groups meet
  if constexpr (LPR == 64) proj.template begin<BLOCK>(pa, F);  // in flight with the partial loads
  T sum = V::zero();
  if (colok) {
    const float* p0 = uniform_ptr(part + (int64_t)hv.y * part_ld);
    for (int32_t s0 = q; s0 < hv.z; s0 += GS * U) {
      T pv[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int32_t sl = s0 + GS * j;
        // base: the row's first slot (wave-uniform); byte offsets stay below
        // kMaxSeg * part_ld * 4 < 2^31 (checked at launch)
        if constexpr (LPR == 64)
          pv[j] = sl < hv.z ? load_coherent_v<T>(p0, (int64_t)sl * part_ld + colv) : V::zero();
        else
          pv[j] = sl < hv.z ? load_coherent<T>(p0 + (int64_t)sl * part_ld + colv) : V::zero();
      }
#pragma unroll
      for (int j = 0; j < U; ++j)
        if (s0 + GS * j < hv.z) V::add(sum, pv[j]);
    }
  }
  wave_group_sum<LPR>(sum);
  if constexpr (WG) {
    __syncthreads();  // s_red reuse
    if (w > 0) s_red[w][lane] = sum;
    __syncthreads();
#pragma unroll
    for (int v = 1; v < WPB; ++v) V::add(sum, s_red[v][lane]);
  }
  if constexpr (LPR == 64) proj.template finish_stage<BLOCK>(pa, F);  // the last arriver (workgroup-uniform)
  if (q == 0) {
    if (hv.w >= 0) {  // a group of a row of > kMaxSeg segments: its sum into the row's slot hv.w
      if constexpr (LPR == 64) {
        if (colok) store_coherent_v(uniform_ptr(part + (int64_t)hv.w * part_ld), colv, sum);
      } else {
        if (colok) store_coherent(part + (int64_t)hv.w * part_ld + colv, sum);
      }
    } else {
      finish_row<LPR, VEC, NP>(sum, hv.x, colv, colok, bv, lg, C, ldc, epi, store_main, proj, pa);
    }
    if (lane == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  stamp(epi, 3);
}

// Rows of more than kMaxSeg segments, after the row kernel: each top heavy
// entry's slots (its groups' sums, in group order) summed, the epilogue applied,
// the row stored.  One workgroup per heavy entry (entries that are not tops
// exit at once) x column tile of 256 VEC.
template <int VEC>
__global__ void __launch_bounds__(256) spmm_heavy_top_kernel(const int4* __restrict__ heavy, int32_t nheavy,
                                                            const float* __restrict__ part, int64_t part_ld, int32_t F,
                                                            float* __restrict__ C, int64_t ldc, Epi epi) {
  resolve_rng(epi);
  using V = Vec<VEC>;
  using T = typename V::T;
  const int4 hv = heavy[blockIdx.x];
  if (hv.w != -2) return;   // (workgroup-uniform)
  const int64_t colv = ((int64_t)blockIdx.y * 256 + threadIdx.x) * VEC;
  if (colv >= F) return;
  T acc = V::zero();
  for (int32_t s = 0; s < hv.z; ++s) V::add(acc, load_coherent<T>(part + (int64_t)(hv.y + s) * part_ld + colv));
  const T bv = epi.bias ? V::load(epi.bias + colv) : V::zero();
  V::store(C + (int64_t)hv.x * ldc + colv, V::epi(epi, acc, bv, hv.x, colv));
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

template <bool VEC4, int NT, bool DIAG>
__device__ __forceinline__ void tile_body(int32_t bx, const int4* __restrict__ tdesc, const int32_t* __restrict__ tcols,
                                          const float* __restrict__ tfrag, const int32_t* __restrict__ trows,
                                          const float* __restrict__ dval, int32_t F, const float* __restrict__ B,
                                          int64_t ldb, float* __restrict__ C, int64_t ldc, const Epi& epi,
                                          float* __restrict__ slabs, int64_t slab_ld, int32_t item0, int32_t nitems,
                                          int32_t nslices) {
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
  // XCD-aware order: workgroups b and b + 8 share an XCD, so the column slices
  // of one chunk are placed 8 apart -- they read the same A fragments (and
  // the same condensed B rows' cache lines) through one L2
  const int32_t per = 8 * nslices;
  const int32_t slice = (bx % per) / 8;
  const int32_t it = (bx / per) * 8 + (bx & 7);
  if (it >= nitems) return;  // padding of the last group of 8 (whole workgroup)
  const int64_t item = (int64_t)it + item0;
  stamp(epi, 0);
  // block, nrows | contiguous run length << 8 | width << 16, slab (-1: single chunk), run start
  const int4 d0 = tdesc[item];
  const int32_t run = (d0.y >> 8) & 0xff;
  const int4 d = make_int4(d0.x, d0.y & 0xff, d0.z, d0.w);
  const int64_t col0 = (int64_t)slice * (NT * 16);  // this workgroup's column slice

  if (run == 0 && tid < kKC) s_cols[tid] = tcols[item * kKC + tid];
  // output rows, their extracted diagonal and the bias: loads issued now, held
  // in registers (their descriptor -> row list -> diagonal chain runs behind the
  // staging and the MFMAs) and parked in LDS only after the MFMA phase
  constexpr int CWP = NT * 16;
  static_assert(CWP <= 256, "one bias element per thread");
  __shared__ int32_t s_rows[kRB];
  __shared__ float s_dv[kRB];
  __shared__ __attribute__((aligned(16))) float s_bias[CWP];
  const bool single = d.z < 0;
  int32_t r_own = -1;
  float dv_own = 0.f, bias_own = 0.f;
  if (tid < kRB) {
    r_own = tid < d.y ? trows[(int64_t)d.x * kRB + tid] : -1;
    dv_own = (single && dval) ? dval[(int64_t)d.x * kRB + tid] : 0.f;  // 0 past the block's rows
  }
  {
    const int64_t c = (int64_t)slice * CWP + tid;
    if (tid < CWP) bias_own = (single && epi.bias && c < F) ? epi.bias[c] : 0.f;
  }
  // A fragments of this wave: 16 consecutive floats per lane
  const float4* af = reinterpret_cast<const float4*>(tfrag + ((item * 4 + wave) * 64 + lane) * 16);
  const float4 a0 = af[0], a1 = af[1], a2 = af[2], a3 = af[3];
  // ---- stage the chunk's B rows, columns [0, 16*NT): element (k, n) -> s_B[k][n&15][n>>4]
  // all of a thread's loads issue before any LDS store (one memory latency, not PT);
  // a contiguous run needs no column list, so its loads issue before the barrier
  // (not behind the descriptor -> row list -> diagonal chain the barrier waits for)
  constexpr int nq = NT * 4;  // float4 per staged row
  constexpr int PT = (kKC * nq + 255) / 256;
  float4 v[PT];
  uint32_t okm = 0;  // VEC4: loads whose piece is real
  static_assert(PT <= 32, "one mask bit per load");
  auto fetch = [&](bool contiguous) {
#pragma unroll
    for (int p = 0; p < PT; ++p) {
      const int q = tid + p * 256;
      const int k = q / nq, c4 = q % nq;
      const int32_t src = q < kKC * nq ? (contiguous ? (k < run ? d.w + k : -1) : s_cols[k]) : -1;
      const int64_t col = col0 + c4 * 4;
      if constexpr (VEC4) {
        // branch-free, so the loads form one straight run and each phase below
        // waits only for its own; an invalid piece reads B[0, 0..3] and is
        // zeroed when it is written to LDS
        const bool ok = src >= 0 && col < F;
        v[p] = *reinterpret_cast<const float4*>(B + (ok ? (int64_t)src * ldb + col : 0));
        okm |= (uint32_t)ok << p;
        continue;
      }
      v[p] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (src >= 0) {
        const float* bp = B + (int64_t)src * ldb + col;
        {
          if (col + 0 < F) v[p].x = bp[0];
          if (col + 1 < F) v[p].y = bp[1];
          if (col + 2 < F) v[p].z = bp[2];
          if (col + 3 < F) v[p].w = bp[3];
        }
      }
    }
  };
  // ---- LDS writes and MFMA k-steps in NPH phases: phase h writes the staged
  //      values of loads [p0, p1) -- the compiler waits only for those (a
  //      wave's loads return in issue order) -- then runs the k-steps whose rows
  //      they complete, so the MFMAs of the first rows overlap the arrival of
  //      the last ones instead of following the whole staging.
  auto put = [&](int p) {
    const int q = tid + p * 256;
    if (q >= kKC * nq) return;
    const int k = q / nq, c4 = q % nq;
    const int n = c4 * 4, nt = n >> 4, nc0 = n & 15;
    float* dst = s_B + k * stride + nc0 * LR + nt;
    const bool ok = !VEC4 || ((okm >> p) & 1);
    dst[0] = ok ? v[p].x : 0.f;
    dst[LR] = ok ? v[p].y : 0.f;
    dst[2 * LR] = ok ? v[p].z : 0.f;
    dst[3 * LR] = ok ? v[p].w : 0.f;
  };
  f32x4 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float a[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                       a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
  const int kr = lane >> 4, nc = lane & 15;
  // all 16 k-steps, padding included: skipping the zero steps of narrow chunks
  // (R8 X's 50-column document blocks: 13 of 16) measured no faster (10.70 vs
  // 10.75 us) and, written as a guarded unrolled loop, slower (12.98 us)
  auto ksteps = [&](auto s0c, auto s1c) {
#pragma unroll
    for (int s = decltype(s0c)::value; s < decltype(s1c)::value; ++s) {
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
  };
  constexpr int NPH = GCNK_TILE_PHASES;
  static_assert(NPH == 1 || NPH == 2 || NPH == 4, "k-step phases");
  // loads [0, pend(h)) hold every staged row below 64 (h + 1) / NPH
  auto phase = [&](auto hc) {
    constexpr int h = decltype(hc)::value;
    constexpr int p0 = h == 0 ? 0 : (h == NPH ? PT : (kKC * h / NPH * nq + 255) / 256);
    constexpr int p1 = h + 1 == NPH ? PT : (kKC * (h + 1) / NPH * nq + 255) / 256;
#pragma unroll
    for (int p = p0 < PT ? p0 : PT; p < (p1 < PT ? p1 : PT); ++p) put(p);
    __syncthreads();
    if (h == 0) stamp(epi, 1);
    ksteps(std::integral_constant<int, 16 * h / NPH>{}, std::integral_constant<int, 16 * (h + 1) / NPH>{});
  };
  // the two staging paths stay apart up to the last MFMA: where they merged
  // the compiler's wait before the first k-steps fell back to (almost) all loads
  auto stage_and_multiply = [&](auto contiguous) {
    if constexpr (decltype(contiguous)::value) {
      fetch(true);
    } else {
      __syncthreads();  // s_cols
      fetch(false);
    }
    phase(std::integral_constant<int, 0>{});
    if constexpr (NPH > 1) phase(std::integral_constant<int, 1>{});
    if constexpr (NPH > 2) {
      phase(std::integral_constant<int, 2>{});
      phase(std::integral_constant<int, 3>{});
    }
  };
  if (run > 0) stage_and_multiply(std::true_type{});
  else stage_and_multiply(std::false_type{});

  stamp(epi, 2);
  // ---- output through LDS: the accumulators (C/D layout: block row 16*wave +
  //      4*(lane>>4) + j, column 16*nt + (lane&15)) are parked row-major in the
  //      (no longer needed) B tile, then every thread writes whole 16-B pieces
  //      of rows: single-chunk blocks finish here (+ extracted diagonal,
  //      epilogue), others leave the block's real rows as a slab for
  //      spmm_tile_reduce_kernel.
  constexpr int CW = NT * 16;                                   // staged columns
  constexpr int CS = (kKC * stride >= kRB * (CW + 4)) ? CW + 4 : CW;  // row stride (floats)
  static_assert(kKC * stride >= kRB * CS, "output tile must fit the B tile");
  __syncthreads();  // all waves are done reading s_B
  if (tid < kRB) {
    s_rows[tid] = r_own;
    s_dv[tid] = dv_own;
  }
  if (tid < CWP) s_bias[tid] = bias_own;
  float* s_C = s_B;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int j = 0; j < 4; ++j) s_C[(16 * wave + 4 * (lane >> 4) + j) * CS + nt * 16 + nc] = acc[nt][j];
  __syncthreads();
  constexpr int nq4 = CW / 4;  // 16-B pieces per staged row
  for (int e = tid; e < kRB * nq4; e += 256) {
    const int rl = e / nq4;
    const int64_t col = col0 + (int64_t)(e % nq4) * 4;
    if (rl >= d.y || col >= F) continue;
    float4 v = *reinterpret_cast<const float4*>(s_C + rl * CS + (col - col0));
    // every path ends in ONE 16-B store (separate store sites are sunk into a
    // common one that the backend splits into dword + dwordx3)
    float* dst;
    if (!single) {  // slab rows are padded to 16 floats: whole pieces stay inside the row
      dst = slabs + ((int64_t)d.z * kRB + rl) * slab_ld + col;
    } else {
      const int64_t row = s_rows[rl];
      const float dv = s_dv[rl];
      dst = C + row * ldc + col;
      if (VEC4 && epi.code <= GCNK_EPI_BIAS_RELU) {
        // common case, vectorised (no dropout): + extracted diagonal * B row piece,
        // + bias, relu
        if (DIAG && dv != 0.f) {  // (a load here would wait for every store before it)
          const float4 b4 = *reinterpret_cast<const float4*>(B + row * ldb + col);
          v.x = fmaf(dv, b4.x, v.x); v.y = fmaf(dv, b4.y, v.y); v.z = fmaf(dv, b4.z, v.z); v.w = fmaf(dv, b4.w, v.w);
        }
        if (epi.code != GCNK_EPI_NONE) {
          const float4 b4 = *reinterpret_cast<const float4*>(s_bias + (col - col0));
          v.x += b4.x; v.y += b4.y; v.z += b4.z; v.w += b4.w;
          if (epi.code == GCNK_EPI_BIAS_RELU) {
            v.x = v.x > 0.f ? v.x : 0.f; v.y = v.y > 0.f ? v.y : 0.f;
            v.z = v.z > 0.f ? v.z : 0.f; v.w = v.w > 0.f ? v.w : 0.f;
          }
        }
      } else {
        float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (col + i >= F) break;
          if (DIAG && dv != 0.f) o[i] = fmaf(dv, B[row * ldb + col + i], o[i]);
          o[i] = apply_epi(epi, o[i], s_bias[col - col0 + i], row, col + i);
        }
        if (!VEC4) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (col + i < F) dst[i] = o[i];
          continue;
        }
        v = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
#if GCNK_TILE_SC1 == 2   // (experiment: nontemporal stores)
    store_nt(dst, v);
#elif GCNK_TILE_SC1
    {
      const float* base = uniform_ptr(single ? C : slabs);
      const int64_t off = dst - base;
      if (off >= 0 && off < ((int64_t)1 << 29)) store_coherent_v(base, off, v);
      else Vec<4>::store_aligned(dst, v);
    }
#else
    Vec<4>::store_aligned(dst, v);
#endif
  }
  stamp(epi, 3);
}

template <bool VEC4, int NT, bool DIAG>
__global__ void __launch_bounds__(256)
spmm_tile_kernel(const int4* __restrict__ tdesc, const int32_t* __restrict__ tcols, const float* __restrict__ tfrag,
                 const int32_t* __restrict__ trows, const float* __restrict__ dval, int32_t F,
                 const float* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc, Epi epi,
                 float* __restrict__ slabs, int64_t slab_ld, int32_t item0, int32_t nitems, int32_t nslices) {
  resolve_rng(epi);
  tile_body<VEC4, NT, DIAG>((int32_t)blockIdx.x, tdesc, tcols, tfrag, trows, dval, F, B, ldb, C, ldc, epi, slabs,
                            slab_ld, item0, nitems, nslices);
}

// Multi-chunk dense blocks: out[row, :] = epi(sum over the block's slabs, in
// chunk order).  256 threads = 16 slab lanes x 16 float4 column lanes; a
// workgroup covers one row x 64 columns; slab lanes take slabs strided by 16,
// then the 16 partial sums are added in lane order through LDS.  The row's
// reduce entry (row, slabs, diagonal) is the only plan read, so the slab loads
// (and the diagonal's B row) issue one latency after entry.
__device__ __forceinline__ void reduce_body(int32_t bx, int32_t by, int32_t bz, const int4* __restrict__ red,
                                            int32_t F, const float* __restrict__ slabs, int64_t slab_ld,
                                            const float* __restrict__ B, int64_t ldb, float* __restrict__ C,
                                            int64_t ldc, const Epi& epi) {
  __shared__ float4 s_acc[16][16];
  const int32_t rl = by;  // row within block
  const int sl = threadIdx.x >> 4, c4 = threadIdx.x & 15;
  const int64_t col = (int64_t)bz * 64 + c4 * 4;
  // the bias first: no wait behind the slab loads
  float bcol[4] = {0.f, 0.f, 0.f, 0.f};
  if (sl == 0 && epi.bias)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (col + i < F) bcol[i] = epi.bias[col + i];
  const int4 rr = red[(int64_t)bx * kRB + rl];  // row, first slab, slabs, diagonal bits
  if (rr.x < 0) return;
  const int64_t row = rr.x;
  const float dv = __int_as_float(rr.w);
  float brow[4] = {0.f, 0.f, 0.f, 0.f};
  if (sl == 0 && dv != 0.f)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (col + i < F) brow[i] = B[row * ldb + col + i];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  // slab rows are padded to 16 floats (slab_ld % 16 == 0): whole float4 reads stay
  // inside the row; lanes past F are never stored.
  if (col < F) {
    // slab lane sl sums slabs sl, sl + 16, ... in order, 8 loads in flight (one
    // round for up to 128 slabs)
    const int64_t step = (int64_t)16 * kRB * slab_ld;
    const float* p = slabs + ((int64_t)(rr.y + sl) * kRB + rl) * slab_ld + col;
    for (int s0 = sl; s0 < rr.z; s0 += 128, p += 8 * step) {
      float4 u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        u[j] = s0 + 16 * j < rr.z ? *reinterpret_cast<const float4*>(p + j * step) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (s0 + 16 * j >= rr.z) break;
        acc.x += u[j].x; acc.y += u[j].y; acc.z += u[j].z; acc.w += u[j].w;
      }
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
  float vals[4] = {t.x, t.y, t.z, t.w};
  for (int i = 0; i < 4 && col + i < F; ++i) {
    if (dv != 0.f) vals[i] = fmaf(dv, brow[i], vals[i]);
    C[row * ldc + col + i] = apply_epi(epi, vals[i], bcol[i], row, col + i);
  }
}

__global__ void __launch_bounds__(256)
spmm_tile_reduce_kernel(const int4* __restrict__ red, int32_t F, const float* __restrict__ slabs, int64_t slab_ld,
                        const float* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc, Epi epi,
                        int32_t nred, SideReduce side) {
  if ((int32_t)blockIdx.x >= nred) {   // extra columns of the grid: a carried side reduce (workgroup-uniform)
    __shared__ float s_side[16][17];
    const int64_t blk = ((int64_t)(blockIdx.x - nred) * gridDim.y + blockIdx.y) * gridDim.z + blockIdx.z;
    if (blk < side_reduce_blocks(side)) side_reduce_body(side, blk, s_side);
    return;
  }
  resolve_rng(epi);
  reduce_body((int32_t)blockIdx.x, (int32_t)blockIdx.y, (int32_t)blockIdx.z, red, F, slabs, slab_ld, B, ldb, C, ldc,
              epi);
}

// ---------------------------------------------------------------------------
// Dispatch

inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// Lanes per group from F alone (a plan does not depend on pointer alignment,
// which only picks VEC at launch): the smallest power of two covering the row
// in VEC-wide vectors, at most 64 (a whole wavefront per row and column tile;
// heavy segments then belong to a 4-wavefront workgroup).  Measured against
// 16/32-lane groups in profiles/r01_sweep_rows*.log.
inline int choose_lpr(int32_t F, int lanes_hint) {
  if (lanes_hint > 0) return next_pow2(lanes_hint > 64 ? 64 : lanes_hint);
  const int Wv = (F % 4 == 0) ? F / 4 : F;
  return Wv <= 64 ? next_pow2(Wv < 1 ? 1 : Wv) : 64;
}

// Narrow groups use one-wave workgroups so a light launch still spans the chip.
inline int choose_block(int lpr) { return lpr == 64 ? kWaveBlock : lpr >= kNarrowMin ? 256 : 64; }

struct RowLaunch {
  RowPlan rp;
  int32_t K;  // rows of B (bounds the 32-bit gather offsets)
  const float* B;
  int64_t ldb;
  int32_t F;
  float* C;
  int64_t ldc;
  Epi epi;
  float* part;  // heavy-segment partial slots
  int64_t part_ld;
  ProjArgs pa;
  hipStream_t s;
};

template <int BLOCK, int LPR, int VEC, int U, int NP>
int launch_rows(const RowLaunch& a) {
  constexpr int SG = BLOCK / LPR, WPB = BLOCK / 64;
  constexpr int LPB = LPR == 64 ? SG * kLightRPW : SG;  // light units per workgroup
  // heavy segments: one per workgroup for whole-wavefront groups, else one per wavefront
  const int64_t nhb = (LPR == 64 || (kNarrowWG && LPR >= kNarrowMin && WPB > 1)) ? (int64_t)a.rp.nhunits
                                                            : ((int64_t)a.rp.nhunits + WPB - 1) / WPB;
  const int64_t nlb = ((int64_t)a.rp.nunits - a.rp.nhunits + LPB - 1) / LPB;
  if (nhb + nlb == 0) return GCNK_OK;
  if (nhb + nlb > (int64_t)INT32_MAX) {
    set_error("gcnk_spmm_csr_f32: %lld workgroups exceed the grid", (long long)(nhb + nlb));
    return GCNK_EUNSUP;
  }
  const int64_t tileF = (int64_t)LPR * VEC;
  const int64_t tiles = (a.F + tileF - 1) / tileF;
  // column windows of at most kMaxColTiles tiles (arrival counters per heavy row x tile;
  // the last arriver re-arms them, so consecutive windows on one stream reuse them)
  for (int64_t t0 = 0; t0 < tiles; t0 += kMaxColTiles) {
    const int64_t c0 = t0 * tileF;
    const int32_t Fw = (int32_t)std::min<int64_t>(a.F - c0, kMaxColTiles * tileF);
    Epi e = a.epi;
    e.bias = e.bias ? e.bias + c0 : nullptr;
    e.mask = e.mask ? e.mask + c0 : nullptr;
    e.offset += (uint64_t)c0;  // hash index shifts with the column
    // 32-bit gather offsets when every byte the launch reads lies within 4 GB of its B base
#ifndef GCNK_ROW_O32
#define GCNK_ROW_O32 1
#endif
    const bool o32 = GCNK_ROW_O32 && (int64_t)a.K * a.ldb * 4 + (int64_t)Fw * 4 < ((int64_t)1 << 32);
    const dim3 grid((unsigned)(nhb + nlb), (unsigned)((Fw + tileF - 1) / tileF));
    if (o32)
      hipLaunchKernelGGL((spmm_row_kernel<BLOCK, LPR, VEC, U, NP, true>), grid, dim3(BLOCK), 0, a.s, a.rp, (int32_t)nhb,
                         a.B + c0, a.ldb, Fw, a.C ? a.C + c0 : nullptr, a.ldc, e, a.part ? a.part + c0 : nullptr,
                         a.part_ld, a.pa);
    else
      hipLaunchKernelGGL((spmm_row_kernel<BLOCK, LPR, VEC, U, NP, false>), grid, dim3(BLOCK), 0, a.s, a.rp,
                         (int32_t)nhb, a.B + c0, a.ldb, Fw, a.C ? a.C + c0 : nullptr, a.ldc, e,
                         a.part ? a.part + c0 : nullptr, a.part_ld, a.pa);
    const int rc = launch_check("spmm_row_kernel");
    if (rc) return rc;
  }
  return GCNK_OK;
}

template <int VEC>
int dispatch_rows(int lpr, const RowLaunch& a) {
  switch (lpr) {
    case 1: return launch_rows<kNarrowMin <= 1 ? 256 : 64, 1, VEC, kRowU, 0>(a);
    case 2: return launch_rows<kNarrowMin <= 2 ? 256 : 64, 2, VEC, kRowU, 0>(a);
    case 4: return launch_rows<kNarrowMin <= 4 ? 256 : 64, 4, VEC, kRowU, 0>(a);
    case 8: return launch_rows<256, 8, VEC, kRowU, 0>(a);
    case 16: return launch_rows<256, 16, VEC, kRowU, 0>(a);
    case 32: return launch_rows<256, 32, VEC, kRowU, 0>(a);
    case 64: return launch_rows<kWaveBlock, 64, VEC, kRowU, 0>(a);
  }
  set_error("gcnk_spmm_csr_f32: unsupported lanes per group %d", lpr);
  return GCNK_EUNSUP;
}

// Fused projection variants: float4 columns, one column tile, groups of >= 16 lanes.
template <int NP>
int dispatch_rows_proj(int lpr, const RowLaunch& a) {
  switch (lpr) {
    case 16: return launch_rows<256, 16, 4, 8, NP>(a);
    case 32: return launch_rows<256, 32, 4, 8, NP>(a);
    case 64: return launch_rows<kWaveBlock, 64, 4, 8, NP>(a);
  }
  set_error("gcnk_spmm_proj_f32: no fused-projection kernel for %d lanes per group", lpr);
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
  int32_t item0;  // first chunk item of this launch
};

template <bool V4, int NT>
int launch_tile_nt(unsigned nitems, const TileArgs& t, hipStream_t s) {
  if (nitems == 0) return GCNK_OK;
  const int32_t slices = (int32_t)((t.F + NT * 16 - 1) / (NT * 16));
  const int64_t blocks = ((int64_t)nitems + 7) / 8 * 8 * slices;
  if (blocks > INT32_MAX) {
    set_error("spmm_tile_kernel: %lld workgroups exceed the grid", (long long)blocks);
    return GCNK_EUNSUP;
  }
  if (t.dval)
    hipLaunchKernelGGL((spmm_tile_kernel<V4, NT, true>), dim3((unsigned)blocks), dim3(256), 0, s, t.tdesc, t.tcols,
                       t.tfrag, t.trows, t.dval, t.F, t.B, t.ldb, t.C, t.ldc, t.epi, t.slabs, t.slab_ld, t.item0,
                       (int32_t)nitems, slices);
  else
    hipLaunchKernelGGL((spmm_tile_kernel<V4, NT, false>), dim3((unsigned)blocks), dim3(256), 0, s, t.tdesc, t.tcols,
                       t.tfrag, t.trows, t.dval, t.F, t.B, t.ldb, t.C, t.ldc, t.epi, t.slabs, t.slab_ld, t.item0,
                       (int32_t)nitems, slices);
  return launch_check("spmm_tile_kernel");
}

template <bool V4>
int launch_tile_v(int nt_need, unsigned nitems, const TileArgs& t, hipStream_t s) {
  if (nt_need <= 1) return launch_tile_nt<V4, 1>(nitems, t, s);
  if (nt_need <= 2) return launch_tile_nt<V4, 2>(nitems, t, s);
  if (nt_need <= 4) return launch_tile_nt<V4, 4>(nitems, t, s);
  if (nt_need <= 6) return launch_tile_nt<V4, 6>(nitems, t, s);
  if (nt_need <= 7) return launch_tile_nt<V4, 7>(nitems, t, s);
  if (nt_need <= 8) return launch_tile_nt<V4, 8>(nitems, t, s);
  if constexpr (kMaxNT > 8) {
    if (nt_need <= 13) return launch_tile_nt<V4, 13>(nitems, t, s);
  }
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
  std::vector<int32_t> units, heavy;  // row-kernel units (int4 each), heavy rows (int4 each)
  std::vector<int32_t> tdesc, tcols, red, trows;
  std::vector<float> tfrag, dval;  // dval: extracted diagonal of tile rows in block order (64 per block, or empty)
};

// rowptr / colind validity (host arrays): monotone row pointers, in-range columns.
int check_csr(const int32_t* rp, const int32_t* ci, int32_t M, int32_t K, int64_t nnz) {
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
    if (ci[k] < 0 || ci[k] >= K) {
      set_error("gcnk_spmm_plan: column index %d out of range [0, %d) at nonzero %lld", ci[k], K, (long long)k);
      return GCNK_EARG;
    }
  return GCNK_OK;
}

// Row-unit + dense-tile plan from host CSR arrays (vv null: layout only).
// (light_sort false: the layout and counts only -- enough for the plan's size)
int host_plan(const int32_t* rp, const int32_t* ci, const float* vv, int32_t M, int32_t K, int64_t nnz, int32_t ipc,
              int32_t groups, float dense_threshold, HostPlan& hp, bool light_sort = true) {
  const bool want_values = vv != nullptr;
  // ---- dense blocks (tile path).  Rows are grouped by degree class (factor-8
  //      buckets of the off-diagonal degree), in row order within a class, 64 per
  //      block, so rows of one shape share blocks (R8: document rows vs topic rows).
  //      A block goes to the MFMA tile path when its nonzeros fill at least
  //      dense_threshold of its condensed column set and each condensed column is
  //      used at least twice on average; its rows' diagonal entries (r < K) are
  //      taken out of the column set and added in the epilogue (dval[r] * B[r,:]).
  std::vector<char> tile_row((size_t)M, 0);
  int32_t ntile = 0, nred = 0, nslabs = 0, ntblk = 0, nsingle = 0;
  bool any_diag = false;
  hp.dval.clear();
  // the diagonal is kept aside for square operands (A-hat's self loops); a
  // rectangular operand (X) has no diagonal to speak of
  auto is_diag = [&](int32_t r, int64_t k) { return M == K && ci[(size_t)k] == r; };
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
    std::vector<int32_t> seen((size_t)K, -1);  // block stamp per column: distinct count without a sort
    int32_t stampv = 0;
    std::vector<int32_t> cols;
    std::vector<float> dv((size_t)M, 0.f);
    for (const std::vector<int32_t>& rows : cls) {
      for (size_t i0 = 0; i0 < rows.size(); i0 += kRB, ++stampv) {
        const size_t i1 = std::min(rows.size(), i0 + kRB);
        int64_t bnnz = 0, ncols = 0;
        for (size_t i = i0; i < i1; ++i) {
          const int32_t r = rows[i];
          for (int64_t k = rp[r]; k < rp[r + 1]; ++k)
            if (!is_diag(r, k)) {
              int32_t& sv = seen[(size_t)ci[(size_t)k]];
              ncols += sv != stampv;
              sv = stampv;
              ++bnnz;
            }
        }
        if (bnnz == 0) continue;
        const int64_t nrows = (int64_t)(i1 - i0);
        // the density test needs only the counts; the sorted column set is built
        // for the blocks that pass it (a sparse operand -- 1M/20M -- has none)
        if ((double)bnnz < (double)dense_threshold * (double)nrows * (double)ncols || bnnz < 2 * ncols) continue;
        cols.clear();
        for (size_t i = i0; i < i1; ++i) {
          const int32_t r = rows[i];
          for (int64_t k = rp[r]; k < rp[r + 1]; ++k)
            if (!is_diag(r, k)) cols.push_back(ci[(size_t)k]);
        }
        std::sort(cols.begin(), cols.end());
        cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
        const int32_t nch = (int32_t)((ncols + kKC - 1) / kKC);
        const int32_t first_slab = nch > 1 ? nslabs : -1;
        const int32_t blk = ntblk++;
        for (int64_t c = 0; c < ncols; ++c) cmap[(size_t)cols[(size_t)c]] = (int32_t)c;
        const size_t base_item = (size_t)ntile;
        for (int32_t ch = 0; ch < nch; ++ch) {
          // a chunk whose condensed columns are one contiguous run (R8's X: the
          // 50 topic columns; 64-column pieces of the dense topic rows) is
          // described by its first column and length (y bits 8.., w), so the
          // kernel stages its B rows without waiting for the column list
          const int64_t c0 = (int64_t)ch * kKC;
          const int32_t kc = (int32_t)std::min<int64_t>(kKC, ncols - c0);
          bool contig = true;
          for (int32_t k = 1; k < kc && contig; ++k) contig = cols[(size_t)(c0 + k)] == cols[(size_t)c0] + k;
          // y: rows | contiguous run << 8 | condensed width << 16 (the kernel's k-steps)
          hp.tdesc.insert(hp.tdesc.end(), {blk, (int32_t)nrows | (contig ? kc << 8 : 0) | kc << 16,
                                           nch > 1 ? first_slab + ch : -1, contig ? cols[(size_t)c0] : 0});
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
        if (nch > 1) {  // one reduce entry per row: the reduce kernel needs no other plan read
          for (int64_t rl = 0; rl < kRB; ++rl) {
            const int32_t r = rl < nrows ? rows[i0 + (size_t)rl] : -1;
            hp.red.insert(hp.red.end(), {r, first_slab, nch, r >= 0 ? __builtin_bit_cast(int32_t, dv[(size_t)r]) : 0});
          }
          ++nred;
          nslabs += nch;
        }
        ntile += nch;
      }
    }
    // chunk items of single-chunk blocks first, then the multi-chunk ones (which
    // also need the reduce launch): the two runs can be launched separately
    // (gcnk_spmm_csr_f32_part), e.g. on two streams
    {
      std::vector<int32_t> order;
      for (int32_t i = 0; i < ntile; ++i)
        if (hp.tdesc[(size_t)i * 4 + 2] < 0) order.push_back(i);
      nsingle = (int32_t)order.size();
      for (int32_t i = 0; i < ntile; ++i)
        if (hp.tdesc[(size_t)i * 4 + 2] >= 0) order.push_back(i);
      std::vector<int32_t> td((size_t)ntile * 4), tc((size_t)ntile * kKC);
      std::vector<float> tf((size_t)ntile * kRB * kKC);
      for (int32_t j = 0; j < ntile; ++j) {
        const size_t i = (size_t)order[(size_t)j];
        std::copy(hp.tdesc.begin() + i * 4, hp.tdesc.begin() + i * 4 + 4, td.begin() + (size_t)j * 4);
        std::copy(hp.tcols.begin() + i * kKC, hp.tcols.begin() + (i + 1) * kKC, tc.begin() + (size_t)j * kKC);
        if (!hp.tfrag.empty())
          std::copy(hp.tfrag.begin() + i * kRB * kKC, hp.tfrag.begin() + (i + 1) * kRB * kKC,
                    tf.begin() + (size_t)j * kRB * kKC);
      }
      hp.tdesc.swap(td);
      hp.tcols.swap(tc);
      if (!hp.tfrag.empty()) hp.tfrag.swap(tf);
    }
    if (any_diag) {  // block order, so kernels index it by (block, row in block) without the row list
      hp.dval.assign((size_t)ntblk * kRB, 0.f);
      for (size_t i = 0; i < hp.trows.size(); ++i)
        if (hp.trows[i] >= 0) hp.dval[i] = dv[(size_t)hp.trows[i]];
    }
  }

  // ---- row units over the other rows.  Launch geometry from `groups` = 64 / LPR.
  if (groups < 1 || groups > 64 || (groups & (groups - 1))) {
    set_error("gcnk_spmm_plan: groups %d is not a power of two in [1, 64]", groups);
    return GCNK_EARG;
  }
  const int lpr = 64 / groups;
  const int block = choose_block(lpr), wpb = block / 64, sg = block / lpr;
  const bool wg_heavy = lpr == 64 || (kNarrowWG && lpr >= kNarrowMin && wpb > 1);  // a heavy segment spans the workgroup
  const int hpb = wg_heavy ? 1 : wpb;                            // heavy units per workgroup
  const int64_t seg = (int64_t)ipc * (lpr == 64 ? wpb : groups * (wg_heavy ? wpb : 1));  // nonzeros per segment
  // light-row limit: 2 * ipc for whole-wavefront groups (two light rows share a
  // wavefront, at most kLightMax64 nonzeros each; a heavy row is walked by a
  // 4-wavefront workgroup), ipc otherwise
  const int64_t light_max = lpr == 64 ? std::min<int64_t>(2 * (int64_t)ipc, kLightMax64) : ipc;
  const int lpb = lpr == 64 ? sg * kLightRPW : sg;  // light units per workgroup
  // XCD classes.  Workgroups b and b + 8 land on one XCD (round-robin dispatch;
  // speed only, never correctness), so every unit of workgroup b is given
  // class b % 8: a light row by its row index, a heavy segment by the column
  // range it gathers (heavy rows are first cut where their sorted column
  // indices cross a class boundary).  Each XCD's L2 then serves 1/8 of B
  // instead of every XCD fetching the rows its segments happen to need
  // (R8 Â: the topic rows gather all document rows).
  constexpr int NX = 8;
  auto cls = [](int64_t i, int64_t n) { return n > 0 ? (int)(i * NX / n) : 0; };
  std::vector<std::vector<int32_t>> hq(NX), lq(NX);  // int4 units per class
  int32_t nheavy = 0;
  int64_t nslots = 0;
  bool any_top = false;
  hp.units.clear();
  hp.heavy.clear();
  std::vector<int64_t> rb, rcl;  // runs of one column class: start, class
  int64_t rr_class = 0;
  for (int32_t r = 0; r < M; ++r) {
    if (tile_row[(size_t)r]) continue;
    const int64_t b = rp[r], e = rp[r + 1], deg = e - b;
    if (deg <= light_max) {
      lq[(size_t)cls(r, M)].insert(lq[(size_t)cls(r, M)].end(), {r, (int32_t)b, (int32_t)e, -1});
      continue;
    }
    rb.clear();
    rcl.clear();
    // cut at column-class boundaries only when the runs average half a segment or
    // more (a 20-nonzero row must not become 8 tiny segments)
    if (deg * 2 >= seg * NX)
      for (int64_t k = b; k < e; ++k) {
        const int c = cls(ci[(size_t)k], K);
        if (rcl.empty() || rcl.back() != c) { rb.push_back(k); rcl.push_back(c); }
      }
    if (rb.empty() || (int64_t)rb.size() > NX) {  // short row, or columns not sorted: one run,
      rb.assign(1, b);                              // classes dealt round-robin (balance)
      rcl.assign(1, (int64_t)(rr_class++ % NX));
    }
    rb.push_back(e);
    const int64_t nruns = (int64_t)rcl.size();
    // segments of `seg` nonzeros (longer only past kMaxSegRow of them, ~200k
    // nonzeros at R8's widths): a row of more than kMaxSeg segments gets two
    // combine levels instead of longer segments, so a power-law hub is walked
    // by many short segments, not by 64 long ones
    int64_t sr = seg, nseg = 0;
    for (;;) {
      nseg = 0;
      for (int64_t i = 0; i < nruns; ++i) nseg += (rb[(size_t)i + 1] - rb[(size_t)i] + sr - 1) / sr;
      if (nseg <= kMaxSegRow) break;
      sr *= 2;
    }
    if (nseg == 1) {
      hq[(size_t)rcl[0]].insert(hq[(size_t)rcl[0]].end(), {r, (int32_t)b, (int32_t)e, -1});
      continue;
    }
    // heavy entries: one (nseg <= kMaxSeg), or a top entry over ng groups of
    // consecutive segments (group g: segments [g nseg / ng, (g + 1) nseg / ng))
    const int64_t ng = nseg <= kMaxSeg ? 1 : (nseg + kMaxSeg - 1) / kMaxSeg;
    int64_t top_slot = -1;
    if (ng > 1) {
      ++nheavy;
      hp.heavy.insert(hp.heavy.end(), {r, (int32_t)nslots, (int32_t)ng, -2});
      top_slot = nslots;
      nslots += ng;
      any_top = true;
    }
    std::vector<int32_t> seg_w((size_t)nseg);
    for (int64_t g = 0; g < ng; ++g) {
      const int64_t s0 = g * nseg / ng, s1 = (g + 1) * nseg / ng;
      const int32_t hid = nheavy++;
      hp.heavy.insert(hp.heavy.end(), {r, (int32_t)nslots, (int32_t)(s1 - s0), ng > 1 ? (int32_t)(top_slot + g) : -1});
      for (int64_t sgi = s0; sgi < s1; ++sgi) seg_w[(size_t)sgi] = (int32_t)((int64_t)hid * 64 + (sgi - s0));
      nslots += s1 - s0;
    }
    int64_t sgi = 0;
    for (int64_t i = 0; i < nruns; ++i) {
      const int64_t pb = rb[(size_t)i], len = rb[(size_t)i + 1] - pb, np = (len + sr - 1) / sr;
      std::vector<int32_t>& q = hq[(size_t)rcl[(size_t)i]];
      for (int64_t s = 0; s < np; ++s, ++sgi)
        q.insert(q.end(), {r, (int32_t)(pb + len * s / np), (int32_t)(pb + len * (s + 1) / np), seg_w[(size_t)sgi]});
    }
  }
  // lay out rounds of NX workgroups, workgroup 8k + c taking `per` units of class c
  // (empty units pad short classes)
  auto layout = [&](std::vector<std::vector<int32_t>>& qs, int per) {
    size_t rounds = 0;
    for (const auto& q : qs) rounds = std::max(rounds, (q.size() / 4 + per - 1) / per);
    for (size_t k = 0; k < rounds; ++k)
      for (int c = 0; c < NX; ++c)
        for (int j = 0; j < per; ++j) {
          const size_t i = (k * per + j) * 4;
          if (i < qs[(size_t)c].size())
            hp.units.insert(hp.units.end(), qs[(size_t)c].begin() + i, qs[(size_t)c].begin() + i + 4);
          else
            hp.units.insert(hp.units.end(), {-1, 0, 0, -1});
        }
  };
#ifndef GCNK_LIGHT_SORT
#define GCNK_LIGHT_SORT 1
#endif
  // light rows of a class ordered by their off-diagonal column lists, so the
  // rows one workgroup (one CU's L1) gathers for share their B rows (R8: the
  // document rows of one topic set); each row still writes its own C row
  // (ordered by a key of the first two off-diagonal columns, the full lists only
  // on equal keys, then by position: the order of a stable sort by the lists;
  // 1M/20M: 0.49 -> 0.05 s per build)
  if (GCNK_LIGHT_SORT && light_sort)
    for (std::vector<int32_t>& q : lq) {
      const size_t n = q.size() / 4;
      std::vector<size_t> ord(n);
      for (size_t i = 0; i < n; ++i) ord[i] = i;
      std::vector<uint64_t> key(n);
      for (size_t i = 0; i < n; ++i) {
        const int32_t r = q[4 * i];
        uint64_t c[2] = {0, 0};  // column + 1, 0 past the list's end (a prefix sorts first)
        int got = 0;
        for (int32_t k = q[4 * i + 1]; k < q[4 * i + 2] && got < 2; ++k)
          if (ci[(size_t)k] != r) c[got++] = (uint64_t)ci[(size_t)k] + 1;
        key[i] = c[0] << 32 | c[1];
      }
      auto less_list = [&](size_t x, size_t y) {
        const int32_t rx = q[4 * x], ry = q[4 * y];
        int32_t kx = q[4 * x + 1], ky = q[4 * y + 1];
        const int32_t ex = q[4 * x + 2], ey = q[4 * y + 2];
        for (;;) {
          while (kx < ex && ci[(size_t)kx] == rx) ++kx;
          while (ky < ey && ci[(size_t)ky] == ry) ++ky;
          if (kx >= ex || ky >= ey) return kx >= ex && ky < ey;
          if (ci[(size_t)kx] != ci[(size_t)ky]) return ci[(size_t)kx] < ci[(size_t)ky];
          ++kx;
          ++ky;
        }
      };
      std::sort(ord.begin(), ord.end(), [&](size_t x, size_t y) {
        if (key[x] != key[y]) return key[x] < key[y];
        if (less_list(x, y)) return true;
        if (less_list(y, x)) return false;
        return x < y;
      });
      std::vector<int32_t> sorted(q.size());
      for (size_t i = 0; i < n; ++i) std::copy(q.begin() + 4 * ord[i], q.begin() + 4 * ord[i] + 4, sorted.begin() + 4 * i);
      q.swap(sorted);
    }
  layout(hq, hpb);
  const int64_t nh = (int64_t)hp.units.size() / 4;
  // padded item copies of the heavy units (whole-wavefront groups): stride = the
  // longest unit, rounded up to 4 items
  int64_t segp = 0;
  if (GCNK_HEAVY_DIRECT && lpr == 64)
    for (int64_t u = 0; u < nh; ++u)
      if (hp.units[(size_t)(4 * u)] >= 0)
        segp = std::max<int64_t>(segp, (int64_t)hp.units[(size_t)(4 * u + 2)] - hp.units[(size_t)(4 * u + 1)]);
  segp = (segp + 3) & ~3LL;
  if (segp >= (1 << 28) || 2 * nh * segp >= (int64_t)INT32_MAX) segp = 0;   // (never for real plans: keep the old path)
  layout(lq, lpb);
  const int64_t nunits = (int64_t)hp.units.size() / 4;
  if (nunits >= (int64_t)INT32_MAX || nslots >= (int64_t)INT32_MAX || nheavy >= (1 << 25)) {
    set_error("gcnk_spmm_plan: %lld row units / %lld partial slots exceed the plan's int32 fields",
              (long long)nunits, (long long)nslots);
    return GCNK_EUNSUP;
  }
  const int32_t h[16] = {kMagic, M,     K,      groups, ipc,  (int32_t)nunits, (int32_t)nh, nheavy,
                         ntile,  nred, nslabs, ntblk,  (any_diag ? 1 : 0) | (int32_t)(segp << 1) | (any_top ? 1 << 30 : 0), (int32_t)nnz,
                         (int32_t)nslots, nsingle};
  std::copy(h, h + 16, hp.hdr);
  return GCNK_OK;
}

// Full classic plan image (header, packed items, units, heavy rows, tile part).
void classic_image(const HostPlan& hp, const int32_t* ci, const float* vv, int64_t nnz, std::vector<int32_t>& img) {
  const Layout L(hp.hdr);
  img.assign((size_t)L.total, 0);
  std::copy(hp.hdr, hp.hdr + 16, img.begin());
  for (int64_t k = 0; k < nnz; ++k) {
    img[(size_t)(L.items + 2 * k)] = ci[k];
    img[(size_t)(L.items + 2 * k + 1)] = vv ? __builtin_bit_cast(int32_t, vv[k]) : 0;
  }
  auto put = [&](int64_t off, const int32_t* p, size_t n) { std::copy(p, p + n, img.begin() + off); };
  auto putf = [&](int64_t off, const std::vector<float>& v) {
    for (size_t i = 0; i < v.size(); ++i) img[(size_t)off + i] = __builtin_bit_cast(int32_t, v[i]);
  };
  put(L.units, hp.units.data(), hp.units.size());
  put(L.heavy, hp.heavy.data(), hp.heavy.size());
  put(L.tdesc, hp.tdesc.data(), hp.tdesc.size());
  put(L.tcols, hp.tcols.data(), hp.tcols.size());
  putf(L.tfrag, hp.tfrag);
  put(L.red, hp.red.data(), hp.red.size());
  put(L.trows, hp.trows.data(), hp.trows.size());
  putf(L.dval, hp.dval);
  for (int64_t u = 0; u < L.nhunits && L.segp > 0; ++u) {
    const int32_t r = hp.units[(size_t)(4 * u)], b = hp.units[(size_t)(4 * u + 1)], e = hp.units[(size_t)(4 * u + 2)];
    for (int64_t i = 0; i < L.segp; ++i) {
      const size_t o = (size_t)(L.hitems + 2 * (u * L.segp + i));
      const bool in = r >= 0 && b + i < e;
      img[o] = in ? ci[b + i] : -1;
      img[o + 1] = in && vv ? __builtin_bit_cast(int32_t, vv[b + i]) : 0;
    }
  }
}

// The row-unit + tile plan image for host CSR arrays.
int build_image(const int32_t* rp, const int32_t* ci, const float* vv, int32_t M, int32_t K, int64_t nnz, int32_t ipc,
                int32_t groups, float dense_threshold, std::vector<int32_t>& img) {
  int rc = check_csr(rp, ci, M, K, nnz);
  if (rc) return rc;
  HostPlan hp;
  if ((rc = host_plan(rp, ci, vv, M, K, nnz, ipc, groups, std::fabs(dense_threshold), hp))) return rc;
  classic_image(hp, ci, vv, nnz, img);
  return GCNK_OK;
}

// Bytes of the plan build_image would make, without making it: the size
// follows from its header (no light-row sort, no image).
int64_t plan_size(const int32_t* rp, const int32_t* ci, int32_t M, int32_t K, int64_t nnz, int32_t ipc, int32_t groups,
                  float dense_threshold) {
  int rc = check_csr(rp, ci, M, K, nnz);
  if (rc) return rc;
  HostPlan hp;
  if ((rc = host_plan(rp, ci, nullptr, M, K, nnz, ipc, groups, std::fabs(dense_threshold), hp, false))) return rc;
  return Layout(hp.hdr).total * 4;
}

bool plan_args_ok(const int32_t* rowptr, const int32_t* colind, int32_t M, int32_t K, int64_t nnz, int32_t ipc,
                  int32_t groups) {
  return rowptr && M >= 0 && K >= 0 && nnz >= 0 && nnz < INT32_MAX && ipc > 0 && groups > 0 && (nnz == 0 || colind);
}

// Device CSR -> host arrays (one-time setup: synchronises `s`).
int fetch_csr(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M, int64_t nnz, hipStream_t s,
              std::vector<int32_t>& rp, std::vector<int32_t>& ci, std::vector<float>& vv) {
  rp.resize((size_t)M + 1);
  ci.resize((size_t)nnz);
  vv.resize(val ? (size_t)nnz : 0);
  int rc = hip_check(hipMemcpyAsync(rp.data(), rowptr, ((size_t)M + 1) * 4, hipMemcpyDeviceToHost, s),
                     "plan rowptr copy");
  if (!rc && nnz > 0)
    rc = hip_check(hipMemcpyAsync(ci.data(), colind, (size_t)nnz * 4, hipMemcpyDeviceToHost, s), "plan colind copy");
  if (!rc && val && nnz > 0)
    rc = hip_check(hipMemcpyAsync(vv.data(), val, (size_t)nnz * 4, hipMemcpyDeviceToHost, s), "plan val copy");
  if (rc) return rc;
  return hip_check(hipStreamSynchronize(s), "plan copy sync");
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

#ifdef GCNK_STAMPS
static unsigned long long* g_stamps = nullptr;
extern "C" int gcnk_debug_set_stamps(void* buf) {
  g_stamps = (unsigned long long*)buf;
  return GCNK_OK;
}
#else
static constexpr unsigned long long* g_stamps = nullptr;
extern "C" int gcnk_debug_set_stamps(void* buf) {
  if (!buf) return GCNK_OK;
  set_error("gcnk_debug_set_stamps: this libgcnk was built without GCNK_STAMPS (scripts/stamps.py builds one)");
  return GCNK_EUNSUP;
}
#endif
unsigned long long* gcnk::debug_stamps() { return g_stamps; }


// Lane groups per wavefront (64 / LPR): identifies the launch geometry a plan
// is laid out for (heavy segments are shared by these groups, or by the 4
// wavefronts of a workgroup when a group is a whole wavefront).
extern "C" int32_t gcnk_spmm_groups(int32_t F, int32_t lanes_hint) { return 64 / choose_lpr(F, lanes_hint); }

extern "C" int32_t gcnk_spmm_default_ipc(int32_t M, int64_t nnz, int32_t F, int32_t lanes_hint) {
  (void)M;
  // each lane group's share of a heavy segment (the light-row limit is 2 * ipc
  // at 64 lanes, ipc below).  Narrow groups: 8 (one U = 8 gather batch; R8
  // F = 8 ipc 8 5.1 us, 16 5.7).  Whole-wavefront groups: heavy segments of
  // 4 * ipc nonzeros over a 4-wavefront workgroup, sized with the operand so
  // the heavy segments stay a few per CU: ipc ~ nnz / 5760 in [12, 32], a
  // multiple of 4.  Sweeps after the 16-B partial accesses
  // (profiles/r01_variants.log): R8 (69k nnz) ipc 12 8.67 us, 16 8.95, 20 9.24,
  // 24 9.72; 20ng-shaped (175k) 12 17.9, 16 17.0, 20 16.4, 24 16.2, 32 16.4;
  // 1M/20M F = 256: 16 and 32 both 3.37 ms.
  // 2-lane groups with workgroup-wide heavy segments (LPR >= kNarrowMin): 16
  // (round 5, after the padded heavy items: R8 F = 8 4.73 us vs 5.41 with
  // one-wave workgroups at ipc 8, profiles/r05_hub_probe_nw2.log).
  const int lpr = choose_lpr(F, lanes_hint);
  // (F = 16, 4 lanes: 8 stays best, 5.52 vs 6.13 us, profiles/r05_hub_probe_nw.log)
  if (lpr != 64) return kNarrowWG && lpr >= kNarrowMin && lpr == 2 ? 16 : 8;
  int64_t ipc = (nnz / 5760 + 2) / 4 * 4;
  return (int32_t)std::min<int64_t>(32, std::max<int64_t>(12, ipc));
}

extern "C" int64_t gcnk_spmm_plan_bytes_host(const int32_t* rowptr, const int32_t* colind, int32_t M, int32_t K,
                                             int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold) {
  if (!plan_args_ok(rowptr, colind, M, K, nnz, ipc, groups)) {
    set_error("gcnk_spmm_plan_bytes: bad argument");
    return GCNK_EARG;
  }
  return plan_size(rowptr, colind, M, K, nnz, ipc, groups, dense_threshold);
}

extern "C" int gcnk_spmm_plan_build_host(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                                         int32_t K, int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold,
                                         int32_t* plan, int64_t plan_bytes) {
  if (!plan_args_ok(rowptr, colind, M, K, nnz, ipc, groups) || !plan || (nnz > 0 && !val)) {
    set_error("gcnk_spmm_plan_build_host: bad argument");
    return GCNK_EARG;
  }
  std::vector<int32_t> img;
  const int rc = build_image(rowptr, colind, val, M, K, nnz, ipc, groups, dense_threshold, img);
  if (rc) return rc;
  if (plan_bytes < (int64_t)img.size() * 4) {
    set_error("gcnk_spmm_plan_build_host: plan buffer %lld B < %lld B", (long long)plan_bytes,
              (long long)img.size() * 4);
    return GCNK_EARG;
  }
  std::copy(img.begin(), img.end(), plan);
  return GCNK_OK;
}

extern "C" int64_t gcnk_spmm_plan_bytes(const int32_t* rowptr, const int32_t* colind, int32_t M, int32_t K,
                                        int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold, void* stream) {
  if (!plan_args_ok(rowptr, colind, M, K, nnz, ipc, groups)) {
    set_error("gcnk_spmm_plan_bytes: bad argument");
    return GCNK_EARG;
  }
  std::vector<int32_t> rp, ci;
  std::vector<float> vv;
  const int rc = fetch_csr(rowptr, colind, nullptr, M, nnz, (hipStream_t)stream, rp, ci, vv);
  return rc ? rc : plan_size(rp.data(), ci.data(), M, K, nnz, ipc, groups, dense_threshold);
}

extern "C" int gcnk_spmm_plan_build(const int32_t* rowptr, const int32_t* colind, const float* val, int32_t M,
                                    int32_t K, int64_t nnz, int32_t ipc, int32_t groups, float dense_threshold,
                                    void* plan, int64_t plan_bytes, void* stream) {
  if (!plan_args_ok(rowptr, colind, M, K, nnz, ipc, groups) || !plan || (nnz > 0 && !val)) {
    set_error("gcnk_spmm_plan_build: bad argument (M=%d nnz=%lld ipc=%d groups=%d)", M, (long long)nnz, ipc, groups);
    return GCNK_EARG;
  }
  hipStream_t s = (hipStream_t)stream;
  std::vector<int32_t> rp, ci, img;
  std::vector<float> vv;
  int rc = fetch_csr(rowptr, colind, val, M, nnz, s, rp, ci, vv);
  if (!rc) rc = build_image(rp.data(), ci.data(), vv.data(), M, K, nnz, ipc, groups, dense_threshold, img);
  if (rc) return rc;
  if (plan_bytes < (int64_t)img.size() * 4) {
    set_error("gcnk_spmm_plan_build: plan buffer %lld B < %lld B", (long long)plan_bytes, (long long)img.size() * 4);
    return GCNK_EARG;
  }
  rc = hip_check(hipMemcpyAsync(plan, img.data(), img.size() * 4, hipMemcpyHostToDevice, s), "plan upload");
  // the host image must outlive the async copy
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

static bool L_tops(const int32_t* hdr) { return ((uint32_t)hdr[12] >> 30) & 1; }

static bool plan_magic(const int32_t* hdr) {
  return hdr && hdr[0] == kMagic;
}

extern "C" int64_t gcnk_spmm_workspace_bytes(const int32_t* hdr, int32_t F) {
  if (!plan_magic(hdr) || F < 0) return GCNK_EARG;
  const int64_t ld = ((int64_t)F + 3) & ~3LL;
  const int64_t rows = (int64_t)hdr[14] * ld * 4;
  const int64_t slabs = (int64_t)hdr[10] * kRB * tile_fpad(F) * 4;
  return ((rows + 255) & ~255LL) + slabs;
}

extern "C" int64_t gcnk_spmm_counter_bytes(const int32_t* hdr) {
  if (!plan_magic(hdr)) return GCNK_EARG;
  return (int64_t)hdr[7] * kMaxColTiles * 4;
}

static int spmm_impl(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F, float* C,
                     int64_t ldc, const float* bias, int32_t epilogue, const uint8_t* drop_mask, int64_t ldm,
                     float drop_scale, float keep_prob, uint64_t seed, uint64_t offset, const uint64_t* rng_base,
                     float* workspace, int64_t workspace_bytes, int32_t* counters, int64_t counter_bytes, int32_t lanes_hint,
                     const ProjArgs& pa, void* stream, int32_t part = 0, const SideReduce* side = nullptr,
                     int* carried = nullptr) {
  if (carried) *carried = 0;
  if (!plan || !plan_magic(hdr) || F < 0 || part < 0 || part > 2) {
    set_error("gcnk_spmm_csr_f32: bad argument (plan/header missing or not a gcnk plan, F=%d)", F);
    return GCNK_EARG;
  }
  const int32_t M = hdr[1], K = hdr[2];
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
  if (hdr[3] != 64 / lpr) {
    set_error("gcnk_spmm_csr_f32: plan built for %d lane groups per wavefront, this F/lanes uses %d (gcnk_spmm_groups)",
              hdr[3], 64 / lpr);
    return GCNK_EARG;
  }
  const int64_t need = gcnk_spmm_workspace_bytes(hdr, F);
  if (need > 0 && (!workspace || workspace_bytes < need)) {
    set_error("gcnk_spmm_csr_f32: plan needs %lld B of workspace, got %lld", (long long)need,
              (long long)workspace_bytes);
    return GCNK_EARG;
  }
  const int64_t cneed = gcnk_spmm_counter_bytes(hdr);
  if (cneed > 0 && (!counters || counter_bytes < cneed)) {
    set_error("gcnk_spmm_csr_f32: plan needs a zeroed counter region of %lld B, got %lld", (long long)cneed,
              (long long)counter_bytes);
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
  e.rng_base = rng_base;
  e.code = epilogue;
  e.stamps = g_stamps;
  const bool vec4 = (F % 4 == 0) && (ldb % 4 == 0) && (ldc % 4 == 0) && aligned16(B) && (!C || aligned16(C)) &&
                    (!workspace || aligned16(workspace)) && (!bias || aligned16(bias));
  hipStream_t s = (hipStream_t)stream;
  if (proj) {
    // the projection needs whole rows in one group: row-kernel rows only, float4, one column tile
    if (hdr[8] > 0 || !vec4 || F > lpr * 4 || pa.P > 32 || lpr < 16 || L_tops(hdr)) {
      set_error("gcnk_spmm_proj_f32: fused projection unsupported here (tile chunks=%d vec4=%d F=%d P=%d lanes=%d)",
                hdr[8], (int)vec4, F, pa.P, lpr);
      return GCNK_EUNSUP;
    }
  }
  const int32_t* p = (const int32_t*)plan;
  const Layout L(hdr);
  const int64_t part_ld = ((int64_t)F + 3) & ~3LL;
  if ((int64_t)kMaxSeg * part_ld * 4 >= ((int64_t)1 << 31)) {  // partial-slot byte offsets of one heavy row
    set_error("gcnk_spmm: F = %d too wide for the partial-slot offsets", F);
    return GCNK_EUNSUP;
  }
  const int64_t rows_ws = ((int64_t)hdr[14] * part_ld * 4 + 255) & ~255LL;
  float* slabs = workspace ? reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + rows_ws) : nullptr;
  const int64_t slab_ld = tile_fpad(F);

  // ---- dense blocks: tile kernel (+ slab reduce)
  const float* dval = L.has_diag ? reinterpret_cast<const float*>(p + L.dval) : nullptr;
  if (L.ntile > 0) {
    // column slices of <= kMaxNT n-tiles on grid.y, balanced (F = 200: 4 x 4 n-tiles),
    // so two workgroups of a chunk share the staging/MFMA/store phases of a CU
    const int32_t nt_total = (int32_t)(slab_ld / 16);
    const int32_t nslices = (nt_total + kMaxNT - 1) / kMaxNT;
    if (nslices > 65535) {
      set_error("gcnk_spmm_csr_f32: F=%d needs %d tile column slices (> 65535)", F, nslices);
      return GCNK_EUNSUP;
    }
    const int4* td = reinterpret_cast<const int4*>(p + L.tdesc);
    // part 1: the single-chunk items [0, nsingle); part 2: the rest; 0: all
    const int32_t nsingle = hdr[15];
    const int nt_need = (nt_total + nslices - 1) / nslices;
    const int32_t i0 = part == 2 ? nsingle : 0, i1 = part == 1 ? nsingle : (int32_t)L.ntile;
    TileArgs ta{td, p + L.tcols, reinterpret_cast<const float*>(p + L.tfrag), p + L.trows, dval, F, B,
                ldb, C, ldc, e, slabs, slab_ld, i0};
    const int rc = launch_tile(vec4, nt_need, (unsigned)(i1 - i0), ta, s);
    if (rc) return rc;
    if (L.nred > 0 && part != 1) {
      // a carried side reduce takes extra x columns of the grid (kRB x column tiles workgroups each)
      const int64_t per_x = (int64_t)kRB * ((F + 63) / 64);
      const int64_t side_x = side ? (side_reduce_blocks(*side) + per_x - 1) / per_x : 0;
      const SideReduce none{nullptr, 0, 0, 0, 0, 0, nullptr, nullptr, nullptr};
      hipLaunchKernelGGL(spmm_tile_reduce_kernel, dim3((unsigned)(L.nred + side_x), kRB, (unsigned)((F + 63) / 64)),
                         dim3(256), 0, s, reinterpret_cast<const int4*>(p + L.red), F, slabs, slab_ld, B, ldb, C, ldc,
                         e, (int32_t)L.nred, side ? *side : none);
      if (side && carried) *carried = 1;
      int rc = launch_check("spmm_tile_reduce_kernel");
      if (rc) return rc;
    }
  }
  // ---- remaining rows: row kernel (heavy rows finished in-launch)
  if (L.nunits > 0 && part != 1) {
    RowPlan rp{reinterpret_cast<const int2*>(p + L.items), reinterpret_cast<const int4*>(p + L.units),
               reinterpret_cast<const int4*>(p + L.heavy), counters, (int32_t)L.nunits, (int32_t)L.nhunits,
               L.segp > 0 ? reinterpret_cast<const int2*>(p + L.hitems) : nullptr, (int32_t)L.segp};
    RowLaunch a{rp, K, B, ldb, F, C, ldc, e, workspace, part_ld, pa, s};
    if (proj) return pa.P <= 8 ? dispatch_rows_proj<8>(lpr, a) : dispatch_rows_proj<32>(lpr, a);
    const int rc = vec4 ? dispatch_rows<4>(lpr, a) : dispatch_rows<1>(lpr, a);
    if (rc || !L.tops) return rc;
    // rows of more than kMaxSeg segments: their groups' sums, after the row kernel
    const int vec = vec4 ? 4 : 1;
    const dim3 grid((unsigned)L.nheavy, (unsigned)((F + 256 * vec - 1) / (256 * vec)));
    if (vec4)
      hipLaunchKernelGGL(spmm_heavy_top_kernel<4>, grid, dim3(256), 0, s, reinterpret_cast<const int4*>(p + L.heavy),
                         (int32_t)L.nheavy, workspace, part_ld, F, C, ldc, e);
    else
      hipLaunchKernelGGL(spmm_heavy_top_kernel<1>, grid, dim3(256), 0, s, reinterpret_cast<const int4*>(p + L.heavy),
                         (int32_t)L.nheavy, workspace, part_ld, F, C, ldc, e);
    return launch_check("spmm_heavy_top_kernel");
  }
  return GCNK_OK;
}

extern "C" int gcnk_spmm_csr_f32(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F,
                                 float* C, int64_t ldc, const float* bias, int32_t epilogue, const uint8_t* drop_mask,
                                 int64_t ldm, float drop_scale, float keep_prob, uint64_t seed, uint64_t offset,
                                 const uint64_t* rng_base, float* workspace, int64_t workspace_bytes, int32_t* counters, int64_t counter_bytes,
                                 int32_t lanes_hint, void* stream) {
  const ProjArgs none{nullptr, 0, 0, nullptr, 0, 1};
  return spmm_impl(plan, hdr, B, ldb, F, C, ldc, bias, epilogue, drop_mask, ldm, drop_scale, keep_prob, seed, offset,
                   rng_base, workspace, workspace_bytes, counters, counter_bytes, lanes_hint, none, stream);
}

int gcnk::spmm_csr_f32_side(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F, float* C,
                            int64_t ldc, float* workspace, int64_t workspace_bytes, int32_t* counters,
                            int64_t counter_bytes, int32_t lanes_hint, void* stream, const SideReduce& side,
                            int* carried) {
  const ProjArgs none{nullptr, 0, 0, nullptr, 0, 1};
  return spmm_impl(plan, hdr, B, ldb, F, C, ldc, nullptr, GCNK_EPI_NONE, nullptr, 0, 1.f, 1.f, 0, 0, nullptr, workspace,
                   workspace_bytes, counters, counter_bytes, lanes_hint, none, stream, 0, &side, carried);
}

extern "C" int gcnk_spmm_csr_f32_part(const void* plan, const int32_t* hdr, const float* B, int64_t ldb,
                                      int32_t F, float* C, int64_t ldc, const float* bias, int32_t epilogue,
                                      const uint8_t* drop_mask, int64_t ldm, float drop_scale, float keep_prob,
                                      uint64_t seed, uint64_t offset, const uint64_t* rng_base, float* workspace,
                                      int64_t workspace_bytes,
                                      int32_t* counters, int64_t counter_bytes, int32_t lanes_hint, int32_t part,
                                      void* stream) {
  const ProjArgs none{nullptr, 0, 0, nullptr, 0, 1};
  return spmm_impl(plan, hdr, B, ldb, F, C, ldc, bias, epilogue, drop_mask, ldm, drop_scale, keep_prob, seed, offset,
                   rng_base, workspace, workspace_bytes, counters, counter_bytes, lanes_hint, none, stream, part);
}

extern "C" int gcnk_spmm_proj_f32(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F,
                                  float* C, int64_t ldc, const float* bias, int32_t epilogue,
                                  const uint8_t* drop_mask, int64_t ldm, float drop_scale, float keep_prob,
                                  uint64_t seed, uint64_t offset, const uint64_t* rng_base, const float* W, int64_t ldw, int32_t P, float* C2,
                                  int64_t ldc2, float* workspace, int64_t workspace_bytes, int32_t* counters,
                                  int64_t counter_bytes, int32_t lanes_hint, void* stream) {
  if (!W) {
    set_error("gcnk_spmm_proj_f32: null projection matrix");
    return GCNK_EARG;
  }
  const ProjArgs pa{W, ldw, P, C2, ldc2, C != nullptr};
  return spmm_impl(plan, hdr, B, ldb, F, C, ldc, bias, epilogue, drop_mask, ldm, drop_scale, keep_prob, seed, offset,
                   rng_base, workspace, workspace_bytes, counters, counter_bytes, lanes_hint, pa, stream);
}
