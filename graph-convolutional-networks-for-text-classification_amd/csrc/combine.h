// Pieces shared by the kernels that hand partial results from workgroup to
// workgroup inside one launch (hub.hip: hub rows; xw.hip: split-K rows):
// LDS-DMA staging, coherent (sc1) raw-buffer accesses, the fused projection
// partial, and the in-launch combine with its counter region.
#pragma once

#include "gcnk_common.h"

namespace gcnk {
namespace {

constexpr int kMaxSlices = 64;          // column slices per launch (counter region size)
constexpr int kLdsMax = 163840;         // gfx950: 160 KiB per workgroup
constexpr int kLdsDyn = kLdsMax - 1024;  // dynamic part (static LDS of a kernel: a few words)
constexpr int kProjMax = 8;             // widest fused projection (gc2's W2: R8 8 classes)
constexpr int kCombineChunks = 8;       // row chunks per column slice, combined by the last 8 arrivals
constexpr int kCombineLanes = 16;       // lanes summing one combined output's partials (power of two)
constexpr int kCombineSpins = 1 << 12;  // poll bound of a waiting combiner (then the last arrival takes over)

__host__ __device__ inline int64_t align4(int64_t x) { return (x + 3) & ~3LL; }

// bytes of the counter region of a plan that combines in-launch
inline int64_t combine_counter_bytes() { return (int64_t)kMaxSlices * (1 + kCombineChunks) * 8; }

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

// Coherent (sc1) raw-buffer accesses from a wave-uniform base: the hub
// partials are handed from every group's workgroup to the combining ones in
// the same launch, stored write-through and loaded past L1
// (MI355X_MICROARCH.md, valid hand-off forms: sc1 stores drained by every
// storing wave, one lane's agent-scope add per workgroup, sc1 loads).
typedef float f32v4 __attribute__((ext_vector_type(4)));
constexpr int kBufSc1 = 16;             // cache-policy aux bit sc1 (gfx950)
constexpr int kBufDword3 = 0x00020000;  // raw buffer resource word 3 (gfx9)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base_uniform) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base_uniform), (short)0, 0x7fffffff, kBufDword3);
}
__device__ __forceinline__ const float* uniform_ptr(const float* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return reinterpret_cast<const float*>(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void store_sc1(const float* base, int64_t off, const float4& v) {
  const f32v4 x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, rsrc(base), (int)(off * 4), 0, kBufSc1);
}
__device__ __forceinline__ void store_sc1(const float* base, int64_t off, const float& v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc(base), (int)(off * 4), 0, kBufSc1);
}
template <typename T>
__device__ __forceinline__ T load_sc1(const float* base, int64_t off);
template <>
__device__ __forceinline__ float4 load_sc1<float4>(const float* base, int64_t off) {
  const f32v4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), (int)(off * 4), 0, kBufSc1);
  return make_float4(x.x, x.y, x.z, x.w);
}
template <>
__device__ __forceinline__ float load_sc1<float>(const float* base, int64_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc(base), (int)(off * 4), 0, kBufSc1));
}

// Optional fused work around the product (template flags of the kernel):
//   PROJ  (gc1 -> gc2, layer.py:106,110,182,185 then :102): every finished
//         element of H = epi(A B) is projected by W [F x P] while in registers;
//         slice c of the launch writes C2[c][row][:P] = H[row, slice c] x
//         W[slice c, :] (the P-wide partial over its columns, summed over the
//         slice's columns in order); the consumer sums the slices in order
//         (gcnk_spmm_sum_csr_f32).  H itself is stored only when C != null.
//   BSUM  (the consumer): B = sum over s < nsum of B_s (B_s at B + s * bstride),
//         summed in order as the rows are staged.
struct HubExtra {
  const float* W;      // PROJ: [F x P], leading dimension ldw
  int64_t ldw;
  int32_t P;
  float* C2;           // PROJ: slice c's partial projection at C2 + c * c2_stride
  int64_t c2_stride, ldc2;
  int32_t nsum;        // BSUM: operand count
  int64_t bstride;
};

// Projection partial of one finished float4 of columns 4 (q0 + j) .. + 3:
// out[p] = sum over the 4 columns of v[col] * W[col, p]  (s_w: the slice's W
// rows, kProjMax wide, zero past P).
__device__ __forceinline__ void project4(const float4& v, int32_t j, const float* s_w, int32_t P, float* out) {
  const float* wr = s_w + (int64_t)4 * j * kProjMax;
#pragma unroll
  for (int pp = 0; pp < kProjMax; ++pp) {
    float a = v.x * wr[pp];
    a = fmaf(v.y, wr[kProjMax + pp], a);
    a = fmaf(v.z, wr[2 * kProjMax + pp], a);
    a = fmaf(v.w, wr[3 * kProjMax + pp], a);
    if (pp < P) out[pp] = a;
  }
}
__device__ __forceinline__ void project4(const float& v, int32_t j, const float* s_w, int32_t P, float* out) {
  (void)v; (void)j; (void)s_w; (void)P; (void)out;  // PROJ is float4-only
}

// In-launch combine of the hub rows of column slice c.  Counter region
// (uint64, zeroed once, never reset -- every value is relative to the launch
// count, so consecutive launches on one stream need no clearing):
//   ctr[c]                 arrivals at slice c, + G per launch
//   ctr[kMaxSlices + c*K + q]  launch count at which chunk q of slice c was
//                              last combined (claim word)
// Every workgroup of slice c adds 1 after its partials are stored (drained).
// The last K arrivals of a launch each combine one chunk of the H hub rows
// (K = 8, or 1 -- the last arrival alone, nobody waits -- when the grid has
// more workgroups than the device has CUs, so a waiter could hold a CU that a
// workgroup it waits for needs)
// (ranks G-K .. G-1 -> chunks 0 .. K-1) once all G have arrived; the very
// last arrival (which never waits) also takes over every chunk nobody has
// claimed, so a waiter that gives up (bounded poll) loses nothing.  A chunk
// is claimed by a compare-and-swap of its claim word from the launch count
// to launch count + 1: exactly one claimant per launch.  Chunk sums run in
// group order (fixed): the result does not depend on who combines.
template <int BLOCK, int VEC, bool PROJ>
__device__ __forceinline__ void hub_combine(uint64_t* ctr, int32_t K, int32_t* s_scr, int32_t G, int32_t c, int32_t h0,
                                            int32_t H, int32_t w, int32_t q0, const float* part_u, int64_t part_ld,
                                            float* C, int64_t ldc, const Epi& epi,
                                            const typename Vec<VEC>::T* s_bias, const float* s_w, float* s_proj,
                                            const HubExtra& x, int tid) {
  using V = Vec<VEC>;
  using T = typename V::T;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores have landed
  __syncthreads();                                   // ... and every other wave's
  uint64_t* cnt = ctr + c;
  __shared__ uint64_t s_old;
  __shared__ int32_t s_flag;
  if (tid == 0) s_old = __hip_atomic_fetch_add(cnt, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  stamp(epi, 2);
  const uint64_t old = s_old;
  const uint64_t launch = old / (uint64_t)G;
  const int32_t rank = (int32_t)(old - launch * (uint64_t)G);
  if (rank < G - K) return;
  const int32_t q_own = rank - (G - K);
  const bool last = rank == G - 1;
  if (!last) {
    if (tid == 0) {
      const uint64_t target = (launch + 1) * (uint64_t)G;
      int32_t ok = 0;
      for (int32_t spin = 0; spin < kCombineSpins; ++spin) {
        if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) {
          ok = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      s_flag = ok;
    }
    __syncthreads();
    if (!s_flag) return;  // gave up: the last arrival combines this chunk
  }
  uint64_t* claim = ctr + kMaxSlices + (int64_t)c * kCombineChunks;
  // chunk order: own chunk first, then (last arrival only) all the others
  for (int32_t k = 0; k < (last ? K : 1); ++k) {
    const int32_t q = (q_own + k) % K;
    __syncthreads();  // s_flag reuse
    if (tid == 0) {
      uint64_t expect = launch;
      s_flag = __hip_atomic_compare_exchange_strong(claim + q, &expect, launch + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT) ? 1 : 0;
    }
    __syncthreads();
    if (!s_flag) continue;
    // chunk q: hubs [t0, t1) x the slice's w vectors; PL lanes per output,
    // lane p summing groups [p G / PL, (p + 1) G / PL) in order, then a
    // fixed-order LDS tree over the PL lanes
    const int32_t t0 = (int32_t)((int64_t)q * H / K), t1 = (int32_t)((int64_t)(q + 1) * H / K);
    const int32_t nout = (t1 - t0) * w;
    // lanes per output: enough that one pass covers the chunk (all its loads
    // in flight at once), at most kCombineLanes
    int PL = kCombineLanes;
    while (PL > 1 && (BLOCK / PL) < nout) PL >>= 1;
    T* s_red = reinterpret_cast<T*>(s_scr);
    for (int32_t o0 = 0; o0 < nout; o0 += BLOCK / PL) {
      const int32_t o = o0 + tid / PL, p = tid % PL;
      T acc = V::zero();
      if (o < nout) {
        const int32_t t = t0 + o / w, j = o % w;
        const int64_t base = (int64_t)t * G * part_ld + (int64_t)(q0 + j) * VEC;
        const int32_t ga = (int32_t)((int64_t)p * G / PL), gb = (int32_t)((int64_t)(p + 1) * G / PL);
#pragma unroll 8
        for (int32_t gg = ga; gg < gb; ++gg) V::add(acc, load_sc1<T>(part_u, base + (int64_t)gg * part_ld));
      }
      s_red[tid] = acc;
      __syncthreads();
      for (int sh = PL / 2; sh >= 1; sh >>= 1) {
        if (p < sh) V::add(s_red[tid], s_red[tid + sh]);
        __syncthreads();
      }
      if (p == 0 && o < nout) {
        const int32_t t = t0 + o / w, j = o % w;
        const int64_t row = (int64_t)h0 + t, cv = (int64_t)(q0 + j) * VEC;
        const T bv = epi.bias ? s_bias[j] : V::zero();
        const T v = V::epi(epi, s_red[tid], bv, row, cv);
        if (C) V::store(C + row * ldc + cv, v);
        if constexpr (PROJ) project4(v, j, s_w, x.P, s_proj + (int64_t)o * kProjMax);
      }
      __syncthreads();
    }
    if constexpr (PROJ) {  // chunk rows' projection partials: sum over the slice's vectors in order
      for (int32_t e = tid; e < (t1 - t0) * x.P; e += BLOCK) {
        const int32_t tt = e / x.P, pp = e - tt * x.P;
        float a = 0.f;
        for (int32_t j = 0; j < w; ++j) a += s_proj[(int64_t)(tt * w + j) * kProjMax + pp];
        x.C2[(int64_t)c * x.c2_stride + ((int64_t)h0 + t0 + tt) * x.ldc2 + pp] = a;
      }
    }
  }
}


}  // namespace
}  // namespace gcnk
