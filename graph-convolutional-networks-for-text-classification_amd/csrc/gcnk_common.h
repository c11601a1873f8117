// Shared helpers for libgcnk (gfx950 / CDNA4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <cstdarg>
#include <vector>
#include <atomic>

#include "../../include/gcnk.h"

namespace gcnk {

// Thread-local error text returned by gcnk_last_error().
void set_error(const char* fmt, ...);

// Debug timeline buffer (gcnk_debug_set_stamps; always null without -DGCNK_STAMPS).
unsigned long long* debug_stamps();

inline int hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return GCNK_EHIP;
  }
  return GCNK_OK;
}

// Launch-error check right after a <<<>>> launch (never synchronises).
inline int launch_check(const char* what) { return hip_check(hipGetLastError(), what); }

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device):
// the attribute belongs to the device the launch runs on, so a process that
// launches a kernel on several GPUs raises it on each (bit d of `done`, set
// after the first successful call on device d; a driver call per launch would
// cost host time on every eager forward).
inline hipError_t dyn_lds_attr(std::atomic<uint64_t>& done, const void* fn, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint64_t bit = dev >= 0 && dev < 64 ? (1ull << dev) : 0;
  if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess && bit) done.fetch_or(bit, std::memory_order_acq_rel);
  return e;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// ----------------------------------------------------------------------------
// Epilogue parameters for SpMM (row-complete elements).
struct Epi {
  const float* bias;     // may be null
  const uint8_t* mask;   // GCNK_EPI_BIAS_RELU_DROP
  int64_t ldm;
  float scale;           // dropout 1/(1-p) as ATen computes it
  float keep_prob;       // GCNK_EPI_BIAS_RELU_HASH
  uint32_t seed_lo, seed_hi;
  uint64_t offset;
  const uint64_t* rng_base;    // device word added to offset (GCNK_EPI_BIAS_RELU_HASH), may be null
  int32_t code;
  unsigned long long* stamps;  // debug timeline (gcnk_debug_set_stamps), normally null
};

// Debug timeline: 4 x s_memrealtime (100 MHz) per workgroup, written by thread 0.
// Compiled in only with -DGCNK_STAMPS (scripts/stamps.py): the runtime branch
// and its store would otherwise sit in every kernel, and the store's vmcnt
// makes the compiler's waits after it conservative.
__device__ __forceinline__ void stamp(const Epi& e, int k) {
#ifndef GCNK_STAMPS
  (void)e;
  (void)k;
  if (false) {
#else
  if (e.stamps && threadIdx.x == 0) {
#endif
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    e.stamps[4 * ((unsigned long long)blockIdx.y * gridDim.x + blockIdx.x) + k] = t;
  }
}

// Counter-based hash RNG (lowbias32-style avalanche, two rounds keyed by seed).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU;
  x ^= x >> 15; x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float hash_uniform(uint32_t seed_lo, uint32_t seed_hi, uint64_t idx) {
  uint32_t h = mix32((uint32_t)idx ^ seed_lo);
  h = mix32(h ^ (uint32_t)(idx >> 32) ^ seed_hi);
  h = mix32(h + 0x9e3779b9U);
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// `b` is bias[col] (0 when there is no bias), preloaded by the caller.
__device__ __forceinline__ float apply_epi(const Epi& e, float acc, float b, int64_t row, int64_t col) {
  if (e.code == GCNK_EPI_NONE) return acc;
  float v = acc + b;
  if (e.code == GCNK_EPI_BIAS) return v;
  v = v > 0.0f ? v : 0.0f;
  if (e.code == GCNK_EPI_BIAS_RELU) return v;
  if (e.code == GCNK_EPI_BIAS_RELU_DROP) return e.mask[row * e.ldm + col] ? v * e.scale : 0.0f;
  // GCNK_EPI_BIAS_RELU_HASH: the device offset *rng_base was folded into offset
  // at the kernel's entry (resolve_rng, every kernel with an Epi calls it).  Not
  // read here: even guarded by rng_base != null, the read left an s_waitcnt
  // vmcnt(0) on every element's path (the compiler cannot see resolve_rng
  // nulled the pointer), serialising the epilogue's H1 stores behind it
  const float u = hash_uniform(e.seed_lo, e.seed_hi, e.offset + (uint64_t)(row * e.ldm + col));
  return u < e.keep_prob ? v * e.scale : 0.0f;
}

// A hash-dropout epilogue's device stream offset (*rng_base), read ONCE at a
// kernel's entry and folded into offset: apply_epi reading it per element put a
// dependent global load in front of every kept / dropped decision (behind the
// epilogue's own stores, so the compiler could not reuse it).
__device__ __forceinline__ void resolve_rng(Epi& e) {
  if (e.code == GCNK_EPI_BIAS_RELU_HASH && e.rng_base) {
    e.offset += *e.rng_base;
    e.rng_base = nullptr;
  }
}

// Column vectors of a lane: VEC = 4 (float4, 16-B accesses) or 1 (scalar).
template <int VEC>
struct Vec;

template <>
struct Vec<4> {
  using T = float4;
  static __device__ __forceinline__ T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  static __device__ __forceinline__ T load(const float* p) { return *reinterpret_cast<const float4*>(p); }
  static __device__ __forceinline__ void store(float* p, const T& v) { *reinterpret_cast<float4*>(p) = v; }
  // one 16-B store instruction whatever the surrounding control flow
  static __device__ __forceinline__ void store_aligned(float* p, const T& v) {
    typedef float f4a __attribute__((ext_vector_type(4), aligned(16)));
    *reinterpret_cast<f4a*>(__builtin_assume_aligned(p, 16)) = f4a{v.x, v.y, v.z, v.w};
  }
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
    // the dropout-free codes tested once for the four elements (per element,
    // each apply_epi carried its own chain of code tests and the dropout paths'
    // blocks sat between them); the same arithmetic as apply_epi
    if (e.code <= GCNK_EPI_BIAS_RELU) {
      if (e.code == GCNK_EPI_NONE) return a;
      r = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
      if (e.code == GCNK_EPI_BIAS) return r;
      r.x = r.x > 0.0f ? r.x : 0.0f; r.y = r.y > 0.0f ? r.y : 0.0f;
      r.z = r.z > 0.0f ? r.z : 0.0f; r.w = r.w > 0.0f ? r.w : 0.0f;
      return r;
    }
    if (e.code == GCNK_EPI_BIAS_RELU_HASH) {   // apply_epi's hash mask, the element index formed once
      const uint64_t i0 = e.offset + (uint64_t)(row * e.ldm + col);
      const float v[4] = {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w};
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float h = v[j] > 0.0f ? v[j] : 0.0f;
        o[j] = hash_uniform(e.seed_lo, e.seed_hi, i0 + (uint64_t)j) < e.keep_prob ? h * e.scale : 0.0f;
      }
      return make_float4(o[0], o[1], o[2], o[3]);
    }
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
  static __device__ __forceinline__ void store_aligned(float* p, const T& v) { *p = v; }
  static __device__ __forceinline__ void fma(T& acc, float a, const T& b) { acc = fmaf(a, b, acc); }
  static __device__ __forceinline__ void add(T& acc, const T& b) { acc += b; }
  static __device__ __forceinline__ T epi(const Epi& e, const T& a, const T& b, int64_t row, int64_t col) {
    return apply_epi(e, a, b, row, col);
  }
};


// One LDS-DMA load per lane (global_load_lds): global gsrc -> LDS at
// lds_wave + BYTES * lane (lds_wave wave-uniform).  Asynchronous: covered by
// the wave's vmcnt.
__device__ __forceinline__ void lds_dma16(const void* gsrc, void* lds_wave) {
  __builtin_amdgcn_global_load_lds(const_cast<void*>(gsrc), (__attribute__((address_space(3))) void*)lds_wave, 16, 0, 0);
}
__device__ __forceinline__ void lds_dma4(const void* gsrc, void* lds_wave) {
  __builtin_amdgcn_global_load_lds(const_cast<void*>(gsrc), (__attribute__((address_space(3))) void*)lds_wave, 4, 0, 0);
}

// ----------------------------------------------------------------------------
// A pending fixed-order sum over per-workgroup partials -- gcn_bwd2's gW2 / gb1
// / gb2 (csrc/bwd.hip) -- that another launch of the same backward carries as
// extra workgroups (round 6: the backward record runs it inside X^T gS1's tile
// reduce launch instead of a launch of its own).  out[e] = sum over b of
// part[b * part_ld + e], b in order: 16 entries x 16 workgroup lanes per
// workgroup of 256 threads, each lane summing workgroups l, l + 16, ... (16
// loads in flight), then the 16 lanes in order through LDS.
struct SideReduce {
  const float* part;
  int64_t part_ld;
  int32_t nblk, N, P, with_g;
  float *gW, *gb1, *gb2;
};

__host__ __device__ inline int64_t side_reduce_entries(const SideReduce& r) {
  return (int64_t)r.N * r.P + r.N + (r.with_g ? r.P : 0);
}
__host__ __device__ inline int64_t side_reduce_blocks(const SideReduce& r) { return (side_reduce_entries(r) + 15) / 16; }

// workgroup `blk` of the side reduce (256 threads; s: 16 x 17 floats of LDS)
__device__ __forceinline__ void side_reduce_body(const SideReduce& r, int64_t blk, float (*s)[17]) {
  const int el = threadIdx.x & 15, bl = threadIdx.x >> 4;
  const int64_t E = side_reduce_entries(r);
  const int64_t e = blk * 16 + el;
  float acc = 0.f;
  if (e < E) {
    for (int32_t b0 = bl; b0 < r.nblk; b0 += 16 * 16) {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = b0 + 16 * j < r.nblk ? r.part[(int64_t)(b0 + 16 * j) * r.part_ld + e] : 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (b0 + 16 * j < r.nblk) acc += v[j];
    }
  }
  s[bl][el] = acc;
  __syncthreads();
  if (bl != 0 || e >= E) return;
  float t = s[0][el];
  for (int q = 1; q < 16; ++q) t += s[q][el];
  const int64_t NP = (int64_t)r.N * r.P;
  if (e < NP) {
    if (r.gW) r.gW[e] = t;
  } else if (e < NP + r.N) {
    if (r.gb1) r.gb1[e - NP] = t;
  } else if (r.gb2) {
    r.gb2[e - NP - r.N] = t;
  }
}

// gcn_bwd2's main launch only, its reduce returned in *side (csrc/bwd.hip), and
// that reduce as a launch of its own
int gcn_bwd2_main(const float* H, int64_t ldh, const float* gS, int64_t ldgs, const float* W, int64_t ldw,
                  const float* G, int64_t ldg, int32_t M, int32_t N, int32_t P, float scale, float* Z, int64_t ldz,
                  float* gW, float* gb1, float* gb2, void* workspace, int64_t workspace_bytes, void* stream,
                  SideReduce* side);
int side_reduce_launch(const SideReduce& side, void* stream);
// gcnk_spmm_csr_f32 carrying `side` in its tile reduce launch when it has one
// (*carried = 1); otherwise the side reduce is left to the caller (*carried = 0)
int spmm_csr_f32_side(const void* plan, const int32_t* hdr, const float* B, int64_t ldb, int32_t F, float* C,
                      int64_t ldc, float* workspace, int64_t workspace_bytes, int32_t* counters,
                      int64_t counter_bytes, int32_t lanes_hint, void* stream, const SideReduce& side, int* carried);

}  // namespace gcnk
