// Shared helpers for libgcnk (gfx950 / CDNA4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <cstdarg>

#include "../../include/gcnk.h"

namespace gcnk {

// Thread-local error text returned by gcnk_last_error().
void set_error(const char* fmt, ...);

inline int hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return GCNK_EHIP;
  }
  return GCNK_OK;
}

// Launch-error check right after a <<<>>> launch (never synchronises).
inline int launch_check(const char* what) { return hip_check(hipGetLastError(), what); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

struct Coord {
  int32_t x;  // row (merge-path: row ends consumed)
  int32_t y;  // nonzero index (merge-path: nonzeros consumed)
};

// Plan header words (see gcnk.h): nslots, nfix, ipc, nchunks, G, nsuper, 0, 0.
constexpr int kPlanHeader = 8;

__host__ __device__ inline int64_t plan_nchunks(int32_t M, int64_t nnz, int32_t ipc) {
  return ((int64_t)M + nnz + ipc - 1) / ipc;
}

// Plan section offsets in int32 words.  Chunks (ipc path items each) are the
// per-group work units; a "super-chunk" is the G consecutive chunks one
// workgroup owns.  Split-row partial slots and the fix-up list are kept per
// super-chunk (rows split inside one workgroup are combined in LDS).
struct PlanLayout {
  int64_t nchunks, nsuper, coords, head, tail, fix, fix_index, total;
  __host__ __device__ PlanLayout(int64_t nc, int32_t G) {
    nchunks = nc;
    nsuper = (nc + G - 1) / G;
    coords = kPlanHeader;
    head = coords + 2 * (nc + 1);
    tail = head + nsuper;
    fix = tail + nsuper;
    fix_index = fix + 2 * nsuper;
    total = fix_index + nsuper;
  }
};

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
  int32_t code;
  unsigned long long* stamps;  // debug timeline (gcnk_debug_set_stamps), normally null
};

// Debug timeline: 4 x s_memrealtime (100 MHz) per workgroup, written by thread 0.
__device__ __forceinline__ void stamp(const Epi& e, int k) {
  if (e.stamps && threadIdx.x == 0) {
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
  // GCNK_EPI_BIAS_RELU_HASH
  const float u = hash_uniform(e.seed_lo, e.seed_hi, e.offset + (uint64_t)(row * e.ldm + col));
  return u < e.keep_prob ? v * e.scale : 0.0f;
}

}  // namespace gcnk
