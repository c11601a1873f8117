// Standalone microbenchmark: R8 A-hat x S1 (F = 200, bias + ReLU) by a
// "push" schedule, measured piece by piece (doc rows, hub partials, hub
// finish) against a copy of the same bytes.  Not the product library: it
// finds out which schedule is worth moving into csrc/.
//   build: hipcc -O3 --offload-arch=gfx950 -std=c++17 hub_micro.hip -o hub_micro
//   run:   python scripts/micro/dump_r8.py /tmp/r8_adj.bin && ./hub_micro /tmp/r8_adj.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      exit(2);                                                                                \
    }                                                                                         \
  } while (0)

constexpr int kBlock = 256;

__device__ __forceinline__ void lds_dma16(const void* g, void* lds_wave) {
  __builtin_amdgcn_global_load_lds(const_cast<void*>(g), (__attribute__((address_space(3))) void*)lds_wave, 16, 0, 0);
}
__device__ __forceinline__ void fma4(float4& a, float s, const float4& b) {
  a.x = fmaf(s, b.x, a.x); a.y = fmaf(s, b.y, a.y); a.z = fmaf(s, b.z, a.z); a.w = fmaf(s, b.w, a.w);
}
__device__ __forceinline__ void add4(float4& a, const float4& b) { a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w; }
__device__ __forceinline__ float4 relu_bias(float4 a, float4 b) {
  a.x = fmaxf(a.x + b.x, 0.f); a.y = fmaxf(a.y + b.y, 0.f); a.z = fmaxf(a.z + b.z, 0.f); a.w = fmaxf(a.w + b.w, 0.f);
  return a;
}
__device__ __forceinline__ int rl(int v, int i) { return __builtin_amdgcn_readlane(v, i); }
__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

struct Args {
  const int* rp; const int* ci; const float* v;  // CSR of A-hat
  const float4* B; float4* C; const float4* bias;
  int M, Q, h0, H, nL;
  // doc role
  int rpw, nD;
  // part role
  const int* rec; int R, G, gs, nslices; float4* part;
  // fin role
  const int* hh_rp; const int2* hh;  // hub x hub items per hub row {col t', val bits}
  unsigned long long* stamps;
  const int2* win;                   // doc2: per-wave item windows {(row << 8) | slot, val}
  const int* rec2; int R2;           // part2: records with hub x hub items
  const int* rec3; int R3;           // slice3: doc entries + hub batches in one record
  const int2* ell;                   // docP: 16 items per light row {col | -1 self, val}
  unsigned long long* ctr;           // slice3c: per-slice arrival counters (never reset)
};

__device__ __forceinline__ int light_row(int l, int h0, int H) { return l < h0 ? l : l + H; }
typedef float f32v4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st_sc1(const void* base, int off_bytes, const float4& v) {
  const f32v4 x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, rsrc(base), off_bytes, 0, 16);
}
__device__ __forceinline__ float4 ld_sc1(const void* base, int off_bytes) {
  const f32v4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), off_bytes, 0, 16);
  return make_float4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void stamp(const Args& a, int k) {
  if (a.stamps && threadIdx.x == 0) a.stamps[4 * blockIdx.x + k] = now();
}

// ---------------------------------------------------------------------------
// Role D: full-width document rows.  Workgroup b: light rows [b*4*rpw, ...),
// wave wv: rpw consecutive rows.  LDS: hub rows [H][Q] | self rows [4*rpw][Q].
template <int RPW, int DV>
__device__ void doc_role(const Args& a, int b, float4* s) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Q = a.Q;
  float4* s_hub = s;
  float4* s_self = s + a.H * Q;
  // hub rows (contiguous in B: rows h0 .. h0+H-1)
  const float4* Bh = a.B + (size_t)a.h0 * Q;
  if (DV != 1)
    for (int e0 = wv * 64; e0 < a.H * Q; e0 += kBlock) {
      const int e = e0 + lane;
      if (e < a.H * Q) lds_dma16(Bh + e, s_hub + e0);
    }
  const int l0 = (b * 4 + wv) * RPW;
  const int nr = max(0, min(RPW, a.nL - l0));
  const int row0 = light_row(l0, a.h0, a.H);  // the wave's rows are contiguous (host-checked)
  float4 self[RPW];
  if (DV != 0) {
#pragma unroll
    for (int k = 0; k < RPW; ++k) self[k] = (k < nr && lane < Q) ? a.B[(size_t)(row0 + k) * Q + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (nr > 0 && DV == 0) {
    const float4* Bs = a.B + (size_t)row0 * Q;
    for (int e0 = 0; e0 < nr * Q; e0 += 64) {
      const int e = e0 + lane;
      if (e < nr * Q) lds_dma16(Bs + e, s_self + wv * RPW * Q + e0);
    }
  }
  const int rpv = (nr > 0 && lane <= nr) ? a.rp[row0 + lane] : 0;
  const int base = rl(rpv, 0);
  const int nit = rl(rpv, nr) - base;
  const int ci0 = lane < nit ? a.ci[base + lane] : 0;
  const int ci1 = lane + 64 < nit ? a.ci[base + 64 + lane] : 0;
  const int vv0 = lane < nit ? __float_as_int(a.v[base + lane]) : 0;
  const int vv1 = lane + 64 < nit ? __float_as_int(a.v[base + 64 + lane]) : 0;
  const float4 bv = lane < Q ? a.bias[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  stamp(a, 1);
  if (DV != 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  stamp(a, 2);
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    if (k < nr) {
      const int row = row0 + k;
      const int ia = rl(rpv, k) - base, ib = rl(rpv, k + 1) - base;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int it = ia; it < ib; it += 4) {
        float4 r[4];
        float w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int idx = it + u;
          int c, wb;
          if (idx < 64) { c = rl(ci0, idx & 63); wb = rl(vv0, idx & 63); }
          else { c = rl(ci1, idx & 63); wb = rl(vv1, idx & 63); }
          const bool ok = idx < ib;
          const bool self_it = ok && c == row;
          w[u] = ok ? __int_as_float(wb) : 0.f;
          if (DV == 0) {
            const int slot = !ok ? 0 : (self_it ? a.H + wv * RPW + k : c - a.h0);
            r[u] = s[slot * Q + lane];
          } else if (DV == 2) {
            r[u] = self_it ? self[k] : s[(ok ? c - a.h0 : 0) * Q + lane];
          } else {
            r[u] = self_it ? self[k] : a.B[(size_t)(ok ? c : a.h0) * Q + min(lane, Q - 1)];
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) fma4(acc, w[u], r[u]);
      }
      if (lane < Q) a.C[(size_t)row * Q + lane] = relu_bias(acc, bv);
    }
  }
}

// ---------------------------------------------------------------------------
// Role P: hub partials of row group g over column slice c.
// Record (int32): 0 n  1 nb  2 o_items  3 -  | batches int2 {t, first item} [nb]
// | hub batch offsets [H + 1] | items int2 {slot, val} (slot n = zero row)
constexpr int kHubBatch = 8;
__device__ void part_role(const Args& a, int bb, float4* s) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Q = a.Q;
  const int g = bb % a.G, c = bb / a.G;
  const int q0 = c * Q / a.nslices, q1 = (c + 1) * Q / a.nslices, w = q1 - q0;
  const int* rec = a.rec + (size_t)g * a.R;
  int* s_rec = reinterpret_cast<int*>(s);
  float4* s_doc = s + a.R / 4;
  for (int k0 = wv * 64; k0 < a.R / 4; k0 += kBlock) {
    const int k = k0 + lane;
    if (k < a.R / 4) lds_dma16(rec + 4 * k, s_rec + 4 * k0);
  }
  const int l0 = g * a.gs;
  const int n = min(a.gs, a.nL - l0);
  for (int e0 = wv * 64; e0 < n * w; e0 += kBlock) {
    const int e = e0 + lane;
    const int i = e / w, j = e - i * w;
    if (e < n * w) lds_dma16(a.B + (size_t)light_row(l0 + i, a.h0, a.H) * Q + q0 + j, s_doc + e0);
  }
  if (tid < w) s_doc[n * w + tid] = make_float4(0.f, 0.f, 0.f, 0.f);
  stamp(a, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(a, 2);
  const int nb = s_rec[1], o_it = s_rec[2];
  const int2* s_b = reinterpret_cast<const int2*>(s_rec + 4);
  const int* s_off = s_rec + 4 + 2 * nb;
  const int4* s_it = reinterpret_cast<const int4*>(s_rec + o_it);
  float4* s_sum = s_doc + (n + 1) * w;
  for (int e = tid; e < nb * w; e += kBlock) {
    const int bi = e / w, j = e - bi * w;
    const int first = s_b[bi].y;
    int4 p[kHubBatch / 2];
#pragma unroll
    for (int u = 0; u < kHubBatch / 2; ++u) p[u] = s_it[first / 2 + u];
    float4 r[kHubBatch];
#pragma unroll
    for (int u = 0; u < kHubBatch / 2; ++u) {
      r[2 * u] = s_doc[p[u].x * w + j];
      r[2 * u + 1] = s_doc[p[u].z * w + j];
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < kHubBatch / 2; ++u) {
      fma4(acc, __int_as_float(p[u].y), r[2 * u]);
      fma4(acc, __int_as_float(p[u].w), r[2 * u + 1]);
    }
    s_sum[e] = acc;
  }
  __syncthreads();
  for (int e = tid; e < a.H * w; e += kBlock) {
    const int t = e / w, j = e - t * w;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int bi = s_off[t]; bi < s_off[t + 1]; ++bi) add4(acc, s_sum[bi * w + j]);
    a.part[((size_t)t * a.G + g) * Q + q0 + j] = acc;
  }
}

// ---------------------------------------------------------------------------
// Role F: hub row outputs (t, j) from the G partials + hub x hub nonzeros.
// 8 lanes per output: lane p sums partials p, p+8, ...; butterfly; lane 0 adds
// the hub x hub terms and applies the epilogue.
constexpr int kFinLanes = 8;
__device__ void fin_role(const Args& a, int bb) {
  const int tid = threadIdx.x;
  const int o = bb * (kBlock / kFinLanes) + tid / kFinLanes, p = tid % kFinLanes;
  const int Q = a.Q;
  const bool ok = o < a.H * Q;
  const int t = ok ? o / Q : 0, j = ok ? o - t * Q : 0;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok)
    for (int g = p; g < a.G; g += kFinLanes) add4(acc, a.part[((size_t)t * a.G + g) * Q + j]);
  if (ok) {
    const int k0 = a.hh_rp[t], k1 = a.hh_rp[t + 1];
    for (int k = k0 + p; k < k1; k += kFinLanes) {
      const int2 it = a.hh[k];
      fma4(acc, __int_as_float(it.y), a.B[(size_t)(a.h0 + it.x) * Q + j]);
    }
  }
  const float4 bj = ok ? a.bias[j] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int m = kFinLanes / 2; m >= 1; m >>= 1) {
    acc.x += __shfl_xor(acc.x, m); acc.y += __shfl_xor(acc.y, m);
    acc.z += __shfl_xor(acc.z, m); acc.w += __shfl_xor(acc.w, m);
  }
  if (ok && p == 0) a.C[(size_t)(a.h0 + t) * Q + j] = relu_bias(acc, bj);
}

// roles by blockIdx range: [0, nD) doc, [nD, nD + nP) part, [nD + nP, ...) fin
template <int RPW, int DV>
__global__ void __launch_bounds__(kBlock) roles_kernel(Args a, int nD, int nP) {
  extern __shared__ __attribute__((aligned(16))) float4 smem[];
  stamp(a, 0);
  const int b = blockIdx.x;
  if (b < nD) doc_role<RPW, DV>(a, b, smem);
  else if (b < nD + nP) part_role(a, b - nD, smem);
  else fin_role(a, b - nD - nP);
  stamp(a, 3);
}


// ===========================================================================
// v2 roles: one dependent memory round trip per workgroup, compiler-visible
// waits, stores last.
constexpr int kWin = 64;       // items per doc2 wave window
constexpr int kSelfSlot = 255;
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0) expcnt(7) lgkmcnt(15)

template <int BS, int RPW, int ABL = 0>
__device__ void doc2_role(const Args& a, int b, float4* s) {
  constexpr int NW = BS / 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Q = a.Q;
  const float4* Bh = a.B + (size_t)a.h0 * Q;
  if (!(ABL & 1))
    for (int e0 = wv * 64; e0 < a.H * Q; e0 += BS) {
      const int e = e0 + lane;
      if (e < a.H * Q) lds_dma16(Bh + e, s + e0);
    }
  const int wave = b * NW + wv;
  const int l0 = wave * RPW;
  const int nr = max(0, min(RPW, a.nL - l0));
  const int row0 = light_row(l0, a.h0, a.H);
  float4 self[RPW];
#pragma unroll
  for (int k = 0; k < RPW; ++k)
    self[k] = (k < nr && lane < Q) ? a.B[(size_t)(row0 + k) * Q + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  const int2 it = nr > 0 ? a.win[(size_t)wave * kWin + lane] : make_int2(0xff00, 0);
  const float4 bv = lane < Q ? a.bias[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  wait_vm0();
  __syncthreads();
  stamp(a, 2);
  float4 out[RPW];
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const unsigned long long m = __ballot((it.x >> 8) == k);
    const int first = m ? __builtin_ctzll(m) : 0, cnt = __builtin_popcountll(m);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ABL & 2) { out[k] = relu_bias(self[k], bv); continue; }
    for (int q = 0; q < cnt; q += 4) {
      float4 r[4];
      float w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = q + u < cnt;
        const int idx = (first + q + u) & 63;
        const int meta = rl(it.x, idx), wb = rl(it.y, idx);
        const int slot = meta & 0xff;
        w[u] = ok ? __int_as_float(wb) : 0.f;
        const bool sf = ok && slot == kSelfSlot;
        r[u] = s[(ok && !sf ? slot : 0) * Q + lane];
        if (sf) r[u] = self[k];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) fma4(acc, w[u], r[u]);
    }
    out[k] = relu_bias(acc, bv);
  }
  if (a.stamps && threadIdx.x == 0) a.stamps[4 * blockIdx.x + 1] = now();  // compute done (overrides "issued")
  if (!(ABL & 4)) {
#pragma unroll
    for (int k = 0; k < RPW; ++k)
      if (k < nr && lane < Q) a.C[(size_t)(row0 + k) * Q + lane] = out[k];
  } else if (out[0].x == 1234.5f) a.C[0] = out[0];
}

// part2: record | LDS rows: doc slices [n][w] | zero row | hub slices [H][w] | batch sums
template <int BS>
__device__ void part2_role(const Args& a, int bb, float4* s) {
  constexpr int NW = BS / 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Q = a.Q;
  const int g = bb % a.G, c = bb / a.G;
  const int q0 = c * Q / a.nslices, q1 = (c + 1) * Q / a.nslices, w = q1 - q0;
  const int l0 = g * a.gs;
  const int n = min(a.gs, a.nL - l0);
  int* s_rec = reinterpret_cast<int*>(s);
  float4* s_row = s + a.R2 / 4;
  if (tid < w) s_row[n * w + tid] = make_float4(0.f, 0.f, 0.f, 0.f);  // before any LDS-DMA is in flight
  const int* rec = a.rec2 + (size_t)g * a.R2;
  for (int k0 = wv * 64; k0 < a.R2 / 4; k0 += BS) {
    const int k = k0 + lane;
    if (k < a.R2 / 4) lds_dma16(rec + 4 * k, s_rec + 4 * k0);
  }
  for (int e0 = wv * 64; e0 < n * w; e0 += BS) {
    const int e = e0 + lane;
    const int i = e / w, j = e - i * w;
    if (e < n * w) lds_dma16(a.B + (size_t)light_row(l0 + i, a.h0, a.H) * Q + q0 + j, s_row + e0);
  }
  float4* s_hubs = s_row + (n + 1) * w;
  for (int e0 = wv * 64; e0 < a.H * w; e0 += BS) {
    const int e = e0 + lane;
    const int t = e / w, j = e - t * w;
    if (e < a.H * w) lds_dma16(a.B + (size_t)(a.h0 + t) * Q + q0 + j, s_hubs + e0);
  }
  stamp(a, 1);
  wait_vm0();
  __syncthreads();
  stamp(a, 2);
  const int nb = s_rec[1], o_it = s_rec[2];
  const int2* s_b = reinterpret_cast<const int2*>(s_rec + 4);
  const int* s_off = s_rec + 4 + 2 * nb;
  const int4* s_it = reinterpret_cast<const int4*>(s_rec + o_it);
  float4* s_sum = s_hubs + a.H * w;
  for (int e = tid; e < nb * w; e += BS) {
    const int bi = e / w, j = e - bi * w;
    const int first = s_b[bi].y;
    int4 p[kHubBatch / 2];
#pragma unroll
    for (int u = 0; u < kHubBatch / 2; ++u) p[u] = s_it[first / 2 + u];
    float4 r[kHubBatch];
#pragma unroll
    for (int u = 0; u < kHubBatch / 2; ++u) {
      r[2 * u] = s_row[p[u].x * w + j];
      r[2 * u + 1] = s_row[p[u].z * w + j];
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < kHubBatch / 2; ++u) {
      fma4(acc, __int_as_float(p[u].y), r[2 * u]);
      fma4(acc, __int_as_float(p[u].w), r[2 * u + 1]);
    }
    s_sum[e] = acc;
  }
  __syncthreads();
  for (int e = tid; e < a.H * w; e += BS) {
    const int t = e / w, j = e - t * w;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int bi = s_off[t]; bi < s_off[t + 1]; ++bi) add4(acc, s_sum[bi * w + j]);
    a.part[((size_t)t * a.G + g) * Q + q0 + j] = acc;
  }
}

// fin2: sum of the G partials only (hub x hub terms are in the partials)
template <int BS>
__device__ void fin2_role(const Args& a, int bb) {
  const int tid = threadIdx.x;
  const int o = bb * (BS / kFinLanes) + tid / kFinLanes, p = tid % kFinLanes;
  const int Q = a.Q;
  const bool ok = o < a.H * Q;
  const int t = ok ? o / Q : 0, j = ok ? o - t * Q : 0;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    float4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int g = p + u * kFinLanes;
      r[u] = g < a.G ? a.part[((size_t)t * a.G + g) * Q + j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) add4(acc, r[u]);
  }
  const float4 bj = ok ? a.bias[j] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int m = kFinLanes / 2; m >= 1; m >>= 1) {
    acc.x += __shfl_xor(acc.x, m); acc.y += __shfl_xor(acc.y, m);
    acc.z += __shfl_xor(acc.z, m); acc.w += __shfl_xor(acc.w, m);
  }
  if (ok && p == 0) a.C[(size_t)(a.h0 + t) * Q + j] = relu_bias(acc, bj);
}

template <int BS, int RPW, int ABL = 0>
__global__ void __launch_bounds__(BS) roles2_kernel(Args a, int nD, int nP) {
  extern __shared__ __attribute__((aligned(16))) float4 smem[];
  stamp(a, 0);
  const int b = blockIdx.x;
  if (b < nD) doc2_role<BS, RPW, ABL>(a, b, smem);
  else if (b < nD + nP) part2_role<BS>(a, b - nD, smem);
  else fin2_role<BS>(a, b - nD - nP);
  stamp(a, 3);
}

// ===========================================================================
// slice3: one workgroup per (row group g, column slice c) computes its doc
// rows' c-slices AND the hub partials of group g over slice c from one LDS
// image (record | rows [(n + 1 + H) x w] | batch sums).  Record (int32):
//   0 n  1 nb  2 o_items  3 -  | doc entries int2 {i | nbatch << 16, first}
//   [n] (degree-sorted) | hub batches int2 {t, first} [nb] | hub batch
//   offsets [H + 1] | items int2 {slot, val}: doc i -> i, zero -> n, hub t -> n+1+t
template <int BS, bool COMB = false>
__device__ void slice3_role(const Args& a, int bb, float4* s) {
  constexpr int NW = BS / 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Q = a.Q;
  const int g = bb % a.G, c = bb / a.G;
  const int q0 = c * Q / a.nslices, q1 = (c + 1) * Q / a.nslices, w = q1 - q0;
  const int l0 = g * a.gs;
  const int n = min(a.gs, a.nL - l0);
  int* s_rec = reinterpret_cast<int*>(s);
  float4* s_row = s + a.R3 / 4;
  if (tid < w) s_row[n * w + tid] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int* rec = a.rec3 + (size_t)g * a.R3;
  for (int k0 = wv * 64; k0 < a.R3 / 4; k0 += BS) {
    const int k = k0 + lane;
    if (k < a.R3 / 4) lds_dma16(rec + 4 * k, s_rec + 4 * k0);
  }
  for (int e0 = wv * 64; e0 < n * w; e0 += BS) {
    const int e = e0 + lane;
    const int i = e / w, j = e - i * w;
    if (e < n * w) lds_dma16(a.B + (size_t)light_row(l0 + i, a.h0, a.H) * Q + q0 + j, s_row + e0);
  }
  float4* s_hubs = s_row + (n + 1) * w;
  for (int e0 = wv * 64; e0 < a.H * w; e0 += BS) {
    const int e = e0 + lane;
    const int t = e / w, j = e - t * w;
    if (e < a.H * w) lds_dma16(a.B + (size_t)(a.h0 + t) * Q + q0 + j, s_hubs + e0);
  }
  const float4 bv = tid < w ? a.bias[q0 + tid] : make_float4(0.f, 0.f, 0.f, 0.f);
  float4* s_bias = s_hubs + a.H * w;  // w vectors
  stamp(a, 1);
  wait_vm0();
  if (tid < w) s_bias[tid] = bv;
  __syncthreads();
  stamp(a, 2);
  const int nb = s_rec[1], o_it = s_rec[2];
  const int2* s_doc = reinterpret_cast<const int2*>(s_rec + 4);
  const int2* s_b = s_doc + n;
  const int* s_off = s_rec + 4 + 2 * n + 2 * nb;
  const int4* s_it = reinterpret_cast<const int4*>(s_rec + o_it);
  float4* s_sum = s_bias + w;
  const int ndt = n * w, ntot = (n + nb) * w;
  for (int e = tid; e < ntot; e += BS) {
    if (e < ndt) {
      const int lo = e / w, j = e - lo * w;
      const int2 de = s_doc[lo];
      const int i = de.x & 0xffff, nbt = de.x >> 16;
      const int4* ip = s_it + de.y / 2;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int bt = 0; bt < nbt; ++bt) {
        const int4 p0 = ip[2 * bt], p1 = ip[2 * bt + 1];
        const float4 r0 = s_row[p0.x * w + j], r1 = s_row[p0.z * w + j], r2 = s_row[p1.x * w + j], r3 = s_row[p1.z * w + j];
        fma4(acc, __int_as_float(p0.y), r0);
        fma4(acc, __int_as_float(p0.w), r1);
        fma4(acc, __int_as_float(p1.y), r2);
        fma4(acc, __int_as_float(p1.w), r3);
      }
      a.C[(size_t)light_row(l0 + i, a.h0, a.H) * Q + q0 + j] = relu_bias(acc, s_bias[j]);
    } else {
      const int eh = e - ndt;
      const int bi = eh / w, j = eh - bi * w;
      const int first = s_b[bi].y;
      int4 p[kHubBatch / 2];
#pragma unroll
      for (int u = 0; u < kHubBatch / 2; ++u) p[u] = s_it[first / 2 + u];
      float4 r[kHubBatch];
#pragma unroll
      for (int u = 0; u < kHubBatch / 2; ++u) {
        r[2 * u] = s_row[p[u].x * w + j];
        r[2 * u + 1] = s_row[p[u].z * w + j];
      }
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < kHubBatch / 2; ++u) {
        fma4(acc, __int_as_float(p[u].y), r[2 * u]);
        fma4(acc, __int_as_float(p[u].w), r[2 * u + 1]);
      }
      s_sum[eh] = acc;
    }
  }
  __syncthreads();
  for (int e = tid; e < a.H * w; e += BS) {
    const int t = e / w, j = e - t * w;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int bi = s_off[t]; bi < s_off[t + 1]; ++bi) add4(acc, s_sum[bi * w + j]);
    if (COMB) st_sc1(a.part, (int)((((size_t)t * a.G + g) * Q + q0 + j) * 16), acc);
    else a.part[((size_t)t * a.G + g) * Q + q0 + j] = acc;
  }
}

// ===========================================================================
// slice3c: slice3 + in-launch combine by the last arriver of each slice
template <int BS>
__device__ void slice3c_tail(const Args& a, int bb, float4* s) {
  // partials were stored sc1 by slice3_role (COMB) -> drain, count in, last arriver combines
  const int tid = threadIdx.x;
  const int Q = a.Q;
  const int c = bb / a.G;
  const int q0 = c * Q / a.nslices, q1 = (c + 1) * Q / a.nslices, w = q1 - q0;
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  __shared__ int s_last;
  if (tid == 0) {
    const unsigned long long old = __hip_atomic_fetch_add(a.ctr + c, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (int)((old + 1) % (unsigned long long)a.G == 0);
  }
  __syncthreads();
  if (!s_last) return;
  stamp(a, 2);
  const float* pb = reinterpret_cast<const float*>(__builtin_amdgcn_readfirstlane(0) == 0 ? a.part : a.part);
  constexpr int PL = 4;
  for (int o0 = 0; o0 < a.H * w; o0 += BS / PL) {
    const int o = o0 + tid / PL, p = tid % PL;
    const bool ok = o < a.H * w;
    const int t = ok ? o / w : 0, j = ok ? o - t * w : 0;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 r[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int g = p * 16 + u;  // G <= 64
      r[u] = (ok && g < a.G) ? ld_sc1(pb, (int)((((size_t)t * a.G + g) * Q + q0 + j) * 16)) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) add4(acc, r[u]);
#pragma unroll
    for (int m = 1; m < PL; m <<= 1) {
      acc.x += __shfl_xor(acc.x, m); acc.y += __shfl_xor(acc.y, m);
      acc.z += __shfl_xor(acc.z, m); acc.w += __shfl_xor(acc.w, m);
    }
    if (ok && p == 0) a.C[(size_t)(a.h0 + t) * Q + q0 + j] = relu_bias(acc, a.bias[q0 + j]);
  }
  (void)s;
}

template <int BS>
__global__ void __launch_bounds__(BS) slice3_kernel(Args a, int nS) {
  extern __shared__ __attribute__((aligned(16))) float4 smem[];
  stamp(a, 0);
  if ((int)blockIdx.x < nS) slice3_role<BS>(a, blockIdx.x, smem);
  else fin2_role<BS>(a, blockIdx.x - nS);
  stamp(a, 3);
}

template <int BS>
__global__ void __launch_bounds__(BS) slice3c_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) float4 smem[];
  stamp(a, 0);
  slice3_role<BS, true>(a, blockIdx.x, smem);
  stamp(a, 1);
  slice3c_tail<BS>(a, blockIdx.x, smem);
  stamp(a, 3);
}

// ===========================================================================
// Pull roles with no LDS staging and no hand-off: docP = one light row per
// wavefront (ELL-16 items, gathers straight from L1/L2, one store at the
// end); topP = one (hub row, column slice) per workgroup, 32 lane groups of 8
// taking interleaved nonzeros, fixed-order LDS tree.
constexpr int kEll = 16;
template <int BS>
__device__ void docP_role(const Args& a, int b) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = b * NW + wv;
  if (l >= a.nL) return;
  const int Q = a.Q;
  const int row = light_row(l, a.h0, a.H);
  const int2 it = a.ell[(size_t)l * kEll + (lane & (kEll - 1))];
  const int ql = min(lane, Q - 1);
  const float4 self = a.B[(size_t)row * Q + ql];
  const float4 bv = a.bias[ql];
  const int n = __builtin_popcountll(__ballot(lane < kEll && it.y != 0)) ;
  float4 r[kEll];
  float w[kEll];
#pragma unroll
  for (int k = 0; k < kEll; ++k) {
    if (k < n) {
      const int c = rl(it.x, k);
      w[k] = __int_as_float(rl(it.y, k));
      if (c >= 0) r[k] = a.B[(size_t)c * Q + ql];
      else r[k] = self;
    }
  }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < kEll; ++k)
    if (k < n) fma4(acc, w[k], r[k]);
  if (lane < Q) a.C[(size_t)row * Q + lane] = relu_bias(acc, bv);
}

constexpr int kTopUB = 16;  // items per lane group in flight
template <int BS>
__device__ void topP_role(const Args& a, int bb, float4* s) {
  constexpr int NG = BS / 8;
  const int tid = threadIdx.x, gi = tid >> 3, j = tid & 7;
  const int Q = a.Q;
  const int t = bb / a.nslices, c = bb % a.nslices;
  const int q0 = c * Q / a.nslices, q1 = (c + 1) * Q / a.nslices, w = q1 - q0;
  const int r = a.h0 + t;
  const int k0 = a.rp[r], k1 = a.rp[r + 1];
  const int jj = min(j, w - 1);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int kb = k0; kb < k1; kb += NG * kTopUB) {
    int cc[kTopUB];
    float vv[kTopUB];
#pragma unroll
    for (int u = 0; u < kTopUB; ++u) {
      const int k = kb + gi + u * NG;
      cc[u] = k < k1 ? a.ci[k] : a.h0;
      vv[u] = k < k1 ? a.v[k] : 0.f;
    }
    float4 g[kTopUB];
#pragma unroll
    for (int u = 0; u < kTopUB; ++u) g[u] = a.B[(size_t)cc[u] * Q + q0 + jj];
#pragma unroll
    for (int u = 0; u < kTopUB; ++u) fma4(acc, vv[u], g[u]);
  }
  s[tid] = acc;
  __syncthreads();
  for (int m = NG / 2; m >= 1; m >>= 1) {
    if (gi < m) add4(s[tid], s[tid + 8 * m]);
    __syncthreads();
  }
  if (gi == 0 && j < w) a.C[(size_t)r * Q + q0 + j] = relu_bias(s[tid], a.bias[q0 + j]);
}

// [0, nT) topic units first (the long ones dispatched first), then doc rows
template <int BS>
__global__ void __launch_bounds__(BS) pull_kernel(Args a, int nT, int nD) {
  __shared__ float4 s_red[BS];
  stamp(a, 0);
  const int b = blockIdx.x;
  if (b < nT) topP_role<BS>(a, b, s_red);
  else docP_role<BS>(a, b - nT);
  stamp(a, 3);
}

__global__ void copy_kernel(const float4* __restrict__ a, float4* __restrict__ b, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) b[i] = a[i];
}

// ---------------------------------------------------------------------------
struct Csr {
  int M = 0, nnz = 0;
  std::vector<int> rp, ci;
  std::vector<float> v;
};

static Csr read_csr(const char* path) {
  Csr c;
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(2); }
  int hdr[2];
  if (fread(hdr, 4, 2, f) != 2) exit(2);
  c.M = hdr[0]; c.nnz = hdr[1];
  c.rp.resize(c.M + 1); c.ci.resize(c.nnz); c.v.resize(c.nnz);
  if (fread(c.rp.data(), 4, c.M + 1, f) != (size_t)c.M + 1) exit(2);
  if (fread(c.ci.data(), 4, c.nnz, f) != (size_t)c.nnz) exit(2);
  if (fread(c.v.data(), 4, c.nnz, f) != (size_t)c.nnz) exit(2);
  fclose(f);
  return c;
}

static int light_row_h(int l, int h0, int H) { return l < h0 ? l : l + H; }
struct HostPlan {
  int h0, H, nL, G, gs, R, R2 = 0, max_nb2 = 0, R3 = 0, max_nb3 = 0;
  std::vector<int> rec, hh_rp, rec2, rec3;
  std::vector<int2> hh, win;
};

// part2 records: hub t's nonzeros over group g's rows (slot i), plus, in group
// t % G, its hub x hub nonzeros (slot n + 1 + t'); slot n = the zero row
static void build_rec2(const Csr& A, HostPlan& P) {
  const int h0 = P.h0, H = P.H, G = P.G;
  auto is_hub = [&](int c) { return c >= h0 && c < h0 + H; };
  auto lidx = [&](int c) { return c < h0 ? c : c - H; };
  std::vector<std::vector<std::vector<std::pair<int, float>>>> items(G, std::vector<std::vector<std::pair<int, float>>>(H));
  for (int t = 0; t < H; ++t) {
    const int r = h0 + t;
    for (int k = A.rp[r]; k < A.rp[r + 1]; ++k) {
      const int c = A.ci[k];
      if (is_hub(c)) {
        const int g = t % G, n = std::min(P.gs, P.nL - g * P.gs);
        items[g][t].push_back({n + 1 + (c - h0), A.v[k]});
      } else {
        const int l = lidx(c), g = l / P.gs;
        items[g][t].push_back({l - g * P.gs, A.v[k]});
      }
    }
  }
  std::vector<std::vector<int>> recs(G);
  int R = 0;
  for (int g = 0; g < G; ++g) {
    const int n = std::min(P.gs, P.nL - g * P.gs);
    std::vector<int2> bt, its;
    std::vector<int> off(H + 1, 0);
    for (int t = 0; t < H; ++t) {
      off[t] = (int)bt.size();
      auto& L = items[g][t];
      for (size_t q = 0; q < L.size(); ++q) {
        if (q % kHubBatch == 0) bt.push_back(make_int2(t, (int)its.size()));
        its.push_back(make_int2(L[q].first, __builtin_bit_cast(int, L[q].second)));
      }
      while (its.size() % kHubBatch) its.push_back(make_int2(n, 0));
    }
    off[H] = (int)bt.size();
    const int nb = (int)bt.size();
    P.max_nb2 = std::max(P.max_nb2, nb);
    const int o_it = (4 + 2 * nb + H + 1 + 3) & ~3;
    std::vector<int>& w = recs[g];
    w.assign(o_it + 2 * its.size(), 0);
    w[0] = n; w[1] = nb; w[2] = o_it;
    for (int b = 0; b < nb; ++b) { w[4 + 2 * b] = bt[b].x; w[5 + 2 * b] = bt[b].y; }
    for (int t = 0; t <= H; ++t) w[4 + 2 * nb + t] = off[t];
    for (size_t i = 0; i < its.size(); ++i) { w[o_it + 2 * i] = its[i].x; w[o_it + 2 * i + 1] = its[i].y; }
    R = std::max(R, (int)w.size());
  }
  P.R2 = (R + 3) & ~3;
  P.rec2.assign((size_t)G * P.R2, 0);
  for (int g = 0; g < G; ++g) std::copy(recs[g].begin(), recs[g].end(), P.rec2.begin() + (size_t)g * P.R2);
}

// slice3 records: rec2's hub part plus degree-sorted doc entries (items padded to 4)
static void build_rec3(const Csr& A, HostPlan& P) {
  const int G = P.G, H = P.H;
  std::vector<std::vector<int>> recs(G);
  int R = 0;
  P.max_nb3 = 0;
  for (int g = 0; g < G; ++g) {
    const int* r2 = P.rec2.data() + (size_t)g * P.R2;
    const int n = r2[0], nb = r2[1], o2 = r2[2];
    std::vector<int> ord(n);
    for (int i = 0; i < n; ++i) ord[i] = i;
    auto deg = [&](int i) { const int r = light_row_h(g * P.gs + i, P.h0, H); return A.rp[r + 1] - A.rp[r]; };
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return deg(x) > deg(y); });
    std::vector<int2> its, ents(n);
    for (int lo = 0; lo < n; ++lo) {
      const int i = ord[lo], r = light_row_h(g * P.gs + i, P.h0, H);
      const int first = (int)its.size();
      for (int k = A.rp[r]; k < A.rp[r + 1]; ++k) {
        const int cc = A.ci[k];
        its.push_back(make_int2(cc == r ? i : n + 1 + (cc - P.h0), __builtin_bit_cast(int, A.v[k])));
      }
      while ((its.size() - first) % 4) its.push_back(make_int2(n, 0));
      ents[lo] = make_int2(i | (int)(((its.size() - first) / 4) << 16), first);
    }
    // hub items from rec2 (their slots are already n-based), re-based after the doc items
    const int hub_first = (int)its.size();
    const int nhit = (int)((P.R2 - o2) / 2);
    int last = 0;
    for (int b = 0; b < nb; ++b) last = std::max(last, r2[5 + 2 * b] + kHubBatch);
    for (int q = 0; q < last; ++q) its.push_back(make_int2(r2[o2 + 2 * q], r2[o2 + 2 * q + 1]));
    (void)nhit;
    const int o_it = (4 + 2 * n + 2 * nb + H + 1 + 3) & ~3;
    std::vector<int>& w = recs[g];
    w.assign(o_it + 2 * its.size(), 0);
    w[0] = n; w[1] = nb; w[2] = o_it;
    for (int lo = 0; lo < n; ++lo) { w[4 + 2 * lo] = ents[lo].x; w[5 + 2 * lo] = ents[lo].y; }
    for (int b = 0; b < nb; ++b) { w[4 + 2 * n + 2 * b] = r2[4 + 2 * b]; w[5 + 2 * n + 2 * b] = r2[5 + 2 * b] + hub_first; }
    for (int t = 0; t <= H; ++t) w[4 + 2 * n + 2 * nb + t] = r2[4 + 2 * nb + t];
    for (size_t i = 0; i < its.size(); ++i) { w[o_it + 2 * i] = its[i].x; w[o_it + 2 * i + 1] = its[i].y; }
    R = std::max(R, (int)w.size());
    P.max_nb3 = std::max(P.max_nb3, nb);
  }
  P.R3 = (R + 3) & ~3;
  P.rec3.assign((size_t)G * P.R3, 0);
  for (int g = 0; g < G; ++g) std::copy(recs[g].begin(), recs[g].end(), P.rec3.begin() + (size_t)g * P.R3);
}

// doc2 windows: wave w = light rows [w * rpw, ...): items {(k << 8) | slot, val},
// slot = hub index or kSelfSlot; padding row 255
static int build_windows(const Csr& A, HostPlan& P, int rpw) {
  const int nw = (P.nL + rpw - 1) / rpw;
  P.win.assign((size_t)nw * kWin, make_int2(0xff00, 0));
  int maxi = 0;
  for (int w = 0; w < nw; ++w) {
    int n = 0;
    for (int k = 0; k < rpw && w * rpw + k < P.nL; ++k) {
      const int l = w * rpw + k, r = l < P.h0 ? l : l + P.H;
      for (int q = A.rp[r]; q < A.rp[r + 1]; ++q) {
        const int c = A.ci[q];
        const int slot = c == r ? kSelfSlot : c - P.h0;
        if (n < kWin) P.win[(size_t)w * kWin + n] = make_int2((k << 8) | slot, __builtin_bit_cast(int, A.v[q]));
        ++n;
      }
    }
    maxi = std::max(maxi, n);
  }
  return maxi;
}

static HostPlan build_plan(const Csr& A, int G) {
  HostPlan P{};
  int h0 = -1, h1 = -1;
  for (int r = 0; r < A.M; ++r)
    if (A.rp[r + 1] - A.rp[r] >= 64) { if (h0 < 0) h0 = r; h1 = r + 1; }
  P.h0 = h0; P.H = h1 - h0; P.nL = A.M - P.H; P.G = G;
  P.gs = (P.nL + G - 1) / G;
  auto is_hub = [&](int c) { return c >= h0 && c < h1; };
  auto lidx = [&](int c) { return c < h0 ? c : c - P.H; };
  for (int l = 0; l < P.nL; ++l) {
    const int r = l < h0 ? l : l + P.H;
    for (int k = A.rp[r]; k < A.rp[r + 1]; ++k)
      if (!is_hub(A.ci[k]) && A.ci[k] != r) { fprintf(stderr, "not a hub graph\n"); exit(2); }
  }
  P.hh_rp.assign(P.H + 1, 0);
  std::vector<std::vector<std::vector<std::pair<int, float>>>> items(G, std::vector<std::vector<std::pair<int, float>>>(P.H));
  for (int t = 0; t < P.H; ++t) {
    const int r = h0 + t;
    for (int k = A.rp[r]; k < A.rp[r + 1]; ++k) {
      const int c = A.ci[k];
      if (is_hub(c)) { P.hh.push_back(make_int2(c - h0, __builtin_bit_cast(int, A.v[k]))); continue; }
      const int l = lidx(c), g = l / P.gs;
      items[g][t].push_back({l - g * P.gs, A.v[k]});
    }
    P.hh_rp[t + 1] = (int)P.hh.size();
  }
  std::vector<std::vector<int>> recs(G);
  int R = 0;
  for (int g = 0; g < G; ++g) {
    const int n = std::min(P.gs, P.nL - g * P.gs);
    std::vector<int2> bt;  // {t, first}
    std::vector<int> off(P.H + 1, 0);
    std::vector<int2> its;
    for (int t = 0; t < P.H; ++t) {
      off[t] = (int)bt.size();
      auto& L = items[g][t];
      for (size_t q = 0; q < L.size(); ++q) {
        if (q % kHubBatch == 0) bt.push_back(make_int2(t, (int)its.size()));
        its.push_back(make_int2(L[q].first, __builtin_bit_cast(int, L[q].second)));
      }
      while (its.size() % kHubBatch) its.push_back(make_int2(n, 0));
    }
    off[P.H] = (int)bt.size();
    const int nb = (int)bt.size();
    int o_it = 4 + 2 * nb + P.H + 1;
    o_it = (o_it + 3) & ~3;
    std::vector<int>& w = recs[g];
    w.assign(o_it + 2 * its.size(), 0);
    w[0] = n; w[1] = nb; w[2] = o_it;
    for (int b = 0; b < nb; ++b) { w[4 + 2 * b] = bt[b].x; w[5 + 2 * b] = bt[b].y; }
    for (int t = 0; t <= P.H; ++t) w[4 + 2 * nb + t] = off[t];
    for (size_t i = 0; i < its.size(); ++i) { w[o_it + 2 * i] = its[i].x; w[o_it + 2 * i + 1] = its[i].y; }
    R = std::max(R, (int)w.size());
  }
  R = (R + 3) & ~3;
  P.R = R;
  P.rec.assign((size_t)G * R, 0);
  for (int g = 0; g < G; ++g) std::copy(recs[g].begin(), recs[g].end(), P.rec.begin() + (size_t)g * R);
  return P;
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/tmp/r8_adj.bin";
  const int G = argc > 2 ? atoi(argv[2]) : 32;
  const int nslices = argc > 3 ? atoi(argv[3]) : 7;
  const Csr A = read_csr(path);
  const int F = 200, Q = F / 4, M = A.M;
  HostPlan P = build_plan(A, G);
  build_rec2(A, P);
  build_rec3(A, P);
  constexpr int RPW2 = 4;
  const int max_win = build_windows(A, P, RPW2);
  if (max_win > kWin) { fprintf(stderr, "doc2 window %d > %d items\n", max_win, kWin); return 2; }
  constexpr int RPW = 8;
  // per-wave item capacity and contiguity of each wave's rows
  int max_items = 0;
  for (int l0 = 0; l0 < P.nL; l0 += RPW) {
    const int nr = std::min(RPW, P.nL - l0);
    const int r0 = l0 < P.h0 ? l0 : l0 + P.H;
    const int rl = (l0 + nr - 1) < P.h0 ? l0 + nr - 1 : l0 + nr - 1 + P.H;
    if (rl - r0 != nr - 1) { fprintf(stderr, "wave rows straddle the hub range\n"); return 2; }
    max_items = std::max(max_items, A.rp[r0 + nr] - A.rp[r0]);
  }
  if (max_items > 128) { fprintf(stderr, "wave items %d > 128\n", max_items); return 2; }
  const int nD = (P.nL + 4 * RPW - 1) / (4 * RPW);
  const int nP = G * nslices;
  const int nF = (P.H * Q * kFinLanes + kBlock - 1) / kBlock;
  const int wmax = (Q + nslices - 1) / nslices;
  int max_nb = 0;
  for (int g = 0; g < G; ++g) max_nb = std::max(max_nb, P.rec[(size_t)g * P.R + 1]);
  const size_t lds_doc = (size_t)(P.H * Q + 4 * RPW * Q + 64) * 16;
  const size_t lds_part = (size_t)P.R * 4 + (size_t)((P.gs + 1) * wmax + max_nb * wmax) * 16;
  printf("{\"M\": %d, \"nnz\": %d, \"h0\": %d, \"H\": %d, \"G\": %d, \"gs\": %d, \"slices\": %d, \"R\": %d, \"nD\": %d, \"nP\": %d, "
         "\"nF\": %d, \"max_wave_items\": %d, \"lds_doc\": %zu, \"lds_part\": %zu, \"part_MB\": %.3f}\n",
         M, A.nnz, P.h0, P.H, G, P.gs, nslices, P.R, nD, nP, nF, max_items, lds_doc, lds_part,
         (double)P.H * G * Q * 16 / 1e6);
  if (lds_doc > 160 * 1024 || lds_part > 160 * 1024) { fprintf(stderr, "LDS too big\n"); return 2; }

  // device data
  int *d_rp, *d_ci, *d_rec, *d_hhrp;
  float* d_v;
  int2* d_hh;
  CHECK(hipMalloc(&d_rp, (M + 1) * 4));
  CHECK(hipMalloc(&d_ci, A.nnz * 4));
  CHECK(hipMalloc(&d_v, A.nnz * 4));
  CHECK(hipMalloc(&d_rec, P.rec.size() * 4));
  CHECK(hipMalloc(&d_hhrp, (P.H + 1) * 4));
  CHECK(hipMalloc(&d_hh, std::max<size_t>(1, P.hh.size()) * 8));
  CHECK(hipMemcpy(d_rp, A.rp.data(), (M + 1) * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_ci, A.ci.data(), A.nnz * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_v, A.v.data(), A.nnz * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_rec, P.rec.data(), P.rec.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_hhrp, P.hh_rp.data(), (P.H + 1) * 4, hipMemcpyHostToDevice));
  // docP ELL-16
  std::vector<int2> ell((size_t)P.nL * kEll, make_int2(P.h0, 0));
  int max_deg = 0;
  for (int l = 0; l < P.nL; ++l) {
    const int r = l < P.h0 ? l : l + P.H;
    max_deg = std::max(max_deg, A.rp[r + 1] - A.rp[r]);
    for (int k = A.rp[r], q = 0; k < A.rp[r + 1] && q < kEll; ++k, ++q)
      ell[(size_t)l * kEll + q] = make_int2(A.ci[k] == r ? -1 : A.ci[k], __builtin_bit_cast(int, A.v[k]));
  }
  if (max_deg > kEll) { fprintf(stderr, "light degree %d > %d\n", max_deg, kEll); return 2; }
  int2* d_ell;
  CHECK(hipMalloc(&d_ell, ell.size() * 8));
  CHECK(hipMemcpy(d_ell, ell.data(), ell.size() * 8, hipMemcpyHostToDevice));
  int* d_rec3;
  CHECK(hipMalloc(&d_rec3, P.rec3.size() * 4));
  CHECK(hipMemcpy(d_rec3, P.rec3.data(), P.rec3.size() * 4, hipMemcpyHostToDevice));
  int* d_rec2;
  int2* d_win;
  CHECK(hipMalloc(&d_rec2, P.rec2.size() * 4));
  CHECK(hipMalloc(&d_win, P.win.size() * 8));
  CHECK(hipMemcpy(d_rec2, P.rec2.data(), P.rec2.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_win, P.win.data(), P.win.size() * 8, hipMemcpyHostToDevice));
  if (!P.hh.empty()) CHECK(hipMemcpy(d_hh, P.hh.data(), P.hh.size() * 8, hipMemcpyHostToDevice));
  const size_t mat = (size_t)M * F;
  const int nsets = std::max(2, (int)(320e6 / (8.0 * mat)) + 1);
  std::vector<float*> Bs(nsets), Cs(nsets);
  std::vector<float> hB(mat), hbias(F);
  srand(1);
  for (auto& x : hbias) x = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
  for (int s = 0; s < nsets; ++s) {
    for (auto& x : hB) x = rand() / (float)RAND_MAX - 0.5f;
    CHECK(hipMalloc(&Bs[s], mat * 4));
    CHECK(hipMalloc(&Cs[s], mat * 4));
    CHECK(hipMemcpy(Bs[s], hB.data(), mat * 4, hipMemcpyHostToDevice));
  }
  // reference for set 0
  CHECK(hipMemcpy(hB.data(), Bs[0], mat * 4, hipMemcpyDeviceToHost));
  std::vector<double> ref(mat);
  for (int r = 0; r < M; ++r)
    for (int f = 0; f < F; ++f) {
      double acc = 0;
      for (int k = A.rp[r]; k < A.rp[r + 1]; ++k) acc += (double)A.v[k] * hB[(size_t)A.ci[k] * F + f];
      ref[(size_t)r * F + f] = std::max(0.0, acc + hbias[f]);
    }
  float *d_bias, *d_part;
  CHECK(hipMalloc(&d_bias, F * 4));
  CHECK(hipMemcpy(d_bias, hbias.data(), F * 4, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&d_part, (size_t)P.H * G * Q * 16));
  unsigned long long* d_st;
  const int maxwg = 4 * (nD + nP + nF) + 1024;
  CHECK(hipMalloc(&d_st, (size_t)65536 * 32));

  CHECK(hipFuncSetAttribute((const void*)&roles2_kernel<256, RPW2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHECK(hipFuncSetAttribute((const void*)&roles2_kernel<512, RPW2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHECK(hipFuncSetAttribute((const void*)&roles_kernel<RPW, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHECK(hipFuncSetAttribute((const void*)&roles_kernel<RPW, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHECK(hipFuncSetAttribute((const void*)&roles_kernel<RPW, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  auto args = [&](int s) {
    Args a{};
    a.rp = d_rp; a.ci = d_ci; a.v = d_v;
    a.B = reinterpret_cast<const float4*>(Bs[s]); a.C = reinterpret_cast<float4*>(Cs[s]);
    a.bias = reinterpret_cast<const float4*>(d_bias);
    a.M = M; a.Q = Q; a.h0 = P.h0; a.H = P.H; a.nL = P.nL;
    a.rpw = RPW; a.nD = nD;
    a.rec = d_rec; a.R = P.R; a.G = G; a.gs = P.gs; a.nslices = nslices; a.part = reinterpret_cast<float4*>(d_part);
    a.hh_rp = d_hhrp; a.hh = d_hh;
    a.win = d_win; a.rec2 = d_rec2; a.R2 = P.R2;
    a.rec3 = d_rec3; a.R3 = P.R3;
    a.ell = d_ell;
    return a;
  };
  const size_t lds_doc_noself = (size_t)(P.H * Q + 64) * 16;
  auto launch = [&](int s, int dv, int d, int p, int f, unsigned long long* stamps = nullptr) {
    Args a = args(s);
    a.stamps = stamps;
    size_t lds = 0;
    if (d) lds = dv == 0 ? lds_doc : dv == 2 ? lds_doc_noself : 0;
    if (p) lds = std::max(lds, lds_part);
    if (dv == 0) hipLaunchKernelGGL((roles_kernel<RPW, 0>), dim3(d + p + f), dim3(kBlock), lds, st, a, d, p);
    if (dv == 1) hipLaunchKernelGGL((roles_kernel<RPW, 1>), dim3(d + p + f), dim3(kBlock), lds, st, a, d, p);
    if (dv == 2) hipLaunchKernelGGL((roles_kernel<RPW, 2>), dim3(d + p + f), dim3(kBlock), lds, st, a, d, p);
  };
  const size_t lds_doc2 = (size_t)P.H * Q * 16;
  const size_t lds_part2 = (size_t)P.R2 * 4 + (size_t)((P.gs + 1 + P.H) * wmax + P.max_nb2 * wmax) * 16;
  const int nD2_256 = (P.nL + 4 * RPW2 - 1) / (4 * RPW2), nD2_512 = (P.nL + 8 * RPW2 - 1) / (8 * RPW2);
  const int nF2_256 = (P.H * Q * kFinLanes + 255) / 256, nF2_512 = (P.H * Q * kFinLanes + 511) / 512;
  printf("{\"lds_doc2\": %zu, \"lds_part2\": %zu, \"max_win\": %d, \"nD2_256\": %d, \"nD2_512\": %d}\n", lds_doc2, lds_part2, max_win, nD2_256, nD2_512);
  if (lds_part2 > 160 * 1024) { fprintf(stderr, "part2 LDS too big\n"); return 2; }
  // v2 launch: dv = -256 / -512 selects roles2_kernel<BS>
  auto launch2 = [&](int s, int bs, int d, int p, int f, unsigned long long* stamps = nullptr) {
    Args a = args(s);
    a.stamps = stamps;
    size_t lds = 0;
    if (d) lds = lds_doc2;
    if (p) lds = std::max(lds, lds_part2);
    if (bs == 256) hipLaunchKernelGGL((roles2_kernel<256, RPW2>), dim3(d + p + f), dim3(256), lds, st, a, d, p);
    else hipLaunchKernelGGL((roles2_kernel<512, RPW2>), dim3(d + p + f), dim3(512), lds, st, a, d, p);
  };
  const size_t lds_s3 = (size_t)P.R3 * 4 + (size_t)((P.gs + 1 + P.H + 1) * wmax + P.max_nb3 * wmax) * 16;
  printf("{\"lds_slice3\": %zu, \"R3\": %d}\n", lds_s3, P.R3);
  if (lds_s3 > 160 * 1024) { fprintf(stderr, "slice3 LDS too big\n"); return 2; }
  CHECK(hipFuncSetAttribute((const void*)&slice3_kernel<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHECK(hipFuncSetAttribute((const void*)&slice3_kernel<512>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const int nF2_1024 = (P.H * Q * kFinLanes + 1023) / 1024;
  auto launch3 = [&](int s, int bs, int ns, int nf, unsigned long long* stamps = nullptr) {
    Args a = args(s);
    a.stamps = stamps;
    const size_t lds = ns ? lds_s3 : 0;
    if (bs == 1024) hipLaunchKernelGGL((slice3_kernel<1024>), dim3(ns + nf), dim3(1024), lds, st, a, ns);
    else hipLaunchKernelGGL((slice3_kernel<512>), dim3(ns + nf), dim3(512), lds, st, a, ns);
  };
  CHECK(hipFuncSetAttribute((const void*)&roles2_kernel<512, RPW2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHECK(hipFuncSetAttribute((const void*)&roles2_kernel<512, RPW2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHECK(hipFuncSetAttribute((const void*)&roles2_kernel<512, RPW2, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHECK(hipFuncSetAttribute((const void*)&roles2_kernel<512, RPW2, 6>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  auto launchA = [&](int s, int abl, unsigned long long* stamps = nullptr) {
    Args a = args(s);
    a.stamps = stamps;
    const int d = nD2_512;
    if (abl == 1) hipLaunchKernelGGL((roles2_kernel<512, RPW2, 1>), dim3(d), dim3(512), lds_doc2, st, a, d, 0);
    if (abl == 2) hipLaunchKernelGGL((roles2_kernel<512, RPW2, 2>), dim3(d), dim3(512), lds_doc2, st, a, d, 0);
    if (abl == 4) hipLaunchKernelGGL((roles2_kernel<512, RPW2, 4>), dim3(d), dim3(512), lds_doc2, st, a, d, 0);
    if (abl == 6) hipLaunchKernelGGL((roles2_kernel<512, RPW2, 6>), dim3(d), dim3(512), lds_doc2, st, a, d, 0);
  };
  unsigned long long* d_ctr;
  CHECK(hipMalloc(&d_ctr, 64 * 8));
  CHECK(hipMemset(d_ctr, 0, 64 * 8));
  CHECK(hipFuncSetAttribute((const void*)&slice3c_kernel<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 256));
  auto launchC = [&](int s, unsigned long long* stamps = nullptr) {
    Args a = args(s);
    a.stamps = stamps;
    a.ctr = d_ctr;
    hipLaunchKernelGGL((slice3c_kernel<1024>), dim3(nP), dim3(1024), lds_s3, st, a);
  };
  auto launchP = [&](int s, int nT, int nDw, unsigned long long* stamps = nullptr) {
    Args a = args(s);
    a.stamps = stamps;
    hipLaunchKernelGGL((pull_kernel<256>), dim3(nT + nDw), dim3(256), 0, st, a, nT, nDw);
  };
  const int nTP = P.H * nslices, nDP = (P.nL + 3) / 4;
  struct Variant { std::string name; std::function<void(int)> run; bool docs, hubs; int dv, d, p, f; };
  std::vector<Variant> vs = {
      {"copy", [&](int s) { hipLaunchKernelGGL(copy_kernel, dim3(1024), dim3(256), 0, st, (const float4*)Bs[s], (float4*)Cs[s], (int)(mat / 4)); }, false, false, -1, 0, 0, 0},
      {"slice3c (one launch, last-arriver combine)", [&](int s) { launchC(s); }, true, true, -4001, nP, 0, 0},
      {"pull docs", [&](int s) { launchP(s, 0, nDP); }, true, false, -3001, 0, nDP, 0},
      {"pull topics", [&](int s) { launchP(s, nTP, 0); }, false, true, -3002, nTP, 0, 0},
      {"pull all (one launch)", [&](int s) { launchP(s, nTP, nDP); }, true, true, -3003, nTP, nDP, 0},
      {"slice3_1024", [&](int s) { launch3(s, 1024, nP, 0); }, true, false, -1024, nP, 0, 0},
      {"slice3_512", [&](int s) { launch3(s, 512, nP, 0); }, true, false, -1025, nP, 0, 0},
      {"s3_1024 | fin2", [&](int s) { launch3(s, 1024, nP, 0); launch3(s, 1024, 0, nF2_1024); }, true, true, -9, 0, 0, 0},
      {"s3_512 | fin2", [&](int s) { launch3(s, 512, nP, 0); launch2(s, 256, 0, 0, nF2_256); }, true, true, -9, 0, 0, 0},
      {"doc2_256", [&](int s) { launch2(s, 256, nD2_256, 0, 0); }, true, false, -256, nD2_256, 0, 0},
      {"doc2_512 abl1 (no hub staging)", [&](int s) { launchA(s, 1); }, false, false, -2001, nD2_512, 0, 0},
      {"doc2_512 abl2 (no compute)", [&](int s) { launchA(s, 2); }, false, false, -2002, nD2_512, 0, 0},
      {"doc2_512 abl4 (no stores)", [&](int s) { launchA(s, 4); }, false, false, -2004, nD2_512, 0, 0},
      {"doc2_512 abl6 (no compute, no stores)", [&](int s) { launchA(s, 6); }, false, false, -2006, nD2_512, 0, 0},
      {"doc2_512", [&](int s) { launch2(s, 512, nD2_512, 0, 0); }, true, false, -512, nD2_512, 0, 0},
      {"part2_256", [&](int s) { launch2(s, 256, 0, nP, 0); }, false, false, -256, 0, nP, 0},
      {"fin2_256", [&](int s) { launch2(s, 256, 0, 0, nF2_256); }, false, false, -256, 0, 0, nF2_256},
      {"v2_256: doc2+part2 | fin2", [&](int s) { launch2(s, 256, nD2_256, nP, 0); launch2(s, 256, 0, 0, nF2_256); }, true, true, -9, 0, 0, 0},
      {"v2_512: doc2+part2 | fin2", [&](int s) { launch2(s, 512, nD2_512, nP, 0); launch2(s, 512, 0, 0, nF2_512); }, true, true, -9, 0, 0, 0},
      {"v2_256: part2 | doc2+fin2", [&](int s) { launch2(s, 256, 0, nP, 0); launch2(s, 256, nD2_256, 0, nF2_256); }, true, true, -9, 0, 0, 0},
      {"doc_lds", [&](int s) { launch(s, 0, nD, 0, 0); }, true, false, 0, nD, 0, 0},
      {"part_only", [&](int s) { launch(s, 1, 0, nP, 0); }, false, false, 1, 0, nP, 0},
      {"fin_only", [&](int s) { launch(s, 1, 0, 0, nF); }, false, false, 1, 0, 0, nF},
  };
  auto pct = [](std::vector<double> x, double q) { std::sort(x.begin(), x.end()); return x.empty() ? 0.0 : x[(size_t)(q * (x.size() - 1))]; };
  std::vector<float> out(mat);
  for (auto& V : vs) {
    CHECK(hipMemset(Cs[0], 0, mat * 4));
    V.run(0);
    CHECK(hipStreamSynchronize(st));
    CHECK(hipGetLastError());
    double maxerr = 0;
    if (V.docs || V.hubs) {
      CHECK(hipMemcpy(out.data(), Cs[0], mat * 4, hipMemcpyDeviceToHost));
      for (int r = 0; r < M; ++r) {
        const bool hub = r >= P.h0 && r < P.h0 + P.H;
        if ((hub && !V.hubs) || (!hub && !V.docs)) continue;
        for (int f = 0; f < F; ++f) {
          const double e = std::fabs(out[(size_t)r * F + f] - ref[(size_t)r * F + f]) / (1.0 + std::fabs(ref[(size_t)r * F + f]));
          maxerr = std::max(maxerr, e);
        }
      }
    }
    double us[2];
    for (int mode = 0; mode < 2; ++mode) {
      const int reps = mode == 0 ? std::max(1, 200 / nsets) : 1;
      const int per = mode == 0 ? nsets : 200;
      hipGraph_t gr;
      hipGraphExec_t ge;
      CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int r = 0; r < reps; ++r)
        for (int s = 0; s < per; ++s) V.run(mode == 0 ? s : 0);
      CHECK(hipStreamEndCapture(st, &gr));
      CHECK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
      CHECK(hipGraphLaunch(ge, st));
      CHECK(hipStreamSynchronize(st));
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0));
      CHECK(hipEventCreate(&e1));
      CHECK(hipEventRecord(e0, st));
      CHECK(hipGraphLaunch(ge, st));
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      us[mode] = ms * 1e3 / (reps * per);
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(gr));
    }
    printf("{\"variant\": \"%s\", \"cold_us\": %.3f, \"warm_us\": %.3f, \"maxerr\": %.3g", V.name.c_str(), us[0], us[1], maxerr);
    // single-launch timeline (cold set, after the graph rotation): phases 0 start 1 issued 2 ready 3 end
    if (V.dv >= 0 || V.dv == -256 || V.dv == -512 || V.dv == -1024 || V.dv == -1025 || V.dv <= -2001) {
      if (V.dv <= -3001 && V.dv > -4000) {
        const int nwg = V.d + V.p;
        CHECK(hipMemset(d_st, 0, (size_t)nwg * 32));
        launchP(nsets - 1, V.d, V.p, d_st);
        CHECK(hipStreamSynchronize(st));
        std::vector<unsigned long long> hs((size_t)4 * nwg);
        CHECK(hipMemcpy(hs.data(), d_st, hs.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull;
        for (int b = 0; b < nwg; ++b) t0 = std::min(t0, hs[4 * b]);
        for (int part = 0; part < 2; ++part) {
          const int lo = part == 0 ? 0 : V.d, hi = part == 0 ? V.d : nwg;
          if (lo == hi) continue;
          for (int k : {0, 3}) {
            std::vector<double> x;
            for (int b = lo; b < hi; ++b) x.push_back((hs[4 * b + k] - t0) / 100.0);
            printf(", \"%s_ph%d\": [%.2f, %.2f, %.2f]", part == 0 ? "top" : "doc", k, pct(x, 0.1), pct(x, 0.5), pct(x, 1.0));
          }
        }
        printf("}\n");
        continue;
      }
      const int nwg = V.d + V.p + V.f;
      CHECK(hipMemset(d_st, 0, (size_t)nwg * 32));
      if (V.dv >= 0) launch(nsets - 1, V.dv, V.d, V.p, V.f, d_st);
      else if (V.dv == -4001) launchC(nsets - 1, d_st);
      else if (V.dv <= -2001) launchA(nsets - 1, -V.dv - 2000, d_st);
      else if (V.dv == -1024) launch3(nsets - 1, 1024, V.d, 0, d_st);
      else if (V.dv == -1025) launch3(nsets - 1, 512, V.d, 0, d_st);
      else launch2(nsets - 1, -V.dv, V.d, V.p, V.f, d_st);
      CHECK(hipStreamSynchronize(st));
      std::vector<unsigned long long> hs((size_t)4 * nwg);
      CHECK(hipMemcpy(hs.data(), d_st, hs.size() * 8, hipMemcpyDeviceToHost));
      unsigned long long t0 = ~0ull;
      for (int b = 0; b < nwg; ++b) t0 = std::min(t0, hs[4 * b]);
      for (int k = 0; k < 4; ++k) {
        std::vector<double> x;
        for (int b = 0; b < nwg; ++b)
          if (hs[4 * b + k]) x.push_back((hs[4 * b + k] - t0) / 100.0);
        printf(", \"ph%d\": [%.2f, %.2f, %.2f]", k, pct(x, 0.1), pct(x, 0.5), pct(x, 1.0));
      }
    }
    printf("}\n");
    fflush(stdout);
  }
  return 0;
}
