// The reference's dropout keep-mask, drawn exactly as its CPU th.dropout draws
// it (layer.py:185 -> ATen dropout -> at::empty_like(x).bernoulli_(1 - p)),
// but without torch's per-element dispatch overhead: 17-27 ms of the R8
// training step went into torch's serial bernoulli_ loop.
//
// torch's CPU bernoulli_(double p) on a float tensor is the serial default
// kernel: for every element, in order, one 64-bit draw of the CPU generator
// (two MT19937 outputs r1, r2 -> (r1 << 32) | r2), a double uniform from its
// low 53 bits, u = (r64 & (2^53 - 1)) * 2^-53, and keep = u < p.  The generator
// is torch's MT19937 (state words, `left`, `next` as in its state tensor,
// CPUGeneratorImplStateLegacy).  This file restates that (checked bit for bit
// against torch in tests/test_rng.py, masks and the generator state after the
// draw), so the caller can write the advanced state back and every later draw
// of the process sees the same stream as under the reference.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <exception>
#include <thread>

#include "gcnk_common.h"

namespace gcnk {
namespace {

constexpr int kN = 624;
constexpr int kM = 397;

inline uint32_t twist_word(uint32_t u, uint32_t v, uint32_t w) {
  const uint32_t y = (u & 0x80000000u) | (v & 0x7fffffffu);
  return w ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

inline uint32_t temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

inline void twist_scalar(uint32_t* mt) {
  int i = 0;
  for (; i < kN - kM; ++i) mt[i] = twist_word(mt[i], mt[i + 1], mt[i + kM]);
  for (; i < kN - 1; ++i) mt[i] = twist_word(mt[i], mt[i + 1], mt[i + kM - kN]);
  mt[kN - 1] = twist_word(mt[kN - 1], mt[0], mt[kM - 1]);
}

// The same recurrence 8 words at a time (AVX2): within a vector every word
// reads mt[i + 1] before it is overwritten and mt[i + kM - kN] after it was,
// exactly as the scalar loop does.
typedef uint32_t v8u __attribute__((vector_size(32)));
__attribute__((target("avx2"))) inline v8u ld8(const uint32_t* p) {
  v8u v;
  __builtin_memcpy(&v, p, 32);
  return v;
}
__attribute__((target("avx2"))) inline void st8(uint32_t* p, v8u v) { __builtin_memcpy(p, &v, 32); }
__attribute__((target("avx2"))) inline v8u twist8(v8u u, v8u v, v8u w) {
  const v8u y = (u & 0x80000000u) | (v & 0x7fffffffu);
  const v8u odd = -(y & 1u);  // all ones where the low bit is set
  return w ^ (y >> 1) ^ (odd & 0x9908b0dfu);
}
__attribute__((target("avx2"))) inline v8u temper8(v8u y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
__attribute__((target("avx2"))) void twist_avx2(uint32_t* mt) {
  int i = 0;
  for (; i + 8 <= kN - kM; i += 8) st8(mt + i, twist8(ld8(mt + i), ld8(mt + i + 1), ld8(mt + i + kM)));
  for (; i < kN - kM; ++i) mt[i] = twist_word(mt[i], mt[i + 1], mt[i + kM]);
  for (; i + 8 <= kN - 1; i += 8) st8(mt + i, twist8(ld8(mt + i), ld8(mt + i + 1), ld8(mt + i + kM - kN)));
  for (; i < kN - 1; ++i) mt[i] = twist_word(mt[i], mt[i + 1], mt[i + kM - kN]);
  mt[kN - 1] = twist_word(mt[kN - 1], mt[0], mt[kM - 1]);
}

inline void twist(uint32_t* mt) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2) twist_avx2(mt);
  else twist_scalar(mt);
}


// u < p  <=>  m < p * 2^53  <=>  m < ceil(p * 2^53) for the integer m = r64 & (2^53 - 1)
// (p * 2^53 is exact in double), so the keep test is one 64-bit integer compare.
inline uint8_t keep(uint32_t hi, uint32_t lo, uint64_t T) {
  return (((uint64_t)(hi & 0x1fffffu) << 32) | lo) < T ? 1 : 0;
}

__attribute__((target("avx2"))) inline void temper_block_avx2(const uint32_t* w, int64_t cnt, uint32_t* t) {
  int64_t i = 0;
  for (; i + 8 <= cnt; i += 8) st8(t + i, temper8(ld8(w + i)));
  for (; i < cnt; ++i) t[i] = temper(w[i]);
}
inline void temper_block(const uint32_t* w, int64_t cnt, uint32_t* t) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2) {
    temper_block_avx2(w, cnt, t);
  } else {
    for (int64_t i = 0; i < cnt; ++i) t[i] = temper(w[i]);
  }
}
// The draw proper; arguments already checked.  No allocation, nothing that
// throws, so it can run on a worker thread (set_error is per thread).
void draw(uint32_t* state, int32_t* left, int64_t* next, int64_t n, double p, uint8_t* mask_out) {
  if (n == 0) return;
  const uint64_t T = (uint64_t)std::ceil(p * 9007199254740992.0);
  // One pass over the stream: each 624-word state block (the tail of the
  // current one first, then one per twist) is tempered 8 words at a time and
  // turned into keep flags straight away; a draw whose two words straddle a
  // block boundary carries its high word over.  No intermediate buffer: the
  // twist chain is serial anyway and the flags cost less than a copy of the
  // stream would.
  const int64_t words = 2 * n;
  int32_t lf = *left;
  int64_t nx = *next;
  int64_t o = 0, d = 0;
  bool have_hi = false;
  uint32_t hi = 0;
  uint32_t t[kN];
  while (o < words) {
    if (lf == 1) {  // torch's operator() decrements `left` first and twists when it reaches 0
      twist(state);
      lf = kN + 1;
      nx = 0;
    }
    const int64_t take = std::min<int64_t>(lf - 1, words - o);  // calls before the next twist
    temper_block(state + nx, take, t);
    int64_t i = 0;
    if (have_hi && take > 0) {
      mask_out[d++] = keep(hi, t[0], T);
      have_hi = false;
      i = 1;
    }
    for (; i + 1 < take; i += 2) mask_out[d++] = keep(t[i], t[i + 1], T);
    if (i < take) {
      hi = t[i];
      have_hi = true;
    }
    o += take;
    nx += take;
    lf -= (int32_t)take;
  }
  *left = lf;
  *next = nx;
}

bool bad_args(const uint32_t* state, const int32_t* left, const int64_t* next, int64_t n, double p,
              const uint8_t* mask_out) {
  return !state || !left || !next || n < 0 || (n > 0 && !mask_out) || *left < 1 || *next < 0 || *next > kN ||
         !(p >= 0.0 && p <= 1.0);
}

struct Job {
  std::thread th;
};
}  // namespace
}  // namespace gcnk

using namespace gcnk;

// state[624] / *left / *next: torch's MT19937 generator state, advanced in
// place by the 2 * n outputs the draw consumes.  mask_out[n]: 1 = kept.
// One thread (`threads` is accepted for ABI stability and ignored): the twist
// chain is serial, and tempering + the keep test run block by block behind it.
extern "C" int gcnk_bernoulli_mt19937(uint32_t* state, int32_t* left, int64_t* next, int64_t n, double p,
                                      uint8_t* mask_out, int32_t threads) {
  (void)threads;
  if (bad_args(state, left, next, n, p, mask_out)) {
    set_error("gcnk_bernoulli_mt19937: bad argument");
    return GCNK_EARG;
  }
  draw(state, left, next, n, p, mask_out);
  return GCNK_OK;
}

// The same draw on a native worker thread, so a training loop can draw the
// next step's mask while the GPU runs this one without any Python thread (and
// its interpreter-lock hand-offs) in the way.  The buffers must stay alive and
// untouched until gcnk_bernoulli_mt19937_wait(*job) returns; every started job
// must be waited for exactly once.
extern "C" int gcnk_bernoulli_mt19937_start(uint32_t* state, int32_t* left, int64_t* next, int64_t n, double p,
                                            uint8_t* mask_out, void** job) {
  if (!job || bad_args(state, left, next, n, p, mask_out)) {
    set_error("gcnk_bernoulli_mt19937_start: bad argument");
    return GCNK_EARG;
  }
  try {
    Job* j = new Job;
    j->th = std::thread(draw, state, left, next, n, p, mask_out);
    *job = j;
    return GCNK_OK;
  } catch (const std::exception& ex) {
    set_error("gcnk_bernoulli_mt19937_start: %s", ex.what());
    return GCNK_EUNSUP;
  }
}

extern "C" int gcnk_bernoulli_mt19937_wait(void* job) {
  if (!job) {
    set_error("gcnk_bernoulli_mt19937_wait: null job");
    return GCNK_EARG;
  }
  Job* j = static_cast<Job*>(job);
  if (j->th.joinable()) j->th.join();
  delete j;
  return GCNK_OK;
}
