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
#include <atomic>
#include <cstdint>
#include <cstring>
#include <exception>
#include <thread>
#include <vector>

#include "gcnk_common.h"

namespace gcnk {
namespace {

constexpr int kN = 624;
constexpr int kM = 397;

inline uint32_t twist_word(uint32_t u, uint32_t v, uint32_t w) {
  const uint32_t y = (u & 0x80000000u) | (v & 0x7fffffffu);
  return w ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
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

inline uint32_t temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// Keep flags of a run of draws from raw (untempered) words w[0..2*cnt).
inline void keep_run(const uint32_t* w, int64_t cnt, double thr, uint8_t* out) {
  for (int64_t k = 0; k < cnt; ++k) {
    const uint64_t r64 = ((uint64_t)temper(w[2 * k]) << 32) | temper(w[2 * k + 1]);
    out[k] = (double)(r64 & ((1ull << 53) - 1)) < thr ? 1 : 0;
  }
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

// state[624] / *left / *next: torch's MT19937 generator state, advanced in
// place by the 2 * n outputs the draw consumes.  mask_out[n]: 1 = kept.
// The word stream is produced by one thread (the twists are a sequential
// chain) and turned into keep flags by threads - 1 workers as it appears.
extern "C" int gcnk_bernoulli_mt19937(uint32_t* state, int32_t* left, int64_t* next, int64_t n, double p,
                                      uint8_t* mask_out, int32_t threads) {
  if (!state || !left || !next || n < 0 || (n > 0 && !mask_out) || *left < 1 || *next < 0 || *next > kN) {
    set_error("gcnk_bernoulli_mt19937: bad argument");
    return GCNK_EARG;
  }
  if (n == 0) return GCNK_OK;
  try {
    const double thr = p * 9007199254740992.0;  // u < p  <=>  m < p * 2^53 (exact: m < 2^53)
    // raw words in consumption order; the draw consumes 2n of them.  The buffer
    // is kept per thread across calls (a training loop draws the same size
    // every step), so its pages are touched once.
    const int64_t words = 2 * n;
    static thread_local std::vector<uint32_t> w;
    if ((int64_t)w.size() < words) w.resize((size_t)words);
    int32_t lf = *left;
    int64_t nx = *next;
    const int nt = (threads > 1 && n >= 65536) ? threads : 1;
    uint32_t* wp = w.data();  // (w is thread_local: workers take the pointer, not the name)
    // The twist chain runs on this thread, publishing how many stream words
    // are ready; `nt` workers temper and compare their share of the draws as
    // soon as its words are out, so the flags overlap the (serial) twists.
    std::atomic<int64_t> ready{0};
    std::vector<std::thread> pool;
    for (int t = 0; t < nt - 1; ++t) {
      const int64_t b = n * t / (nt - 1), e = n * (t + 1) / (nt - 1);
      pool.emplace_back([wp, b, e, thr, mask_out, &ready] {
        int64_t k = b;
        while (k < e) {
          const int64_t avail = ready.load(std::memory_order_acquire) / 2;  // whole draws ready
          if (avail <= k) {
            std::this_thread::yield();
            continue;
          }
          const int64_t upto = std::min(avail, e);
          keep_run(wp + 2 * k, upto - k, thr, mask_out + k);
          k = upto;
        }
      });
    }
    int64_t o = 0;
    // torch's operator() decrements `left` first and twists when it reaches 0
    while (o < words) {
      if (lf == 1) {  // the next call twists
        twist(state);
        lf = kN + 1;
        nx = 0;
      }
      const int64_t avail = lf - 1;  // calls before the next twist
      const int64_t take = std::min<int64_t>(avail, words - o);
      std::memcpy(wp + o, state + nx, (size_t)take * 4);
      o += take;
      nx += take;
      lf -= (int32_t)take;
      ready.store(o, std::memory_order_release);
    }
    *left = lf;
    *next = nx;
    if (nt == 1) keep_run(wp, n, thr, mask_out);
    for (std::thread& th : pool) th.join();
    return GCNK_OK;
  } catch (const std::exception& ex) {
    set_error("gcnk_bernoulli_mt19937: %s", ex.what());
    return GCNK_EUNSUP;
  }
}
