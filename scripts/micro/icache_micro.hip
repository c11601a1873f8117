// Does a kernel's straight-line code size cost start-up time on MI355X when
// every CU runs it at once (a cold instruction fetch of the same lines by all
// CUs)?  Round 6 found an 8-wave dense gc1 whose waves spent ~7 us before
// their first barrier even with no memory load in it (profiles/r06_dense_ab.log);
// its code was 41-58 KB against the committed kernel's 16 KB.
//
// Kernels of N back-to-back `s_nop 0` (4 B each, one cycle each) between two
// s_memrealtime reads; 256 or 512 workgroups of 512 threads; per launch the
// HIP-event time and the per-workgroup in-kernel span (median / max), first
// launch (cold code) and warm repeats.  A fetch-bound start-up shows as spans
// far above N cycles that grow with N (4 KB per 1,024 nops).
//
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/micro/icache_micro scripts/micro/icache_micro.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      return 1;                                                               \
    }                                                                         \
  } while (0)

#define NOPS_STR2(n) #n
#define NOPS_STR(n) NOPS_STR2(n)

template <int N>
__global__ void __launch_bounds__(512) nop_kernel(unsigned long long* stamps) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  asm volatile(".rept %c0\n s_nop 0\n .endr" ::"i"(N));
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  if (threadIdx.x == 0) {   // vector global stores
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t1;
  }
}

template <int N>
int run(int nblk, unsigned long long* d_st, std::vector<unsigned long long>& h) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int rep = 0; rep < 6; ++rep) {
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(nop_kernel<N>, dim3(nblk), dim3(512), 0, 0, d_st);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipMemcpy(h.data(), d_st, 2 * nblk * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    std::vector<double> span(nblk);
    unsigned long long first = ~0ull, last = 0;
    for (int i = 0; i < nblk; ++i) {
      span[i] = (h[2 * i + 1] - h[2 * i]) / 100.0;   // s_memrealtime: 100 MHz -> us
      first = std::min(first, h[2 * i]);
      last = std::max(last, h[2 * i + 1]);
    }
    std::sort(span.begin(), span.end());
    std::printf("{\"nops\": %d, \"code_kb\": %.1f, \"blocks\": %d, \"rep\": %d, \"event_us\": %.2f, "
                "\"span_p50_us\": %.2f, \"span_max_us\": %.2f, \"first_to_last_us\": %.2f, "
                "\"nop_cycles_us_at_2.4GHz\": %.2f}\n",
                N, N * 4 / 1024.0, nblk, rep, ms * 1e3, span[nblk / 2], span[nblk - 1], (last - first) / 100.0,
                N / 2400.0);
  }
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return 0;
}

int main() {
  const int maxblk = 512;
  unsigned long long* d_st = nullptr;
  CHECK(hipMalloc(&d_st, 2 * maxblk * sizeof(unsigned long long)));
  std::vector<unsigned long long> h(2 * maxblk);
  for (int nblk : {256, 512}) {
    if (run<16>(nblk, d_st, h)) return 1;
    if (run<1024>(nblk, d_st, h)) return 1;
    if (run<4096>(nblk, d_st, h)) return 1;
    if (run<12288>(nblk, d_st, h)) return 1;
  }
  CHECK(hipFree(d_st));
  return 0;
}
