// Launch-floor microbenchmark: per-kernel time of back-to-back launches of
// near-empty kernels inside a hipGraph (and eagerly), for several grid sizes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_empty() {}
__global__ void k_touch(float* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + 1.0f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <typename F>
float time_graph(hipStream_t s, int reps, F launch) {
  hipGraph_t g; hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < reps; ++i) launch();
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s); hipStreamSynchronize(s);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float best = 1e30f;
  for (int t = 0; t < 5; ++t) {
    hipEventRecord(a, s); hipGraphLaunch(ge, s); hipEventRecord(b, s); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
  }
  hipGraphExecDestroy(ge); hipGraphDestroy(g);
  return best * 1e3f / reps;
}

int main() {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* p; CK(hipMalloc(&p, 64 << 20));
  CK(hipMemset(p, 0, 64 << 20));
  const int reps = 500;
  printf("{\"empty_1wg_us\": %.3f", time_graph(s, reps, [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); }));
  printf(", \"empty_1024wg_us\": %.3f", time_graph(s, reps, [&] { hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s); }));
  for (int n : {256, 65536, 1 << 20, 4 << 20}) {
    printf(", \"touch_%d_us\": %.3f", n, time_graph(s, reps, [&] { hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, s, p, n); }));
  }
  printf("}\n");
  return 0;
}
