// Streaming floor for measurements (bench.py "roofline_rocprof.copy"): dst = src
// for n floats, float4 grid-stride, 1024 x 256 threads, nontemporal stores.  It
// moves exactly the north-star SpMM's dense bytes (read B once, write C once)
// with no CSR and no gathers, so its cold duration is the ceiling any single
// launch over those bytes can reach (MI355X, R8's 2 x 6.18 MB, cold,
// scripts/micro/ns_micro.hip: 4.35 us with plain stores, 3.25 us with
// nontemporal ones = 50 % of 8 TB/s).  Not on the GCN path.
#include "gcnk_common.h"

namespace gcnk {
namespace {

__global__ void __launch_bounds__(256) stream_copy_kernel(const float4* __restrict__ src, float4* __restrict__ dst,
                                                          int64_t n4) {
  typedef float f4a __attribute__((ext_vector_type(4), aligned(16)));
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = src[i];
    __builtin_nontemporal_store(f4a{v.x, v.y, v.z, v.w}, reinterpret_cast<f4a*>(dst + i));
  }
}

__global__ void __launch_bounds__(256) stream_copy_tail_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                               int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int gcnk_stream_copy_f32(const float* src, float* dst, int64_t n, void* stream) {
  if (n < 0 || (n > 0 && (!src || !dst))) {
    set_error("gcnk_stream_copy_f32: bad argument (n=%lld)", (long long)n);
    return GCNK_EARG;
  }
  if (n == 0) return GCNK_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (aligned16(src) && aligned16(dst)) {
    const int64_t n4 = n / 4;
    if (n4 > 0) hipLaunchKernelGGL(stream_copy_kernel, dim3(1024), dim3(256), 0, s, reinterpret_cast<const float4*>(src),
                                   reinterpret_cast<float4*>(dst), n4);
    if (n % 4)
      hipLaunchKernelGGL(stream_copy_tail_kernel, dim3(1), dim3(256), 0, s, src + 4 * n4, dst + 4 * n4, n % 4);
  } else {
    hipLaunchKernelGGL(stream_copy_tail_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst, n);
  }
  return launch_check("stream_copy_kernel");
}
