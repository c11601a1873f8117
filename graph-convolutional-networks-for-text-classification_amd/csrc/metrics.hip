// Evaluation metrics without host syncs.
//
// The reference's accuracy / macro_f1 (utils.py:25-109) take th.max(pred, 1)
// and then issue one .item() per count: 3 * nclass + 1 device->host syncs per
// evaluation (25 on R8, 61 on 20ng), each a full stream drain next to a ~40 us
// forward.  gcnk_class_stats computes every count in one launch -- argmax per
// scored row (first maximal index, NaN counts as maximal, as torch.max does),
// then per-class TP / FP / FN and the number of correct rows -- so the caller
// copies 3 * nclass + 1 integers back once.  Integer atomics: exact and
// order-independent.
#include "gcnk_common.h"

namespace gcnk {
namespace {

constexpr int kMaxClasses = 1024;

__global__ void __launch_bounds__(256)
class_stats_kernel(const float* __restrict__ logits, int64_t ld, const int64_t* __restrict__ target,
                   const int64_t* __restrict__ idx, int64_t n, int32_t nclass, int32_t* __restrict__ counts) {
  __shared__ int32_t s_cnt[3 * kMaxClasses + 1];  // tp | fp | fn | correct
  for (int i = threadIdx.x; i < 3 * nclass + 1; i += blockDim.x) s_cnt[i] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int64_t row = idx ? idx[i] : i;
    const float* p = logits + row * ld;
    int32_t best = 0;
    float bv = p[0];
    for (int32_t c = 1; c < nclass; ++c) {
      const float v = p[c];
      if (!(bv != bv) && (v > bv || v != v)) {  // first maximum; a NaN wins and stays
        bv = v;
        best = c;
      }
    }
    const int64_t t = target[row];
    if (best == t) {
      atomicAdd(&s_cnt[best], 1);                    // tp
      atomicAdd(&s_cnt[3 * nclass], 1);              // correct
    } else {
      atomicAdd(&s_cnt[nclass + best], 1);           // fp of the predicted class
      if (t >= 0 && t < nclass) atomicAdd(&s_cnt[2 * nclass + t], 1);  // fn of the true class
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 3 * nclass + 1; j += blockDim.x)
    if (s_cnt[j]) atomicAdd(&counts[j], s_cnt[j]);
}

}  // namespace
}  // namespace gcnk

using namespace gcnk;

extern "C" int gcnk_class_stats(const float* logits, int64_t ld, const int64_t* target, const int64_t* idx, int64_t n,
                                int32_t nclass, int32_t* counts, void* stream) {
  if (nclass < 1 || nclass > kMaxClasses || n < 0 || ld < nclass || !counts || (n > 0 && (!logits || !target))) {
    set_error("gcnk_class_stats: bad argument (n=%lld nclass=%d ld=%lld)", (long long)n, nclass, (long long)ld);
    return GCNK_EARG;
  }
  hipStream_t s = (hipStream_t)stream;
  int rc = hip_check(hipMemsetAsync(counts, 0, ((size_t)3 * nclass + 1) * 4, s), "class_stats memset");
  if (rc || n == 0) return rc;
  hipLaunchKernelGGL(class_stats_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, logits, ld, target, idx,
                     n, nclass, counts);
  return launch_check("class_stats_kernel");
}
