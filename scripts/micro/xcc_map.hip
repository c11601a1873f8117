// Which XCD runs workgroup b?  The row plan deals units to workgroups assuming
// round-robin dispatch (workgroup b on XCD b % 8, csrc/spmm.hip "XCD classes");
// this reads each workgroup's XCC_ID hardware register and reports how often
// that holds, for the north-star launch shape (1,832 x 256 threads) and others.
//   hipcc -O3 --offload-arch=gfx950 xcc_map.hip -o xcc_map && ./xcc_map
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void xcc_of_block(int* out, int spin) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  // a little work so that workgroups overlap as in a real launch
  float acc = 0.f;
  for (int i = 0; i < spin; ++i) acc += __builtin_sinf(acc + i);
  if (threadIdx.x == 0) out[blockIdx.x] = (int)(x & 0xF) + (acc == 12345.f ? 100 : 0);
}

int main() {
  const int shapes[][2] = {{1832, 256}, {968, 256}, {242, 512}, {4096, 64}, {280, 256}};
  int* d = nullptr;
  if (hipMalloc(&d, 8192 * sizeof(int)) != hipSuccess) return 2;
  for (auto& sh : shapes) {
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(xcc_of_block, dim3(sh[0]), dim3(sh[1]), 0, 0, d, 64);
      if (hipDeviceSynchronize() != hipSuccess) return 3;
      std::vector<int> h(sh[0]);
      if (hipMemcpy(h.data(), d, sh[0] * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 4;
      int same = 0, cnt[16] = {0};
      for (int b = 0; b < sh[0]; ++b) {
        same += (h[b] & 0xF) == b % 8;
        cnt[h[b] & 0xF]++;
      }
      printf("{\"grid\": %d, \"block\": %d, \"rep\": %d, \"xcc_eq_b_mod_8\": %.4f, \"first16\": [", sh[0], sh[1], rep,
             (double)same / sh[0]);
      for (int b = 0; b < 16 && b < sh[0]; ++b) printf("%d%s", h[b], b < 15 ? ", " : "");
      printf("], \"per_xcc\": [");
      for (int x = 0; x < 8; ++x) printf("%d%s", cnt[x], x < 7 ? ", " : "");
      printf("]}\n");
    }
  }
  (void)hipFree(d);
  return 0;
}
