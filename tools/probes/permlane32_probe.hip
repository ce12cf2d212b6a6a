// Checks that xor32() (v_permlane32_swap) returns lane l ^ 32's value, as __shfl_xor(v, 32).
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ inline int xor32(int v) {
  const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (threadIdx.x & 32) ? p[0] : p[1];
}
__global__ void k(int* o) {
  const int v = threadIdx.x * 7 + 3;
  o[threadIdx.x] = (xor32(v) == __shfl_xor(v, 32, 64)) ? 1 : 0;
}
int main() {
  int* d;
  int h[256];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
  int ok = 0;
  for (int i = 0; i < 256; ++i) ok += h[i];
  printf("permlane32 xor32 matches shfl_xor 32: %d / 256\n", ok);
  return ok == 256 ? 0 : 1;
}
