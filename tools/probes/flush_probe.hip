// What does the end-of-pass flush of per-workgroup K-Means sums cost?  256 workgroups (one per
// CU, as the lean / exact passes run) each add a k x d block of int64 partial sums into one
// device array:
//   A  device-scope atomicAdd of every entry (what kmeans_lean_img / kmeans_exact_rows do now),
//   B  plain stores into a [grid][k*d] slab + one reduction kernel over the grid,
//   C  atomics into 8 per-XCD copies (blockIdx & 7) + one reduction over the 8.
// hipcc --offload-arch=gfx950 -O3 tools/probes/flush_probe.hip -o tools/probes/flush_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef unsigned long long u64;

__global__ __launch_bounds__(1024) void flush_atomic(u64* sums, int kd) {
  for (int i = threadIdx.x; i < kd; i += blockDim.x) atomicAdd(&sums[i], u64(blockIdx.x + i));
}

__global__ __launch_bounds__(1024) void flush_slab(u64* slab, int kd) {
  u64* s = slab + size_t(blockIdx.x) * kd;
  for (int i = threadIdx.x; i < kd; i += blockDim.x) s[i] = u64(blockIdx.x + i);
}

__global__ __launch_bounds__(256) void reduce_slab(const u64* slab, int kd, int parts, u64* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kd) return;
  u64 t = 0;
  for (int p = 0; p < parts; ++p) t += slab[size_t(p) * kd + i];
  out[i] = t;
}

__global__ __launch_bounds__(1024) void flush_xcd(u64* sums8, int kd) {
  u64* s = sums8 + size_t(blockIdx.x & 7) * kd;
  for (int i = threadIdx.x; i < kd; i += blockDim.x) atomicAdd(&s[i], u64(blockIdx.x + i));
}

int main(int argc, char** argv) {
  const int kd = argc > 1 ? std::atoi(argv[1]) : 10000;
  const int grid = argc > 2 ? std::atoi(argv[2]) : 256;
  const int reps = 20;
  u64 *sums, *slab, *out;
  CK(hipMalloc(&sums, size_t(kd) * 8 * 8));
  CK(hipMalloc(&slab, size_t(kd) * 8 * grid));
  CK(hipMalloc(&out, size_t(kd) * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](auto fn) {
    fn();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) fn();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / reps;
  };
  const int rb = (kd + 255) / 256;
  const float ta = time([&] { hipLaunchKernelGGL(flush_atomic, grid, 1024, 0, 0, sums, kd); });
  const float tb = time([&] {
    hipLaunchKernelGGL(flush_slab, grid, 1024, 0, 0, slab, kd);
    hipLaunchKernelGGL(reduce_slab, rb, 256, 0, 0, slab, kd, grid, out);
  });
  const float tc = time([&] {
    hipLaunchKernelGGL(flush_xcd, grid, 1024, 0, 0, sums, kd);
    hipLaunchKernelGGL(reduce_slab, rb, 256, 0, 0, sums, kd, 8, out);
  });
  const float tw = time([&] { hipLaunchKernelGGL(flush_slab, grid, 1024, 0, 0, slab, kd); });
  CK(hipGetLastError());
  std::printf("{\"kd\": %d, \"grid\": %d, \"atomic_us\": %.2f, \"slab_plus_reduce_us\": %.2f, "
              "\"slab_write_only_us\": %.2f, \"xcd_atomic_plus_reduce_us\": %.2f}\n",
              kd, grid, ta, tb, tw, tc);
  return 0;
}
