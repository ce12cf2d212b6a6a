// Throughput probe: v_mfma_f64_16x16x4_f64 issue rate on one GPU (registers only, no memory).
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_f64_probe.hip -o build/mfma_f64_probe
// Prints achieved TFLOP/s for 1, 2 and 4 waves per SIMD and 8 / 16 independent accumulators.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void probe(double* out, int iters, double a0, double b0) {
  f64x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f64x4{0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
void run(int waves_per_simd, int cus) {
  const int threads = 256 * waves_per_simd > 1024 ? 1024 : 256 * waves_per_simd;
  const int blocks = cus * (256 * waves_per_simd / threads);
  double* out;
  hipMalloc(&out, sizeof(double) * blocks * threads);
  const int iters = 4000;
  hipLaunchKernelGGL(probe<NACC>, dim3(blocks), dim3(threads), 0, 0, out, 10, 1.0, 2.0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<NACC>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0, 2.0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = double(blocks) * (threads / 64) * iters * NACC * 16.0 * 16 * 4 * 2;
  std::printf("nacc=%d waves/simd=%d: %.2f ms  %.1f TFLOP/s\n", NACC, waves_per_simd, ms,
              flops / (ms * 1e-3) / 1e12);
  hipFree(out);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  std::printf("%s CUs=%d clock=%d kHz\n", p.gcnArchName, cus, p.clockRate);
  for (int w : {1, 2, 4}) {
    run<8>(w, cus);
    run<16>(w, cus);
  }
  return 0;
}
