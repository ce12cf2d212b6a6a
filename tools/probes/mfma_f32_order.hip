// Which scalar fp32 arithmetic does v_mfma_f32_32x32x2_f32 reproduce bitwise?  The exact K-Means
// re-decision (kernels/kmeans_lloyd.hip oap_kmeans_exact_rows) decides on these MFMA dot
// products; a VALU evaluation of a few candidate centers can replace the full MFMA sweep only if
// it rounds the same way.  Random operands (mixed magnitudes and signs, so rounding differences
// show), one 32x32x2 step and a chain of 28 steps, compared element by element with:
//   F01  fmaf(a1, b1, fmaf(a0, b0, acc))      (k = 0 first)
//   F10  fmaf(a0, b0, fmaf(a1, b1, acc))      (k = 1 first)
//   DOT  acc + (a0 b0 + a1 b1) with the pair summed exactly (fp64) and one fp32 rounding at the end
// hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_f32_order.hip -o tools/probes/mfma_f32_order
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kSteps = 28;

// lane l: A[i = l & 31][k = l >> 5] per step (32 x 2), B[k = l >> 5][j = l & 31] (2 x 32);
// acc element e of lane l: row i = 8 (e / 4) + 4 (l >> 5)... use the documented C layout:
// C[i][j] with j = l & 31 and i = (e & 3) + 8 (e >> 2) + 4 (l >> 5)
__global__ void probe(const float* A, const float* B, const float* C0, float* out, int steps) {
  const int l = threadIdx.x;
  f32x16 acc;
  for (int e = 0; e < 16; ++e) {
    const int i = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5), j = l & 31;
    acc[e] = C0[i * 32 + j];
  }
  for (int s = 0; s < steps; ++s) {
    const float a = A[s * 64 + (l >> 5) * 32 + (l & 31)];  // A[s][k][i]
    const float b = B[s * 64 + (l >> 5) * 32 + (l & 31)];  // B[s][k][j]
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  for (int e = 0; e < 16; ++e) {
    const int i = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5), j = l & 31;
    out[i * 32 + j] = acc[e];
  }
}

static float frand(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  const float u = float(s >> 8) / float(1u << 24) - 0.5f;
  s = s * 1664525u + 1013904223u;
  const int ex = int(s >> 27) - 16;  // magnitudes 2^-16 .. 2^15
  return std::ldexp(u, ex);
}

int main() {
  for (int steps : {1, kSteps}) {
    std::vector<float> A(steps * 64), B(steps * 64), C0(1024), out(1024);
    unsigned s = 12345u + steps;
    for (auto& v : A) v = frand(s);
    for (auto& v : B) v = frand(s);
    for (auto& v : C0) v = frand(s);
    float *dA, *dB, *dC, *dO;
    hipMalloc(&dA, A.size() * 4);
    hipMalloc(&dB, B.size() * 4);
    hipMalloc(&dC, 4096);
    hipMalloc(&dO, 4096);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC, C0.data(), 4096, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, 1, 64, 0, 0, dA, dB, dC, dO, steps);
    hipMemcpy(out.data(), dO, 4096, hipMemcpyDeviceToHost);
    int m01 = 0, m10 = 0, mdot = 0;
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        float f01 = C0[i * 32 + j], f10 = f01, fd = f01;
        for (int t = 0; t < steps; ++t) {
          const float a0 = A[t * 64 + i], a1 = A[t * 64 + 32 + i];
          const float b0 = B[t * 64 + j], b1 = B[t * 64 + 32 + j];
          f01 = std::fmaf(a1, b1, std::fmaf(a0, b0, f01));
          f10 = std::fmaf(a0, b0, std::fmaf(a1, b1, f10));
          fd = float(double(fd) + (double(a0) * b0 + double(a1) * b1));
        }
        const float g = out[i * 32 + j];
        m01 += std::memcmp(&g, &f01, 4) == 0;
        m10 += std::memcmp(&g, &f10, 4) == 0;
        mdot += std::memcmp(&g, &fd, 4) == 0;
      }
    std::printf("{\"steps\": %d, \"of\": 1024, \"F01\": %d, \"F10\": %d, \"DOT\": %d}\n", steps,
                m01, m10, mdot);
  }
  return 0;
}
