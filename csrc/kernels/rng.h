// Counter-based hashing RNG shared by device kernels and the host (CPU engine) code, so both
// engines draw identical values (K-Means sampling, synthetic data, ALS initial factors).
#pragma once

#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define OAP_HD __host__ __device__
#else
#define OAP_HD
#endif

namespace oap {
namespace kern {

OAP_HD inline uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

OAP_HD inline float u01_24(uint64_t h) {  // [0,1) with 24 random bits
  return static_cast<float>(h >> 40) * (1.0f / 16777216.0f);
}

// Initial ALS factor component f of the row with (global, user-facing) id: a standard normal
// from a counter-based hash, so every rank / world size / engine draws the same value.
OAP_HD inline double als_init_gaussian(uint64_t seed, int32_t id, int f) {
  const uint64_t h1 = splitmix64(seed ^ splitmix64(uint64_t(uint32_t(id)) * 0x9E3779B97F4A7C15ull +
                                                   uint64_t(f) * 0xD1B54A32D192ED03ull));
  const uint64_t h2 = splitmix64(h1);
  const double u1 = (double(h1 >> 11) + 1.0) * (1.0 / 9007199254740992.0);  // (0, 1]
  const double u2 = double(h2 >> 11) * (1.0 / 9007199254740992.0);
  return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

}  // namespace kern
}  // namespace oap
