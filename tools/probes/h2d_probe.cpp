// Host -> device ingestion paths for a large pageable numpy-like buffer (what
// KMeans.fit(ndarray) uploads), measured on the box:
//   A  pinned peak: hipMemcpyAsync from a hipHostMalloc buffer (chunks of 256 MB, 2 streams)
//   B  staged, one thread: memcpy into a pinned slot, then its DMA (the round-5 upload)
//   C  staged, T threads: the memcpy split over T host threads, DMA of slot i overlapped with
//      the copy into slot i ^ 1
//   D  registered in place: hipHostRegister of the pageable buffer (timed), DMA straight from it,
//      hipHostUnregister (timed)
// hipcc -O3 -std=c++17 -pthread tools/probes/h2d_probe.cpp -o tools/probes/h2d_probe
//   ./h2d_probe [GiB=8] [threads=16]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));           \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

static void par_memcpy(char* dst, const char* src, size_t n, int T) {
  std::vector<std::thread> th;
  const size_t per = (n + T - 1) / T;
  for (int t = 0; t < T; ++t) {
    const size_t b = std::min(n, size_t(t) * per), e = std::min(n, b + per);
    if (e > b) th.emplace_back([=] { std::memcpy(dst + b, src + b, e - b); });
  }
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? std::atof(argv[1]) : 8.0;
  const int T = argc > 2 ? std::atoi(argv[2]) : 16;
  const size_t N = size_t(gib * double(1ull << 30));
  const size_t C = size_t(256) << 20;
  char* host = static_cast<char*>(std::malloc(N));
  for (size_t i = 0; i < N; i += 4096) host[i] = char(i >> 12);  // touch every page
  std::memset(host, 1, N);
  char* dev = nullptr;
  CK(hipMalloc(&dev, N));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  char* pin[2];
  CK(hipHostMalloc(&pin[0], C));
  CK(hipHostMalloc(&pin[1], C));
  hipEvent_t ev[2];
  CK(hipEventCreate(&ev[0]));
  CK(hipEventCreate(&ev[1]));
  auto gbs = [&](double s) { return double(N) / s / 1e9; };

  // A: pinned peak (re-sending the same pinned chunk)
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipDeviceSynchronize());
    double t0 = now();
    for (size_t o = 0; o < N; o += C)
      CK(hipMemcpyAsync(dev + o, pin[(o / C) & 1], std::min(C, N - o), hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    std::printf("A pinned peak            %.3f s  %.1f GB/s\n", now() - t0, gbs(now() - t0));
  }
  // B / C: staged through two pinned slots, T copy threads
  for (int threads : {1, 4, 8, T}) {
    CK(hipDeviceSynchronize());
    double t0 = now();
    bool used[2] = {false, false};
    int slot = 0;
    for (size_t o = 0; o < N; o += C, slot ^= 1) {
      const size_t n = std::min(C, N - o);
      if (used[slot]) CK(hipEventSynchronize(ev[slot]));
      par_memcpy(pin[slot], host + o, n, threads);
      CK(hipMemcpyAsync(dev + o, pin[slot], n, hipMemcpyHostToDevice, st));
      CK(hipEventRecord(ev[slot], st));
      used[slot] = true;
    }
    CK(hipStreamSynchronize(st));
    const double s = now() - t0;
    std::printf("%c staged, %2d threads     %.3f s  %.1f GB/s\n", threads == 1 ? 'B' : 'C', threads,
                s, gbs(s));
  }
  // D: register in place
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipDeviceSynchronize());
    double t0 = now();
    CK(hipHostRegister(host, N, hipHostRegisterDefault));
    double t1 = now();
    for (size_t o = 0; o < N; o += C)
      CK(hipMemcpyAsync(dev + o, host + o, std::min(C, N - o), hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    double t2 = now();
    CK(hipHostUnregister(host));
    double t3 = now();
    std::printf("D registered: register %.3f s, DMA %.3f s (%.1f GB/s), unregister %.3f s, "
                "total %.3f s  %.1f GB/s\n",
                t1 - t0, t2 - t1, gbs(t2 - t1), t3 - t2, t3 - t0, gbs(t3 - t0));
  }
  CK(hipFree(dev));
  CK(hipHostFree(pin[0]));
  CK(hipHostFree(pin[1]));
  std::free(host);
  return 0;
}
