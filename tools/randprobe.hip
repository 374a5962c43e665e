// randprobe.hip -- microbenchmark: random-gather latency and throughput of MI355X HBM (NOT part of
// libketogpu).  The check kernels are pointer chasers whose unit of work is one random 16-64 B
// read; this measures what the memory system delivers for exactly that access pattern, so the
// kernels' roofline can be stated as a fraction of the random-line rate as well as of 8 TB/s.
//   latency:    one lane per CU walks a random cycle (each load's address comes from the last)
//   throughput: every lane of W waves per CU issues K independent random 16-B (or 64-B) loads
//               per round, R rounds; lines/s and GB/s of requested bytes
// usage: randprobe <GiB> <waves_per_cu> <bytes_per_load 16|64> [<in_flight_per_lane>]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                    \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

__global__ void k_fill(uint4* a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t nx = mix(i + 1) % n;  // a pseudo-random successor (a chase, not a permutation)
    a[i] = make_uint4((uint32_t)nx, (uint32_t)(nx >> 32), (uint32_t)i, 0);
  }
}

__global__ void k_chase(const uint4* a, uint64_t n, int steps, uint64_t* out, unsigned long long* cyc) {
  if (threadIdx.x != 0) return;
  uint64_t p = mix(blockIdx.x * 977 + 5) % n;
  const unsigned long long t0 = wall_clock64();
  for (int s = 0; s < steps; s++) {
    const uint4 v = a[p];
    p = ((uint64_t)v.y << 32) | v.x;
  }
  const unsigned long long t1 = wall_clock64();
  out[blockIdx.x] = p;
  cyc[blockIdx.x] = t1 - t0;
}

template <int K, int W>
__global__ __launch_bounds__(256) void k_gather(const uint4* a, uint64_t n, int rounds, uint32_t* sink) {
  // W = 16-B words per load (1: 16 B, 4: 64 B)
  uint64_t h = mix(blockIdx.x * 256ull + threadIdx.x + 1);
  uint32_t acc = 0;
  for (int r = 0; r < rounds; r++) {
    uint4 v[K][W];
#pragma unroll
    for (int k = 0; k < K; k++) {
      h = mix(h + k);
      const uint64_t i = (h % (n / W)) * W;
#pragma unroll
      for (int w = 0; w < W; w++) v[k][w] = a[i + w];
    }
#pragma unroll
    for (int k = 0; k < K; k++)
#pragma unroll
      for (int w = 0; w < W; w++) acc += v[k][w].x ^ v[k][w].z;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 4.0;
  const int wpc = argc > 2 ? atoi(argv[2]) : 8;
  const int bytes = argc > 3 ? atoi(argv[3]) : 16;
  const uint64_t n = (uint64_t)(gib * (1ull << 30)) / 16;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint4* a;
  uint32_t* sink;
  uint64_t* out;
  unsigned long long* cyc;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&out, cus * 8));
  CK(hipMalloc(&cyc, cus * 8));
  k_fill<<<4096, 256>>>(a, n);
  CK(hipDeviceSynchronize());
  // latency: one chaser per CU (idle chip otherwise)
  const int steps = 20000;
  k_chase<<<cus, 64>>>(a, n, steps, out, cyc);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> c(cus);
  CK(hipMemcpy(c.data(), cyc, cus * 8, hipMemcpyDeviceToHost));
  double mean = 0;
  for (auto x : c) mean += (double)x;
  mean /= cus;
  printf("{\"array_gib\": %.2f, \"chase_ns_per_load\": %.1f", gib, mean / steps * 10.0);  // wall_clock64: 100 MHz
  // throughput
  const int rounds = 64;
  const int blocks = cus * (wpc / 4 > 0 ? wpc / 4 : 1);
  auto run = [&](auto kern, int loads_per_round, int w) {
    kern<<<blocks, 256>>>(a, n, 4, sink);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    kern<<<blocks, 256>>>(a, n, rounds, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double loads = (double)blocks * 256 * rounds * loads_per_round;
    printf(", \"k%d_x%dB\": {\"Gloads_per_s\": %.2f, \"GB_per_s\": %.1f}", loads_per_round, 16 * w, loads / ms / 1e6,
           loads * 16 * w / ms / 1e6);
  };
  if (bytes == 64) {
    run(k_gather<1, 4>, 1, 4);
    run(k_gather<4, 4>, 4, 4);
  } else {
    run(k_gather<1, 1>, 1, 1);
    run(k_gather<4, 1>, 4, 1);
    run(k_gather<8, 1>, 8, 1);
  }
  printf(", \"waves_per_cu\": %d}\n", (blocks / cus) * 4);
  return 0;
}
