// Probe: does a tile-contiguous candidate layout stream faster than the ABI's
// step-major SoA?  Both read exactly 16 B per candidate-step (v and beta,
// fp64) with 16-B vector loads, one tile = 512 candidates per 256-thread
// block (2 per lane, the chained kernel's tiling), N steps, nothing computed
// (an XOR keeps the loads alive).
//   A  step-major SoA (the ABI): v[s*C + c], b[s*C + c]
//   B  tile-contiguous: tile t's N steps x {v, b} x 512 values in one block
//      of 80 KiB at N = 10
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/layout_probe tools/micro/layout_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef double d2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(const double* __restrict__ v,
                                               const double* __restrict__ b, int64_t C, int N,
                                               uint64_t* __restrict__ sink) {
  const int64_t tile = blockIdx.x;
  const int64_t c = tile * 512 + threadIdx.x * 2;
  uint64_t acc = 0;
  if (c < C) {
#pragma unroll 2
    for (int s = 0; s < N; ++s) {
      const double* pv;
      const double* pb;
      if (MODE == 0) {
        pv = v + s * C + c;
        pb = b + s * C + c;
      } else {
        const double* base = v + tile * (int64_t)N * 1024 + s * 1024;
        pv = base + threadIdx.x * 2;
        pb = base + 512 + threadIdx.x * 2;
      }
      const d2 x = __builtin_nontemporal_load(reinterpret_cast<const d2*>(pv));
      const d2 y = __builtin_nontemporal_load(reinterpret_cast<const d2*>(pb));
      acc ^= __double_as_longlong(x.x) ^ __double_as_longlong(x.y) ^ __double_as_longlong(y.x) ^
             __double_as_longlong(y.y);
    }
  }
  if (acc == 0x123456789ull) sink[blockIdx.x] = acc;
}

int main() {
  const int N = 10;
  const int nbuf = 4;
  for (int64_t C : {1000000LL, 8000000LL}) {
    const size_t bytes = (size_t)C * N * 8;
    double* v[nbuf];
    double* b[nbuf];
    for (int i = 0; i < nbuf; ++i) {
      hipMalloc(&v[i], 2 * bytes);   // B uses v as one array of 2 x bytes
      hipMemset(v[i], 1, 2 * bytes);
      b[i] = v[i] + (size_t)C * N;
    }
    uint64_t* sink;
    hipMalloc(&sink, 1 << 20);
    const int grid = (int)((C + 511) / 512);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int mode = 0; mode < 2; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        for (int i = 0; i < 100; ++i) {
          if (mode == 0) k_probe<0><<<grid, 256>>>(v[i % nbuf], b[i % nbuf], C, N, sink);
          else k_probe<1><<<grid, 256>>>(v[i % nbuf], b[i % nbuf], C, N, sink);
        }
        hipEventRecord(e0);
        const int reps = 200;
        for (int i = 0; i < reps; ++i) {
          if (mode == 0) k_probe<0><<<grid, 256>>>(v[i % nbuf], b[i % nbuf], C, N, sink);
          else k_probe<1><<<grid, 256>>>(v[i % nbuf], b[i % nbuf], C, N, sink);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / reps;
        printf("C %lld N %d layout %s: %.2f us per launch, %.3f TB/s\n", (long long)C, N,
               mode == 0 ? "A step-major SoA " : "B tile-contiguous", us,
               2.0 * bytes / (us * 1e-6) / 1e12);
      }
    }
    for (int i = 0; i < nbuf; ++i) hipFree(v[i]);
    hipFree(sink);
  }
  return 0;
}
