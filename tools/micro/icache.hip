// Probe: how much of a one-wave serial phase is instruction fetch?  One
// block of 64 threads runs the same straight-line code twice (a loop of two
// passes, so the second pass executes the instructions the first fetched)
// and stamps s_memrealtime (100 MHz) before, between and after.  Launched
// back to back as the chained step's block 0 is, with a streaming kernel in
// between (optional) to evict L2 as the tiles' controls would.
//   A: 512 independent v_add_f32 (4 KiB of code), no data dependences
//   B: the wave's 64-bit lexicographic arg-min (DPP) repeated 8 times
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/icache tools/micro/icache.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

#define ADD8 "v_add_f32 %0, %0, 1.0\n\tv_add_f32 %1, %1, 1.0\n\tv_add_f32 %2, %2, 1.0\n\tv_add_f32 %3, %3, 1.0\n\t" \
             "v_add_f32 %0, %0, 1.0\n\tv_add_f32 %1, %1, 1.0\n\tv_add_f32 %2, %2, 1.0\n\tv_add_f32 %3, %3, 1.0\n\t"
#define ADD64 ADD8 ADD8 ADD8 ADD8 ADD8 ADD8 ADD8 ADD8
#define ADD512 ADD64 ADD64 ADD64 ADD64 ADD64 ADD64 ADD64 ADD64

__global__ __launch_bounds__(64) void k_straight(uint64_t* stamps, float* sink) {
  float a = threadIdx.x, b = 1, c = 2, d = 3;
  uint64_t t[3];
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    t[pass] = now();
    asm volatile(ADD512 : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  }
  t[2] = now();
  if (threadIdx.x == 0)
    for (int q = 0; q < 3; ++q) stamps[q] = t[q];
  if (a + b + c + d == 12345.f) sink[threadIdx.x] = a;
}

template <int CTRL, int RM = 0xf>
__device__ __forceinline__ void lvl(uint64_t& k, int64_t& i) {
  auto mv = [](uint64_t x) {
    const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(x), CTRL, RM, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(x >> 32), CTRL, RM, 0xf, true);
    return (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo);
  };
  const uint64_t ok = mv(k);
  const int64_t oi = static_cast<int64_t>(mv(static_cast<uint64_t>(i)));
  const bool lt = ok < k || (ok == k && oi < i);
  k = lt ? ok : k;
  i = lt ? oi : i;
}

__global__ __launch_bounds__(64) void k_argmin(const uint64_t* keys, uint64_t* stamps, uint64_t* sink) {
  uint64_t k = keys[threadIdx.x];
  int64_t i = threadIdx.x;
  uint64_t t[3];
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    t[pass] = now();
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      lvl<0xB1>(k, i);
      lvl<0x4E>(k, i);
      lvl<0x141>(k, i);
      lvl<0x140>(k, i);
      lvl<0x142, 0xA>(k, i);
      lvl<0x143, 0xC>(k, i);
      k ^= static_cast<uint64_t>(r) << (threadIdx.x & 7);
    }
  }
  t[2] = now();
  if (threadIdx.x == 0)
    for (int q = 0; q < 3; ++q) stamps[q] = t[q];
  if (k == 0x1234567) sink[threadIdx.x] = k + i;
}

typedef double d2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_stream(const d2* __restrict__ x, int64_t n, double* sink) {
  double acc = 0;
  for (int64_t j = blockIdx.x * 256 + threadIdx.x; j < n; j += (int64_t)gridDim.x * 256) {
    const d2 v = __builtin_nontemporal_load(&x[j]);
    acc += v.x + v.y;
  }
  if (acc == 1.2345) sink[0] = acc;
}

int main() {
  uint64_t* st;
  float* sinkf;
  uint64_t* sinku;
  uint64_t* keys;
  d2* big;
  double* sinkd;
  const int64_t nbig = 16ll << 20;   // 256 MiB
  hipMalloc(&st, 4096);
  hipMalloc(&sinkf, 4096);
  hipMalloc(&sinku, 4096);
  hipMalloc(&keys, 4096);
  hipMalloc(&sinkd, 64);
  hipMalloc(&big, nbig * sizeof(d2));
  hipMemset(big, 0, nbig * sizeof(d2));
  hipMemset(keys, 7, 4096);
  for (int evict = 0; evict < 2; ++evict) {
    for (int kind = 0; kind < 2; ++kind) {
      double s0 = 0, s1 = 0;
      const int reps = 50;
      for (int r = 0; r < reps + 5; ++r) {
        if (evict) k_stream<<<4096, 256>>>(big, nbig, sinkd);
        if (kind == 0) k_straight<<<1, 64>>>(st, sinkf);
        else k_argmin<<<1, 64>>>(keys, st, sinku);
        uint64_t h[3];
        hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost);
        if (r >= 5) {
          s0 += (h[1] - h[0]) * 0.01;
          s1 += (h[2] - h[1]) * 0.01;
        }
      }
      printf("%s%s: first pass %.3f us, second pass %.3f us\n",
             kind == 0 ? "A 512 independent v_add_f32 (4 KiB code)" : "B 8 x 64-bit DPP arg-min",
             evict ? " after a 256-MiB stream" : "", s0 / reps, s1 / reps);
    }
  }
  return 0;
}
