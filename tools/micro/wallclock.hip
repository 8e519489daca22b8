// Probe: the rates of wall_clock64() (the bounded waits' clock, mpc_episode.h)
// and clock64() (torch.cuda._sleep's) on this GPU, against HIP events.
//   hipcc --offload-arch=gfx950 -O2 -o tools/micro/wallclock tools/micro/wallclock.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_probe(unsigned long long* out, int iters) {
  const long long w0 = wall_clock64(), c0 = clock64();
  for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
  const long long w1 = wall_clock64(), c1 = clock64();
  if (threadIdx.x == 0) {
    out[0] = w1 - w0;
    out[1] = c1 - c0;
  }
}

int main() {
  unsigned long long* d;
  unsigned long long h[2];
  hipMalloc(&d, 16);
  int rate_khz = 0;
  hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int iters : {1000, 100000, 1000000}) {
    hipEventRecord(a);
    k_probe<<<1, 64>>>(d, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("iters %d: %.3f ms; wall_clock64 %llu ticks = %.1f MHz (attribute %d kHz); "
           "clock64 %llu = %.1f MHz\n",
           iters, ms, h[0], h[0] / (ms * 1e3), rate_khz, h[1], h[1] / (ms * 1e3));
  }
  return 0;
}
