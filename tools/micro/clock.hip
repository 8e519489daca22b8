// Probe: shader clock over a graph replay. k_clock writes (s_memtime,
// s_memrealtime) into slot `i` of a device buffer with a vector store; two of
// them bracket the chained steps inside a captured graph, so
// d(memtime)/d(realtime) x 100 MHz is the average shader clock over the replay.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/micro/libclock.so tools/micro/clock.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void k_clock(uint64_t* out, int i) {
  uint64_t t = __builtin_amdgcn_s_memtime();
  uint64_t r = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[2 * i] = t;
    out[2 * i + 1] = r;
  }
}

extern "C" int clock_stamp(void* out, int i, void* stream) {
  hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, (hipStream_t)stream, (uint64_t*)out, i);
  return (int)hipGetLastError();
}
