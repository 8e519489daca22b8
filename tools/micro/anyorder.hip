// anyorder.hip — does a kernel launched with hipExtAnyOrderLaunch start
// before the previous kernel on the same stream has completed (AQL barrier
// bit cleared), eagerly and inside a captured HIP graph?
//
//   waiter: 1 block, spins (bounded by s_memrealtime, ~2 ms) until `flag`
//           becomes 1; records whether it saw it.
//   setter: 1 block, stores flag = 1.
// With the barrier bit set the setter runs only after the waiter timed out
// (seen = 0); with it cleared the setter runs beside the waiter (seen = 1).
// Test D: a 2048-block kernel whose blocks each stream-wait ~20 us, then an
// any-order kernel whose blocks record their start ticks: overlap = how long
// before the first kernel's last block ended the second one started.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void waiter(unsigned* flag, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned seen = 0;
  unsigned long long t = t0;
  while (t - t0 < 200000ull) {   // 100 MHz ticks: 2 ms
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u) {
      seen = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(8);
    t = __builtin_amdgcn_s_memrealtime();
  }
  out[0] = seen;
  out[1] = t - t0;
}

__global__ void setter(unsigned* flag) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Test D kernels.
__global__ void busy(unsigned long long* end_ticks, unsigned ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
  if (threadIdx.x == 0) end_ticks[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

__global__ void stamp(unsigned long long* start_ticks) {
  if (threadIdx.x == 0) start_ticks[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

static void pair_test(const char* name, hipStream_t st, unsigned* flag, unsigned long long* out,
                      int any, bool graph) {
  CHECK(hipMemsetAsync(flag, 0, 4, st));
  CHECK(hipMemsetAsync(out, 0, 16, st));
  CHECK(hipStreamSynchronize(st));
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  if (graph) CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  void* a1[] = {&flag, &out};
  CHECK(hipExtLaunchKernel(reinterpret_cast<const void*>(&waiter), dim3(1), dim3(64), a1, 0, st,
                           nullptr, nullptr, 0));
  void* a2[] = {&flag};
  CHECK(hipExtLaunchKernel(reinterpret_cast<const void*>(&setter), dim3(1), dim3(64), a2, 0, st,
                           nullptr, nullptr, any ? hipExtAnyOrderLaunch : 0));
  if (graph) {
    CHECK(hipStreamEndCapture(st, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHECK(hipGraphLaunch(ge, st));
  }
  CHECK(hipStreamSynchronize(st));
  unsigned long long h[2];
  CHECK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
  printf("%-34s seen=%llu waited=%.1f us\n", name, h[0], h[1] * 0.01);
  if (ge) CHECK(hipGraphExecDestroy(ge));
  if (g) CHECK(hipGraphDestroy(g));
}

int main() {
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned* flag;
  unsigned long long* out;
  CHECK(hipMalloc(&flag, 4));
  CHECK(hipMalloc(&out, 16));
  pair_test("plain launch, same stream", st, flag, out, 0, false);
  pair_test("any-order launch, same stream", st, flag, out, 1, false);
  pair_test("plain launch, graph", st, flag, out, 0, true);
  pair_test("any-order launch, graph", st, flag, out, 1, true);

  const int nb = 2048;
  unsigned long long *ends, *starts;
  CHECK(hipMalloc(&ends, nb * 8));
  CHECK(hipMalloc(&starts, nb * 8));
  for (int any = 0; any < 2; ++any) {
    for (int rep = 0; rep < 3; ++rep) {
      unsigned ticks = 2000;   // 20 us per block
      void* a1[] = {&ends, &ticks};
      void* a2[] = {&starts};
      CHECK(hipExtLaunchKernel(reinterpret_cast<const void*>(&busy), dim3(nb), dim3(256), a1, 0,
                               st, nullptr, nullptr, 0));
      CHECK(hipExtLaunchKernel(reinterpret_cast<const void*>(&stamp), dim3(nb), dim3(256), a2, 0,
                               st, nullptr, nullptr, any ? hipExtAnyOrderLaunch : 0));
      CHECK(hipStreamSynchronize(st));
      static unsigned long long he[nb], hs[nb];
      CHECK(hipMemcpy(he, ends, sizeof(he), hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(hs, starts, sizeof(hs), hipMemcpyDeviceToHost));
      unsigned long long emax = 0, emin = ~0ull, smin = ~0ull, smax = 0;
      for (int i = 0; i < nb; ++i) {
        emax = he[i] > emax ? he[i] : emax;
        emin = he[i] < emin ? he[i] : emin;
        smin = hs[i] < smin ? hs[i] : smin;
        smax = hs[i] > smax ? hs[i] : smax;
      }
      printf("busy(2048 x 20us) then stamp, %s: first busy end +0, last busy end %+.1f us, "
             "first stamp %+.1f us, last stamp %+.1f us\n",
             any ? "any-order" : "plain    ", (emax - emin) * 0.01,
             ((double)smin - (double)emin) * 0.01, ((double)smax - (double)emin) * 0.01);
    }
  }
  CHECK(hipFree(ends));
  CHECK(hipFree(starts));
  CHECK(hipFree(flag));
  CHECK(hipFree(out));
  CHECK(hipStreamDestroy(st));
  return 0;
}
