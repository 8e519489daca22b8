// Co-residency probe: how many blocks of a given shape (threads, LDS bytes,
// VGPR budget) are resident at once.  Every block increments a counter and
// then waits (bounded, ~2 ms) for the counter to reach the grid size; the
// largest count any block saw is the number resident together.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/resid tools/micro/resid.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int THREADS, int LDS_BYTES>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_num_vgpr(128)))
k_resid(unsigned* cnt, unsigned* seen, unsigned grid) {
  __shared__ unsigned char pad[LDS_BYTES];
  __shared__ unsigned got;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned c = 0;
    for (int it = 0; it < 20000; ++it) {
      c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (c >= grid) break;
      __builtin_amdgcn_s_sleep(10);
    }
    got = c;
    pad[c % LDS_BYTES] = 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_max(seen, got + pad[0] * 0, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
}

template <int THREADS, int LDS_BYTES>
void run(const char* name, unsigned* d) {
  int per_cu = 0, cus = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)&k_resid<THREADS, LDS_BYTES>,
                                               THREADS, 0);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int per : {1, 2, 3, 4}) {
    unsigned grid = per * cus;
    hipMemset(d, 0, 8);
    k_resid<THREADS, LDS_BYTES><<<grid, THREADS>>>(d, d + 1, grid);
    unsigned h[2];
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("%-28s occupancy-API %d/CU  grid %4u -> max co-resident %u\n", name, per_cu, grid, h[1]);
  }
}

int main() {
  unsigned* d;
  hipMalloc(&d, 64);
  int lds = 0;
  hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 0);
  printf("LDS per CU (attribute): %d\n", lds);
  run<320, 47000>("320 thr, 47 KB LDS", d);
  run<256, 47000>("256 thr, 47 KB LDS", d);
  run<320, 16000>("320 thr, 16 KB LDS", d);
  run<256, 40000>("256 thr, 40 KB LDS", d);
  hipFree(d);
  return 0;
}
