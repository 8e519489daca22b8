// Probe: one wave's latency per dependent instruction (the cost model of the
// chained step's block 0, which is one serial chain of such instructions).
// Each case runs a dependent chain of 256 instructions twice (second pass
// timed, s_memrealtime at 100 MHz) in a single 64-thread block.
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/latency tools/micro/latency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint64_t now() {
  uint64_t t = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return t;
}

#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))
#define R256(x) R64(x) R64(x) R64(x) R64(x)

template <int CASE>
__global__ __launch_bounds__(64) void k_lat(double* io, uint64_t* stamps, int* lds_idx) {
  __shared__ double s[64];
  double a = io[threadIdx.x], b = io[64 + threadIdx.x];
  float f = static_cast<float>(a);
  int li = lds_idx[threadIdx.x];
  s[threadIdx.x] = a;
  __syncthreads();
  uint64_t t[3];
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    t[pass] = now();
    if (CASE == 0) asm volatile(R256("v_fma_f64 %0, %0, %1, %1\n\t") : "+v"(a) : "v"(b));
    if (CASE == 1) asm volatile(R256("v_add_f64 %0, %0, %1\n\t") : "+v"(a) : "v"(b));
    if (CASE == 2) asm volatile(R256("v_fma_f32 %0, %0, %0, 1.0\n\t") : "+v"(f));
    if (CASE == 3) asm volatile(R256("v_rcp_f64 %0, %0\n\t") : "+v"(a));
    if (CASE == 4) asm volatile(R256("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t") : "+v"(f));
    if (CASE == 5) {   // dependent LDS loads: the address comes from the previous load
      asm volatile(R64("ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)\n\t") : "+v"(li));
    }
    if (CASE == 6) {   // v_cmp + v_cndmask chain on 64-bit values (the arg-min's compare/select)
      uint32_t x = li, y = threadIdx.x;
      asm volatile(R64("v_cmp_lt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc\n\t") : "+v"(x) : "v"(y) : "vcc");
      li = x;
    }
  }
  t[2] = now();
  if (threadIdx.x == 0) {
    stamps[0] = t[0];
    stamps[1] = t[1];
    stamps[2] = t[2];
  }
  io[128 + threadIdx.x] = a + f + li + s[(threadIdx.x + 1) & 63];
}

template <int CASE>
void run(const char* what, int n_instr, double* io, uint64_t* st, int* li) {
  double sum = 0;
  const int reps = 30;
  for (int r = 0; r < reps + 3; ++r) {
    k_lat<CASE><<<1, 64>>>(io, st, li);
    uint64_t h[3];
    (void)hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost);
    if (r >= 3) sum += (h[2] - h[1]) * 10.0;   // ns
  }
  const double ns = sum / reps;
  printf("%-44s %7.1f ns per chain of %d = %5.2f ns = %5.1f cycles at 2.4 GHz each\n", what, ns,
         n_instr, ns / n_instr, ns / n_instr * 2.4);
}

int main() {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  double* io;
  uint64_t* st;
  int* li;
  (void)hipMalloc(&io, 4096);
  (void)hipMalloc(&st, 64);
  (void)hipMalloc(&li, 4096);
  (void)hipMemset(io, 0, 4096);
  (void)hipMemset(li, 0, 4096);   // LDS chain: address 0 -> value 0 -> address 0 ...
  run<0>("dependent v_fma_f64", 256, io, st, li);
  run<1>("dependent v_add_f64", 256, io, st, li);
  run<2>("dependent v_fma_f32", 256, io, st, li);
  run<3>("dependent v_rcp_f64", 256, io, st, li);
  run<4>("dependent v_mov_b32_dpp", 256, io, st, li);
  run<5>("dependent ds_read_b32 + waitcnt", 64, io, st, li);
  run<6>("v_cmp_lt_u32 + v_cndmask_b32 pair", 64, io, st, li);
  return 0;
}
