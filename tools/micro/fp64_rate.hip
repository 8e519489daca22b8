// fp64 VALU issue-rate microbenchmark (developer tool): independent FMA
// chains per lane, variants with VGPR / SGPR / inline-constant operands,
// v_mul_f64, v_add_f64, and a mixed chain with v_rcp_f64.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int CH, int MODE>
__global__ __launch_bounds__(256) void k(double* out, double a, double b, int iters) {
  double x[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) x[j] = threadIdx.x * 1e-3 + j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if constexpr (MODE == 0) {  // v_fma_f64 all-VGPR: x = x*x2 + x3 (keeps 3 vgpr operands)
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[j]) : "v"(x[(j + 1) % CH]), "v"(x[(j + 2) % CH]));
      } else if constexpr (MODE == 1) {  // VOP3 with SGPR coefficient
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[j]) : "v"(x[(j + 1) % CH]), "s"(a));
      } else if constexpr (MODE == 2) {  // v_mul_f64
        asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x[j]) : "v"(x[(j + 1) % CH]));
      } else if constexpr (MODE == 3) {  // v_add_f64
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[j]) : "v"(x[(j + 1) % CH]));
      } else if constexpr (MODE == 4) {  // v_fmac_f64 (VOP2)
        asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(x[j]) : "v"(x[(j + 1) % CH]), "v"(x[(j + 2) % CH]));
      } else if constexpr (MODE == 5) {  // fp32 fma for comparison
        float f = (float)x[j];
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f) : "v"(f), "v"(f));
        x[j] = f;
      } else {  // v_rcp_f64
        asm volatile("v_rcp_f64 %0, %0" : "+v"(x[j]));
      }
    }
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < CH; ++j) s += x[j];
  if (s == 1.2345) out[blockIdx.x] = s;
}

template <int CH, int MODE>
void run(const char* name, int blocks_per_cu) {
  double* out;
  hipMalloc(&out, 1 << 20);
  const int blocks = 256 * blocks_per_cu, iters = 2000;
  k<CH, MODE><<<blocks, 256>>>(out, 1.0000001, 0.5, 10);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  k<CH, MODE><<<blocks, 256>>>(out, 1.0000001, 0.5, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double wave_instr = (double)blocks * 4 * iters * CH;       // wave64 instructions
  const double per_simd = wave_instr / 1024.0;
  const double ns = ms * 1e6;
  printf("%-12s chains=%d blocks/CU=%d: %.3f ms, %.2f ns per wave-instr per SIMD (%.2f cycles @2.4GHz)\n",
         name, CH, blocks_per_cu, ms, ns / per_simd, ns / per_simd * 2.4);
  hipFree(out);
}

int main() {
  for (int occ : {1, 2, 4}) {
    run<8, 0>("fma_vvv", occ);
    run<8, 1>("fma_vvs", occ);
    run<8, 4>("fmac", occ);
    run<8, 2>("mul", occ);
    run<8, 3>("add", occ);
    run<8, 5>("fma_f32", occ);
    run<8, 6>("rcp_f64", occ);
  }
  run<2, 1>("fma_vvs", 4);
  run<4, 1>("fma_vvs", 4);
  run<2, 1>("fma_vvs", 8);
  return 0;
}
