// v_rcp_f64 accuracy probe (developer tool): over a dense sample of q in
// [0.5, 1] (the denominator range of trig::tan_small is [0.59, 1]) it reports
//   - the largest relative error of the raw estimate, |1 - q*r0|;
//   - how often one Newton step, r1 = fma(r0, fma(-q, r0, 1), r0), differs
//     from the correctly rounded 1/q (the host replica's reciprocal);
//   - the same for r1 formed from the estimate of a product q*q' (the
//     two-candidate shared reciprocal: 1/q = q' * (1/(q*q'))).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k(uint64_t n, unsigned long long* out) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  double worst = 0.0;
  unsigned long long miss1 = 0, miss_pair = 0;
  for (uint64_t j = i; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const double q = 0.5 + 0.5 * ((double)j / (double)n);
    const double r0 = __builtin_amdgcn_rcp(q);
    const double e = fabs(fma(-q, r0, 1.0));
    worst = e > worst ? e : worst;
    const double r1 = fma(r0, fma(-q, r0, 1.0), r0);
    const double cr = 1.0 / q;
    miss1 += (r1 != cr);
    const double q2 = 0.59 + 0.41 * ((double)((j * 2654435761ull) % n) / (double)n);
    const double pr = q * q2;
    double rp = __builtin_amdgcn_rcp(pr);
    rp = fma(rp, fma(-pr, rp, 1.0), rp);
    miss_pair += (rp != 1.0 / pr);
  }
  atomicMax(&out[0], (unsigned long long)__double_as_longlong(worst));
  atomicAdd(&out[1], miss1);
  atomicAdd(&out[2], miss_pair);
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 3 * sizeof(unsigned long long));
  hipMemset(d, 0, 3 * sizeof(unsigned long long));
  const uint64_t n = 1ull << 30;
  k<<<4096, 256>>>(n, d);
  unsigned long long h[3];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  double w;
  __builtin_memcpy(&w, &h[0], 8);
  printf("samples %llu: max |1 - q*rcp(q)| = %.3e (2^%.1f); Newton-1 != 1/q: %llu; "
         "product Newton-1 != 1/(q q'): %llu\n",
         (unsigned long long)n, w, w > 0 ? __builtin_log2(w) : -1e9, h[1], h[2]);
  return 0;
}
