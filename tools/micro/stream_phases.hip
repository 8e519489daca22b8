// stream_phases.hip — where the streaming rollout's time goes, per block:
// s_memrealtime (100 MHz) stamps around the phases of the production device
// code (rollout_lane_glds_k in the rect+cum form the chained step runs, the
// lane -> block arg-min, the record store), one launch among back-to-back
// ones.  Prints, over the blocks of the launch, percentiles of each phase's
// end relative to the first block's entry, and the launch period by events.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -I include -I diplomjourney_amd/csrc -o tools/micro/stream_phases \
//     tools/micro/stream_phases.hip
//   tools/micro/stream_phases N_CAND N_STEPS
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "mpc_kernels.h"

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

using namespace mpc;

constexpr int kStamps = 6;

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

struct Stamp {
  uint64_t* t;
  int q;
  __device__ void operator()() const {
    const uint64_t v = now();
    if (threadIdx.x == 0) t[q] = v;
  }
};

__global__ __launch_bounds__(kBlock, kStreamWaves) void k_phases(
    const Consts* __restrict__ Kdev, const double* __restrict__ v, const double* __restrict__ b,
    int64_t n_cand, int n_steps, Rec* __restrict__ part, uint64_t* __restrict__ stamps) {
  uint64_t* my = stamps + blockIdx.x * kStamps;
  if (threadIdx.x == 0) my[0] = now();
  const Consts K = *Kdev;
  const int64_t c0 = blockIdx.x * (kBlock * 2) + threadIdx.x * 2;
  const int64_t cl = c0 < n_cand ? c0 : n_cand - 2;
  double cst[2];
  rollout_lane_glds_k<MPC_INTEG_RECT, kRotCum, true, Stamp, Stamp, NoPre, false>(
      K, K, v, b, n_cand, cl, n_steps, cst, Stamp{my, 2}, Stamp{my, 1});
  if (threadIdx.x == 0) my[3] = now();
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  if (c0 < n_cand) {
    for (int j = 0; j < 2; ++j) {
      const uint64_t kk = cost_key(cst[j]);
      if (kk < best_k) {
        best_k = kk;
        best_i = c0 + j;
      }
    }
  }
  block_argmin(best_k, best_i);
  if (threadIdx.x == 0) {
    my[4] = now();
    part[blockIdx.x] = Rec{best_k, best_i};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    my[5] = now();
  }
}

__global__ void k_fill(double* v, double* b, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < n) {
    const uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    v[i] = 0.1 + 0.5 * (double)((h >> 11) & 0xfffff) / 1048576.0;
    b[i] = -0.6 + 1.2 * (double)((h >> 33) & 0xfffff) / 1048576.0;
  }
}

__global__ void k_consts(Consts* K) {
  mpc_problem_t p{};
  p.x = 0.1;
  p.y = 0.2;
  p.phi = 0.3;
  p.x_t = 2.0;
  p.y_t = 3.0;
  p.x_0 = 0.0;
  p.y_0 = 0.0;
  p.L = 0.5;
  p.t_a = 0.1;
  p.t_b = 0.2;
  if (threadIdx.x == 0) *K = consts_from_problem(p);
}

static void report(const char* name, const std::vector<uint64_t>& h, int nb) {
  uint64_t t0 = ~0ull;
  for (int i = 0; i < nb; ++i) t0 = std::min(t0, h[i * kStamps]);
  printf("%-8s blocks %d (us after the first entry: p10 / p50 / p90 / max)\n", name, nb);
  const char* names[kStamps] = {"entry", "DMAs issued", "loop end", "cost", "block argmin",
                                "record stored"};
  for (int q = 0; q < kStamps; ++q) {
    std::vector<double> x;
    for (int i = 0; i < nb; ++i) x.push_back((h[i * kStamps + q] - (double)t0) * 0.01);
    std::sort(x.begin(), x.end());
    auto pct = [&](double p) { return x[std::min<size_t>(x.size() - 1, (size_t)(p * x.size()))]; };
    printf("  %-14s %6.2f %6.2f %6.2f %6.2f\n", names[q], pct(0.1), pct(0.5), pct(0.9), x.back());
  }
}

static void run(const char* name, int64_t n, int ns, const Consts* K, const double* v,
                const double* b, Rec* part, uint64_t* stamps, hipStream_t st) {
  const int nb = (int)((n + 2 * kBlock - 1) / (2 * kBlock));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 300; ++i)
    k_phases<<<nb, kBlock, 0, st>>>(K, v, b, n, ns, part, stamps);
  CHECK(hipEventRecord(e0, st));
  for (int i = 0; i < 200; ++i)
    k_phases<<<nb, kBlock, 0, st>>>(K, v, b, n, ns, part, stamps);
  CHECK(hipEventRecord(e1, st));
  CHECK(hipStreamSynchronize(st));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<uint64_t> h(nb * kStamps);
  CHECK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
  printf("launch period %.2f us (200 back-to-back)\n", ms * 1e3 / 200);
  report(name, h, nb);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 100000;
  const int ns = argc > 2 ? atoi(argv[2]) : 3;
  if (n % 2 || n > (1 << 26) || ns < 1 || ns > 32) return 2;
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  double *v, *b;
  Consts* K;
  Rec* part;
  uint64_t* stamps;
  const int nb = (int)((n + 2 * kBlock - 1) / (2 * kBlock));
  CHECK(hipMalloc(&v, n * ns * 8));
  CHECK(hipMalloc(&b, n * ns * 8));
  CHECK(hipMalloc(&K, sizeof(Consts)));
  CHECK(hipMalloc(&part, nb * sizeof(Rec)));
  CHECK(hipMalloc(&stamps, nb * kStamps * 8));
  k_fill<<<(int)((n * ns + 255) / 256), 256, 0, st>>>(v, b, n * ns);
  k_consts<<<1, 64, 0, st>>>(K);
  CHECK(hipStreamSynchronize(st));
  printf("n_cand %lld, N %d, %d blocks (one tile each)\n", (long long)n, ns, nb);
  run("rollout", n, ns, K, v, b, part, stamps, st);
  CHECK(hipFree(v));
  CHECK(hipFree(b));
  CHECK(hipFree(K));
  CHECK(hipFree(part));
  CHECK(hipFree(stamps));
  CHECK(hipStreamDestroy(st));
  return 0;
}
