// cumask.hip — can a CU-masked stream keep CUs free for another stream's
// kernel, eagerly and through a captured HIP graph, and do a graph's two
// branches (fork/join over two streams) run side by side?  (The design
// question behind overlapping the exchange's all_gather with the next
// chained launch: RCCL's kernel needs ~280 registers per wave, which never
// fit beside a chained launch that fills every CU.)
//
//   A  k_where on an unmasked stream: the set of (XCC, SE, CU) that ran blocks
//   B  the same on a stream whose CU mask clears bits 0..7 (cuMask[0] low byte)
//   C  graph captured on the masked stream, launched on the masked stream
//   D  the same graph launched on an unmasked stream
//   E  fork/join graph: branch 1 a 2-ms spinner on the masked stream, branch 2
//      (second stream, unmasked) one block that records its start; overlap
//      when branch 2 starts before branch 1 ends.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <set>
#include <tuple>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void k_where(uint32_t* out) {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  // a short busy wait so that the grid spreads over every available CU
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 200) {}
  if (threadIdx.x == 0) out[blockIdx.x] = ((xcc & 0xf) << 16) | (hw & 0xffff);
}

__global__ void k_spin(uint64_t* t) {   // ~2 ms, records start and end
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 200000) {}
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    t[0] = t0;
    t[1] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ void k_stamp(uint64_t* t) {
  if (threadIdx.x == 0) t[2] = __builtin_amdgcn_s_memrealtime();
}

static std::set<std::tuple<int, int, int>> cus(const uint32_t* h, int n) {
  std::set<std::tuple<int, int, int>> s;
  for (int i = 0; i < n; ++i) {
    const uint32_t v = h[i];
    s.insert({int(v >> 16), int((v >> 13) & 7), int((v >> 8) & 0xf)});   // XCC, SE, CU
  }
  return s;
}

int main() {
  const int nb = 8192;
  uint32_t* d;
  CHECK(hipMalloc(&d, nb * 4));
  std::vector<uint32_t> h(nb);
  hipStream_t plain, masked, other;
  CHECK(hipStreamCreate(&plain));
  CHECK(hipStreamCreate(&other));
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<uint32_t> mask((ncu + 31) / 32, 0xffffffffu);
  mask[0] &= ~0xffu;   // clear logical CUs 0..7
  CHECK(hipExtStreamCreateWithCUMask(&masked, static_cast<uint32_t>(mask.size()), mask.data()));
  auto run = [&](hipStream_t s, const char* name, std::set<std::tuple<int, int, int>>* keep) {
    CHECK(hipMemsetAsync(d, 0xff, nb * 4, s));
    k_where<<<nb, 64, 0, s>>>(d);
    CHECK(hipStreamSynchronize(s));
    CHECK(hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost));
    auto c = cus(h.data(), nb);
    printf("%s: %zu distinct CUs\n", name, c.size());
    if (keep) *keep = c;
  };
  std::set<std::tuple<int, int, int>> all, msk;
  run(plain, "A plain stream", &all);
  run(masked, "B masked stream (bits 0-7 cleared)", &msk);
  std::vector<std::tuple<int, int, int>> missing;
  for (auto& t : all)
    if (!msk.count(t)) missing.push_back(t);
  printf("B: CUs not used on the masked stream:");
  for (auto& t : missing) printf(" (xcc %d se %d cu %d)", std::get<0>(t), std::get<1>(t), std::get<2>(t));
  printf("\n");
  // C / D: a graph captured on the masked stream
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(masked, hipStreamCaptureModeGlobal));
  k_where<<<nb, 64, 0, masked>>>(d);
  CHECK(hipStreamEndCapture(masked, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int pass = 0; pass < 2; ++pass) {
    hipStream_t s = pass == 0 ? masked : plain;
    CHECK(hipMemsetAsync(d, 0xff, nb * 4, s));
    CHECK(hipGraphLaunch(ge, s));
    CHECK(hipStreamSynchronize(s));
    CHECK(hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost));
    auto c = cus(h.data(), nb);
    int hit = 0;
    for (auto& t : missing) hit += c.count(t);
    printf("%s: %zu distinct CUs, %d of the %zu masked-off CUs used\n",
           pass == 0 ? "C graph on masked stream" : "D graph on plain stream", c.size(), hit,
           missing.size());
  }
  // E: fork / join
  uint64_t* t;
  CHECK(hipMalloc(&t, 3 * 8));
  hipEvent_t fork, join;
  CHECK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CHECK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  hipGraph_t g2;
  hipGraphExec_t ge2;
  CHECK(hipStreamBeginCapture(masked, hipStreamCaptureModeGlobal));
  CHECK(hipEventRecord(fork, masked));
  CHECK(hipStreamWaitEvent(other, fork, 0));
  k_spin<<<1024, 256, 0, masked>>>(t);
  k_stamp<<<1, 64, 0, other>>>(t);
  CHECK(hipEventRecord(join, other));
  CHECK(hipStreamWaitEvent(masked, join, 0));
  CHECK(hipStreamEndCapture(masked, &g2));
  CHECK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
  for (int pass = 0; pass < 3; ++pass) {
    CHECK(hipGraphLaunch(ge2, masked));
    CHECK(hipStreamSynchronize(masked));
    uint64_t ht[3];
    CHECK(hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost));
    const double us0 = (double)(int64_t)(ht[2] - ht[0]) / 100.0, us1 = (double)(int64_t)(ht[1] - ht[2]) / 100.0;
    printf("E fork/join graph: branch 2 started %.1f us after branch 1 began, %.1f us before it ended -> %s\n",
           us0, us1, us1 > 0 ? "concurrent" : "serialised");
  }
  // eager fork/join for comparison
  CHECK(hipEventRecord(fork, masked));
  k_spin<<<1024, 256, 0, masked>>>(t);
  CHECK(hipStreamWaitEvent(other, fork, 0));
  k_stamp<<<1, 64, 0, other>>>(t);
  CHECK(hipDeviceSynchronize());
  uint64_t ht[3];
  CHECK(hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost));
  printf("E eager: branch 2 started %.1f us before branch 1 ended\n",
         (double)(int64_t)(ht[1] - ht[2]) / 100.0);
  printf("done\n");
  return 0;
}
