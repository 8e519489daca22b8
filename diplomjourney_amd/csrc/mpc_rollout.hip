// mpc_rollout.hip — MI355X (gfx950) kernels + C ABI for the MPC candidate
// expansion of ShittyWizard/DiplomJourney (math_model_tree.py:278-362).
//
// Kernels
//   k_rollout_argmin   one lane per candidate (CPL=2: two adjacent candidates
//                      per lane so each control load is 16 B/lane = 1 KiB per
//                      wave-instruction), N-step rollout in registers, terminal
//                      cost, lane -> wave (shuffle) -> block (LDS) lexicographic
//                      (cost, index) arg-min, one 16-B record per block.
//   k_finalize         one block: arg-min over the block records, then one lane
//                      re-rolls the winner to emit its per-step trajectory
//                      (bitwise the same arithmetic as the rollout lane).
//   k_rollout_argmin_batched / k_finalize_batched   robot-segmented variant.
//   k_select_winner    lexicographic min over gathered per-rank results.
//   k_sample_controls  synthetic control sequences (splitmix64 -> grid entry).
//
// HBM traffic of k_rollout_argmin: 16 B per candidate-step read once
// (v, beta fp64 SoA), 16 B per block written.  See DESIGN.md for the roofline.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "../../include/mpc_rollout.h"
#include "mpc_device.h"

namespace mpc {
namespace {

constexpr int kBlock = 256;           // 4 waves of 64
// Build-time tuning knobs (A/B-tested with tools/probe_gpu.py variants):
#ifndef MPC_CPL
#define MPC_CPL 2            // candidates per lane on the aligned path (2 or 4)
#endif
#ifndef MPC_UNROLL_STEPS
#define MPC_UNROLL_STEPS 0   // 1: fully unroll compile-time horizons
#endif
#ifndef MPC_MIN_WAVES
#define MPC_MIN_WAVES 1      // __launch_bounds__ minimum waves per SIMD
#endif
constexpr int kCplWide = MPC_CPL;
static_assert(kCplWide == 2 || kCplWide == 4, "MPC_CPL must be 2 or 4");
constexpr int kWaves = kBlock / 64;
constexpr int64_t kMaxBlocks = 2048;  // 256 CUs x 8 resident blocks upper bound
constexpr int kFinBlock = 1024;

struct Rec {
  uint64_t key;
  int64_t idx;
};

// ---------------------------------------------------------------------------
// Block-level arg-min: wave shuffle, then the kWaves wave records via LDS.
// Returns the block winner in thread 0.
__device__ __forceinline__ void block_argmin(uint64_t& k, int64_t& i) {
  __shared__ uint64_t s_key[kWaves];
  __shared__ int64_t s_idx[kWaves];
  wave_argmin(k, i);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    s_key[wave] = k;
    s_idx[wave] = i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 1; w < kWaves; ++w)
      if (rec_less(s_key[w], s_idx[w], k, i)) {
        k = s_key[w];
        i = s_idx[w];
      }
  }
}

// Rollout of CPL adjacent candidates starting at column c0 (local index).
// NS > 0: compile-time horizon (fully unrolled); NS == 0: runtime n_steps.
template <int NS, int CPL, int INTEG, bool STATES>
__device__ __forceinline__ void rollout_lane(const Consts& K, const double* __restrict__ v,
                                             const double* __restrict__ b, int64_t ld, int64_t c0,
                                             int n_steps, double (&cst)[CPL],
                                             double* __restrict__ states, int64_t n_cand) {
  double x[CPL], y[CPL], ph[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    x[j] = K.x;
    y[j] = K.y;
    ph[j] = K.phi;
  }
  // Controls of step sr for this lane's CPL candidates: 16 B per lane per
  // array on the wide path (one 1 KiB wave-instruction each).
  auto load = [&](int sr, double (&vv)[CPL], double (&bb)[CPL]) {
    if constexpr (CPL >= 2) {
#pragma unroll
      for (int h = 0; h < CPL; h += 2) {
        const double2 v2 = *reinterpret_cast<const double2*>(v + sr * ld + c0 + h);
        const double2 b2 = *reinterpret_cast<const double2*>(b + sr * ld + c0 + h);
        vv[h] = v2.x;
        vv[h + 1] = v2.y;
        bb[h] = b2.x;
        bb[h + 1] = b2.y;
      }
    } else {
      vv[0] = v[sr * ld + c0];
      bb[0] = b[sr * ld + c0];
    }
  };
  auto body = [&](int sr, const double (&vv)[CPL], const double (&bb)[CPL]) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      step<INTEG>(x[j], y[j], ph[j], vv[j], bb[j], K);
      if constexpr (STATES) {
        states[(sr * 3 + 0) * n_cand + c0 + j] = x[j];
        states[(sr * 3 + 1) * n_cand + c0 + j] = y[j];
        states[(sr * 3 + 2) * n_cand + c0 + j] = ph[j];
      }
    }
  };
  double va[CPL], ba[CPL], vb[CPL], bb_[CPL];
  load(0, va, ba);
  if constexpr (NS > 0 && MPC_UNROLL_STEPS) {
#pragma unroll
    for (int s = 0; s < NS; s += 2) {
      if (s + 1 < NS) load(s + 1, vb, bb_);
      body(s, va, ba);
      if (s + 1 < NS) {
        if (s + 2 < NS) load(s + 2, va, ba);
        body(s + 1, vb, bb_);
      }
    }
  } else {
    const int ns = NS > 0 ? NS : n_steps;
    // Software pipeline, two steps per trip (ping-pong registers, no copies):
    // the next step's controls are in flight while this step's trig chain runs.
#pragma unroll 1
    for (int s = 0; s < ns; s += 2) {
      if (s + 1 < ns) load(s + 1, vb, bb_);
      body(s, va, ba);
      if (s + 1 < ns) {
        if (s + 2 < ns) load(s + 2, va, ba);
        body(s + 1, vb, bb_);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < CPL; ++j) cst[j] = cost(x[j], y[j], K);
}

template <int NS, int CPL, int INTEG, bool STATES>
__global__ __launch_bounds__(kBlock, MPC_MIN_WAVES) void k_rollout_argmin(Consts K, const double* __restrict__ v,
                                                           const double* __restrict__ b,
                                                           int64_t n_cand, int n_steps,
                                                           int64_t n_tiles, Rec* __restrict__ part,
                                                           double* __restrict__ states) {
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t c0 = tile * (kBlock * CPL) + threadIdx.x * CPL;
    if (c0 < n_cand) {  // CPL > 1 requires n_cand % CPL == 0: the whole group is valid
      double cst[CPL];
      rollout_lane<NS, CPL, INTEG, STATES>(K, v, b, n_cand, c0, n_steps, cst, states, n_cand);
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const uint64_t kk = cost_key(cst[j]);
        if (kk < best_k) {  // ascending index per lane: strict < keeps the first
          best_k = kk;
          best_i = c0 + j;
        }
      }
    }
  }
  block_argmin(best_k, best_i);
  if (threadIdx.x == 0) part[blockIdx.x] = Rec{best_k, best_i};
}

// Re-roll the winner and fill the result record.  Called by ALL threads of
// the block once thread 0 holds the winner (key, col).  The N-step recurrence
// is split so that only additions stay serial: lane s computes the state-free
// heading increment dphi_s = Q((v_s/L) tan(beta_s)); lane 0 accumulates the
// headings phi_s = phi_{s-1} + dphi_s; lane s evaluates sincos(phi_s) and the
// two position increments; lane 0 accumulates x and y.  Every operation and
// every accumulation order is that of step<INTEG>(), so the emitted states
// are bitwise those the arg-min scored, at ~3N dependent adds of latency
// instead of N dependent trig chains.
template <int INTEG>
__device__ void emit_winner(const Consts& K, const double* __restrict__ v,
                            const double* __restrict__ b, int64_t ld, int n_steps, uint64_t key,
                            int64_t col, int64_t reported_index, double incumbent,
                            mpc_result_t* __restrict__ out) {
  __shared__ double s_dphi[MPC_MAX_STEPS], s_phi[MPC_MAX_STEPS];
  __shared__ double s_dx[MPC_MAX_STEPS], s_dy[MPC_MAX_STEPS], s_v0, s_b0;
  __shared__ uint64_t s_key;
  __shared__ int64_t s_col, s_rep;
  if (threadIdx.x == 0) {
    s_key = key;
    s_col = col;
    s_rep = reported_index;
  }
  __syncthreads();
  key = s_key;
  col = s_col;
  const int lane = threadIdx.x;
  double vs = 0.0;
  if (key != ~0ull && lane < n_steps) {
    vs = v[lane * ld + col];
    const double bs = b[lane * ld + col];
    if (lane == 0) {
      s_v0 = vs;
      s_b0 = bs;
    }
    const double w = K.L_pow2 ? vs * K.inv_L : vs / K.L;
    s_dphi[lane] = quad_const<INTEG>(w * trig::tan_fast(bs), K);
  }
  __syncthreads();
  if (lane == 0 && key != ~0ull) {
    double ph = K.phi;
    for (int st = 0; st < n_steps; ++st) {
      ph = ph + s_dphi[st];
      s_phi[st] = ph;
    }
  }
  __syncthreads();
  if (key != ~0ull && lane < n_steps) {
    double sn, cs;
    trig::sincos_fast(s_phi[lane], &sn, &cs);
    s_dx[lane] = quad_const<INTEG>(vs * cs, K);
    s_dy[lane] = quad_const<INTEG>(vs * sn, K);
  }
  __syncthreads();
  if (lane != 0) return;
  out->n_steps = n_steps;
  if (key == ~0ull) {
    out->cost = __builtin_inf();
    out->index = -1;
    out->found = 0;
    out->v = 0.0;
    out->beta = 0.0;
    return;
  }
  const double c = key_cost(key);
  out->cost = c;
  out->index = s_rep;
  out->found = c < incumbent ? 1 : 0;
  out->v = s_v0;
  out->beta = s_b0;
  double x = K.x, y = K.y;
  for (int st = 0; st < n_steps; ++st) {
    x = x + s_dx[st];
    y = y + s_dy[st];
    out->traj[st][0] = x;
    out->traj[st][1] = y;
    out->traj[st][2] = s_phi[st];
  }
}

template <int INTEG>
__global__ __launch_bounds__(kFinBlock) void k_finalize(const Rec* __restrict__ part, int n_part,
                                                        Consts K, const double* __restrict__ v,
                                                        const double* __restrict__ b,
                                                        int64_t n_cand, int n_steps,
                                                        int64_t index_base, double incumbent,
                                                        mpc_result_t* __restrict__ out) {
  __shared__ uint64_t s_key[kFinBlock / 64];
  __shared__ int64_t s_idx[kFinBlock / 64];
  uint64_t k = ~0ull;
  int64_t i = INT64_MAX;
  for (int p = threadIdx.x; p < n_part; p += kFinBlock)
    if (rec_less(part[p].key, part[p].idx, k, i)) {
      k = part[p].key;
      i = part[p].idx;
    }
  wave_argmin(k, i);
  if ((threadIdx.x & 63) == 0) {
    s_key[threadIdx.x >> 6] = k;
    s_idx[threadIdx.x >> 6] = i;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kFinBlock / 64; ++w)
      if (rec_less(s_key[w], s_idx[w], k, i)) {
        k = s_key[w];
        i = s_idx[w];
      }
  }
  emit_winner<INTEG>(K, v, b, n_cand, n_steps, k, i, index_base + i, incumbent, out);
}

// --------------------------- batched robots --------------------------------
__device__ __forceinline__ Consts consts_from_problem(const mpc_problem_t& p) {
  Consts K;
  K.x = p.x;
  K.y = p.y;
  K.phi = p.phi;
  K.x_t = p.x_t;
  K.y_t = p.y_t;
  K.x_0 = p.x_0;
  K.y_0 = p.y_0;
  K.A = p.y_t - p.y_0;
  K.B = p.x_t - p.x_0;
  K.C1 = p.x_t * p.y_0;
  K.C2 = p.y_t * p.x_0;
  // Device squares are x*x (glibc pow(x, 2.0) differs by 1 ulp in ~0.1% of
  // inputs); the single-problem path derives this on the host with libm pow.
  K.den = sqrt(K.A * K.A + K.B * K.B);
  K.L = p.L;
  int e;
  const double m = frexp(p.L, &e);
  K.L_pow2 = (m == 0.5) ? 1 : 0;
  K.inv_L = K.L_pow2 ? 1.0 / p.L : 0.0;
  K.h = p.t_b - p.t_a;
  K.hlgth = 0.5 * (p.t_b - p.t_a);
  K.pad_ = 0;
  return K;
}

template <int NS, int CPL, int INTEG>
__global__ __launch_bounds__(kBlock, MPC_MIN_WAVES) void k_rollout_argmin_batched(
    const mpc_problem_t* __restrict__ probs, const double* __restrict__ v,
    const double* __restrict__ b, int64_t cand, int n_steps, int64_t ld, Rec* __restrict__ part) {
  const int r = blockIdx.y;
  const Consts K = consts_from_problem(probs[r]);
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  const int64_t tiles = (cand + kBlock * CPL - 1) / (kBlock * CPL);
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int64_t cl = tile * (kBlock * CPL) + threadIdx.x * CPL;  // local index
    if (cl < cand) {
      double cst[CPL];
      rollout_lane<NS, CPL, INTEG, false>(K, v, b, ld, r * cand + cl, n_steps, cst, nullptr, 0);
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const uint64_t kk = cost_key(cst[j]);
        if (kk < best_k) {
          best_k = kk;
          best_i = cl + j;
        }
      }
    }
  }
  block_argmin(best_k, best_i);
  if (threadIdx.x == 0) part[static_cast<int64_t>(r) * gridDim.x + blockIdx.x] = Rec{best_k, best_i};
}

template <int INTEG>
__global__ __launch_bounds__(kBlock) void k_finalize_batched(
    const Rec* __restrict__ part, int n_part, const mpc_problem_t* __restrict__ probs,
    const double* __restrict__ incumbents, const double* __restrict__ v,
    const double* __restrict__ b, int64_t cand, int n_steps, int64_t ld,
    mpc_result_t* __restrict__ out) {
  const int r = blockIdx.x;
  uint64_t k = ~0ull;
  int64_t i = INT64_MAX;
  for (int p = threadIdx.x; p < n_part; p += kBlock) {
    const Rec q = part[static_cast<int64_t>(r) * n_part + p];
    if (rec_less(q.key, q.idx, k, i)) {
      k = q.key;
      i = q.idx;
    }
  }
  block_argmin(k, i);
  const Consts K = consts_from_problem(probs[r]);
  const double inc = incumbents ? incumbents[r] : __builtin_inf();
  emit_winner<INTEG>(K, v, b, ld, n_steps, k, r * cand + i, i, inc, &out[r]);
}

// --------------------------- exchange + sampler ----------------------------
__global__ void k_select_winner(const mpc_result_t* __restrict__ res, int n, double incumbent,
                                mpc_result_t* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int best = 0;
  uint64_t bk = ~0ull;
  int64_t bi = INT64_MAX;
  for (int r = 0; r < n; ++r) {
    const uint64_t k = res[r].index < 0 ? ~0ull : cost_key(res[r].cost);
    const int64_t i = res[r].index < 0 ? INT64_MAX : res[r].index;
    if (r == 0 || rec_less(k, i, bk, bi)) {
      best = r;
      bk = k;
      bi = i;
    }
  }
  *out = res[best];
  out->found = (bk != ~0ull && out->cost < incumbent) ? 1 : 0;
}

// Grid entry of one (step, candidate): candidate g < n_grid of the constant
// prefix is the reference's enumeration k = g; otherwise the top 32 bits of
// splitmix64(seed ^ s<<40 ^ g) are mapped onto [0, n_grid) by multiply-shift
// (Lemire's fastrange: no integer division on the VALU).
__device__ __forceinline__ uint32_t grid_entry(uint64_t seed, int s, uint64_t g, uint32_t n_grid,
                                               int cprefix) {
  if (cprefix && g < n_grid) return static_cast<uint32_t>(g);
  const uint64_t h = splitmix64(seed ^ (static_cast<uint64_t>(s) << 40) ^ g);
  return static_cast<uint32_t>(((h >> 32) * static_cast<uint64_t>(n_grid)) >> 32);
}

constexpr int kSampleLdsEntries = 2048;  // expanded (v, beta) grid staged in LDS

// One thread per candidate pair (16-B stores), looping over the steps.  The
// grid |V| x |B| (<= 451 entries for the reference's acceleration limits) is
// expanded once per block into LDS, so the per-element lookup is one
// ds_read_b128 instead of a division by |B| and two global loads.
__global__ __launch_bounds__(kBlock) void k_sample_controls(
    const double* __restrict__ vg, int nv, const double* __restrict__ bg, int nb, int64_t n_cand,
    int n_steps, uint64_t seed, int64_t base, int cprefix, double* __restrict__ v,
    double* __restrict__ b, int64_t ld, int pairs) {
  __shared__ double2 s_grid[kSampleLdsEntries];
  const uint32_t n_grid = static_cast<uint32_t>(nv) * static_cast<uint32_t>(nb);
  const bool in_lds = n_grid <= kSampleLdsEntries;
  if (in_lds) {
    for (uint32_t k = threadIdx.x; k < n_grid; k += kBlock)
      s_grid[k] = make_double2(vg[k / nb], bg[k % nb]);
    __syncthreads();
  }
  auto lookup = [&](uint32_t k) -> double2 {
    return in_lds ? s_grid[k] : make_double2(vg[k / nb], bg[k % nb]);
  };
  const int cpt = pairs ? 2 : 1;
  const int64_t n_items = n_cand / cpt;
  for (int64_t it = blockIdx.x * static_cast<int64_t>(kBlock) + threadIdx.x; it < n_items;
       it += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t c = it * cpt;
    const uint64_t g = static_cast<uint64_t>(base + c);
    for (int st = 0; st < n_steps; ++st) {
      const double2 e0 = lookup(grid_entry(seed, st, g, n_grid, cprefix));
      if (pairs) {
        const double2 e1 = lookup(grid_entry(seed, st, g + 1, n_grid, cprefix));
        *reinterpret_cast<double2*>(v + st * ld + c) = make_double2(e0.x, e1.x);
        *reinterpret_cast<double2*>(b + st * ld + c) = make_double2(e0.y, e1.y);
      } else {
        v[st * ld + c] = e0.x;
        b[st * ld + c] = e0.y;
      }
    }
  }
}

// ------------------------------- host side ---------------------------------
// libm pow through a volatile pointer: the compiler must not fold pow(x, 2.0)
// into x*x (Python's `a ** 2` is libm pow, which is not always x*x).
double (*volatile g_libm_pow)(double, double) = pow;

Consts host_consts(const mpc_problem_t& p) {
  Consts K;
  memset(&K, 0, sizeof(K));
  K.x = p.x;
  K.y = p.y;
  K.phi = p.phi;
  K.x_t = p.x_t;
  K.y_t = p.y_t;
  K.x_0 = p.x_0;
  K.y_0 = p.y_0;
  K.A = p.y_t - p.y_0;
  K.B = p.x_t - p.x_0;
  K.C1 = p.x_t * p.y_0;
  K.C2 = p.y_t * p.x_0;
  K.den = sqrt(g_libm_pow(K.A, 2.0) + g_libm_pow(K.B, 2.0));
  K.L = p.L;
  int e;
  K.L_pow2 = (frexp(p.L, &e) == 0.5) ? 1 : 0;
  K.inv_L = K.L_pow2 ? 1.0 / p.L : 0.0;
  K.h = p.t_b - p.t_a;
  K.hlgth = 0.5 * (p.t_b - p.t_a);
  return K;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline int64_t rollout_blocks(int64_t n_cand) {
  // CPL=1 tiling has the most tiles; the workspace is sized for it.
  return std::max<int64_t>(1, std::min<int64_t>(cdiv(n_cand, kBlock), kMaxBlocks));
}

template <int NS, int CPL, int INTEG>
void launch_fixed(dim3 grid, hipStream_t st, const Consts& K, const double* v, const double* b,
                  int64_t n_cand, int n_steps, int64_t tiles, Rec* part) {
  k_rollout_argmin<NS, CPL, INTEG, false>
      <<<grid, kBlock, 0, st>>>(K, v, b, n_cand, n_steps, tiles, part, nullptr);
}

template <int CPL, int INTEG>
void launch_by_steps(dim3 grid, hipStream_t st, const Consts& K, const double* v, const double* b,
                     int64_t n_cand, int n_steps, int64_t tiles, Rec* part) {
  switch (n_steps) {
    case 3: launch_fixed<3, CPL, INTEG>(grid, st, K, v, b, n_cand, n_steps, tiles, part); break;
    case 8: launch_fixed<8, CPL, INTEG>(grid, st, K, v, b, n_cand, n_steps, tiles, part); break;
    case 10: launch_fixed<10, CPL, INTEG>(grid, st, K, v, b, n_cand, n_steps, tiles, part); break;
    case 12: launch_fixed<12, CPL, INTEG>(grid, st, K, v, b, n_cand, n_steps, tiles, part); break;
    default: launch_fixed<0, CPL, INTEG>(grid, st, K, v, b, n_cand, n_steps, tiles, part); break;
  }
}

template <int CPL, int INTEG>
void launch_batched_by_steps(dim3 grid, hipStream_t st, const mpc_problem_t* probs,
                             const double* v, const double* b, int64_t cand, int n_steps,
                             int64_t ld, Rec* part) {
#define MPC_BATCHED(NS) \
  k_rollout_argmin_batched<NS, CPL, INTEG><<<grid, kBlock, 0, st>>>(probs, v, b, cand, n_steps, ld, part)
  switch (n_steps) {
    case 3: MPC_BATCHED(3); break;
    case 8: MPC_BATCHED(8); break;
    case 10: MPC_BATCHED(10); break;
    case 12: MPC_BATCHED(12); break;
    default: MPC_BATCHED(0); break;
  }
#undef MPC_BATCHED
}

int last_hip_status() { return hipGetLastError() == hipSuccess ? MPC_OK : MPC_ERR_HIP; }

}  // namespace
}  // namespace mpc

using namespace mpc;

extern "C" {

const char* mpc_version(void) { return "diplomjourney_amd mpc_rollout 0.1 (gfx950)"; }

const char* mpc_strerror(int status) {
  switch (status) {
    case MPC_OK: return "ok";
    case MPC_ERR_ARG: return "invalid argument";
    case MPC_ERR_WORKSPACE: return "workspace too small";
    case MPC_ERR_HIP: return "HIP runtime error";
    case MPC_ERR_UNSUPPORTED: return "unsupported option";
    default: return "unknown status";
  }
}

size_t mpc_workspace_bytes(int64_t n_cand, int32_t n_steps) {
  (void)n_steps;
  if (n_cand < 0) return 0;
  return static_cast<size_t>(rollout_blocks(n_cand)) * sizeof(Rec);
}

// Number of block records phase 1 writes (phase 2 must agree).
static bool wide_ok(const double* v_sc, const double* beta_sc, int64_t n) {
  return (n % kCplWide == 0) && aligned16(v_sc) && aligned16(beta_sc);
}

static int64_t partial_count(const double* v_sc, const double* beta_sc, int64_t n_cand,
                             bool with_states) {
  const bool wide = !with_states && wide_ok(v_sc, beta_sc, n_cand);
  const int64_t tiles = cdiv(n_cand, kBlock * (wide ? kCplWide : 1));
  return std::min<int64_t>(tiles, kMaxBlocks);
}

static int check_args(const mpc_problem_t* p, const double* v_sc, const double* beta_sc,
                      int64_t n_cand, int32_t n_steps, int32_t integrator, void* ws,
                      size_t ws_bytes) {
  if (!p || n_cand < 1 || n_steps < 1 || n_steps > MPC_MAX_STEPS || !v_sc || !beta_sc)
    return MPC_ERR_ARG;
  if (integrator != MPC_INTEG_QK21 && integrator != MPC_INTEG_RECT) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  return MPC_OK;
}

int mpc_rollout_partials(const mpc_problem_t* p, const double* v_sc, const double* beta_sc,
                         int64_t n_cand, int32_t n_steps, int32_t integrator, double* states_out,
                         void* ws, size_t ws_bytes, mpc_stream_t stream) {
  const int a = check_args(p, v_sc, beta_sc, n_cand, n_steps, integrator, ws, ws_bytes);
  if (a != MPC_OK) return a;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const Consts K = host_consts(*p);
  Rec* part = static_cast<Rec*>(ws);
  const bool rect = integrator == MPC_INTEG_RECT;
  const int64_t grid = partial_count(v_sc, beta_sc, n_cand, states_out != nullptr);
  if (states_out) {
    // CoordinateTree materialisation path: runtime horizon, one candidate/lane.
    const int64_t tiles = cdiv(n_cand, kBlock);
    if (rect)
      k_rollout_argmin<0, 1, MPC_INTEG_RECT, true>
          <<<grid, kBlock, 0, st>>>(K, v_sc, beta_sc, n_cand, n_steps, tiles, part, states_out);
    else
      k_rollout_argmin<0, 1, MPC_INTEG_QK21, true>
          <<<grid, kBlock, 0, st>>>(K, v_sc, beta_sc, n_cand, n_steps, tiles, part, states_out);
  } else {
    const bool wide = wide_ok(v_sc, beta_sc, n_cand);
    const int64_t tiles = cdiv(n_cand, kBlock * (wide ? kCplWide : 1));
    if (wide) {
      if (rect) launch_by_steps<kCplWide, MPC_INTEG_RECT>(grid, st, K, v_sc, beta_sc, n_cand, n_steps, tiles, part);
      else launch_by_steps<kCplWide, MPC_INTEG_QK21>(grid, st, K, v_sc, beta_sc, n_cand, n_steps, tiles, part);
    } else {
      if (rect) launch_by_steps<1, MPC_INTEG_RECT>(grid, st, K, v_sc, beta_sc, n_cand, n_steps, tiles, part);
      else launch_by_steps<1, MPC_INTEG_QK21>(grid, st, K, v_sc, beta_sc, n_cand, n_steps, tiles, part);
    }
  }
  return last_hip_status();
}

int mpc_rollout_finalize(const mpc_problem_t* p, const double* v_sc, const double* beta_sc,
                         int64_t n_cand, int32_t n_steps, int64_t index_base, double incumbent,
                         int32_t integrator, int32_t with_states, void* ws, size_t ws_bytes,
                         mpc_result_t* out, mpc_stream_t stream) {
  const int a = check_args(p, v_sc, beta_sc, n_cand, n_steps, integrator, ws, ws_bytes);
  if (a != MPC_OK) return a;
  if (!out || index_base < 0) return MPC_ERR_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const Consts K = host_consts(*p);
  const Rec* part = static_cast<const Rec*>(ws);
  const int n_part = static_cast<int>(partial_count(v_sc, beta_sc, n_cand, with_states != 0));
  if (integrator == MPC_INTEG_RECT)
    k_finalize<MPC_INTEG_RECT><<<1, kFinBlock, 0, st>>>(part, n_part, K, v_sc, beta_sc, n_cand,
                                                        n_steps, index_base, incumbent, out);
  else
    k_finalize<MPC_INTEG_QK21><<<1, kFinBlock, 0, st>>>(part, n_part, K, v_sc, beta_sc, n_cand,
                                                        n_steps, index_base, incumbent, out);
  return last_hip_status();
}

int mpc_rollout_argmin(const mpc_problem_t* p, const double* v_sc, const double* beta_sc,
                       int64_t n_cand, int32_t n_steps, int64_t index_base, double incumbent,
                       int32_t integrator, double* states_out, void* ws, size_t ws_bytes,
                       mpc_result_t* out, mpc_stream_t stream) {
  if (!out || index_base < 0) return MPC_ERR_ARG;
  const int a = mpc_rollout_partials(p, v_sc, beta_sc, n_cand, n_steps, integrator, states_out,
                                     ws, ws_bytes, stream);
  if (a != MPC_OK) return a;
  return mpc_rollout_finalize(p, v_sc, beta_sc, n_cand, n_steps, index_base, incumbent,
                              integrator, states_out != nullptr, ws, ws_bytes, out, stream);
}

size_t mpc_batched_workspace_bytes(int32_t n_problems, int64_t cand_per_problem, int32_t n_steps) {
  (void)n_steps;
  if (n_problems < 0 || cand_per_problem < 0) return 0;
  return static_cast<size_t>(n_problems) * static_cast<size_t>(rollout_blocks(cand_per_problem)) *
         sizeof(Rec);
}

int mpc_rollout_argmin_batched(const mpc_problem_t* problems, const double* incumbents,
                               int32_t n_problems, const double* v_sc, const double* beta_sc,
                               int64_t cand_per_problem, int32_t n_steps, int32_t integrator,
                               void* ws, size_t ws_bytes, mpc_result_t* out, mpc_stream_t stream) {
  if (!problems || !out || !v_sc || !beta_sc || n_problems < 1 || n_problems > 65535 ||
      cand_per_problem < 1 || n_steps < 1 || n_steps > MPC_MAX_STEPS)
    return MPC_ERR_ARG;
  if (integrator != MPC_INTEG_QK21 && integrator != MPC_INTEG_RECT) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_batched_workspace_bytes(n_problems, cand_per_problem, n_steps))
    return MPC_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t ld = static_cast<int64_t>(n_problems) * cand_per_problem;
  const bool pair = wide_ok(v_sc, beta_sc, cand_per_problem) &&
                    (static_cast<int64_t>(n_problems) * cand_per_problem) % kCplWide == 0;
  const int cpl = pair ? kCplWide : 1;
  const int64_t tiles = cdiv(cand_per_problem, kBlock * cpl);
  const int64_t per_robot = std::min<int64_t>(tiles, rollout_blocks(cand_per_problem));
  const dim3 grid(static_cast<unsigned>(per_robot), static_cast<unsigned>(n_problems));
  Rec* part = static_cast<Rec*>(ws);
  const bool rect = integrator == MPC_INTEG_RECT;
  if (pair) {
    if (rect) launch_batched_by_steps<kCplWide, MPC_INTEG_RECT>(grid, st, problems, v_sc, beta_sc, cand_per_problem, n_steps, ld, part);
    else launch_batched_by_steps<kCplWide, MPC_INTEG_QK21>(grid, st, problems, v_sc, beta_sc, cand_per_problem, n_steps, ld, part);
  } else {
    if (rect) launch_batched_by_steps<1, MPC_INTEG_RECT>(grid, st, problems, v_sc, beta_sc, cand_per_problem, n_steps, ld, part);
    else launch_batched_by_steps<1, MPC_INTEG_QK21>(grid, st, problems, v_sc, beta_sc, cand_per_problem, n_steps, ld, part);
  }
  if (last_hip_status() != MPC_OK) return MPC_ERR_HIP;
  if (rect)
    k_finalize_batched<MPC_INTEG_RECT><<<n_problems, kBlock, 0, st>>>(
        part, static_cast<int>(per_robot), problems, incumbents, v_sc, beta_sc, cand_per_problem,
        n_steps, ld, out);
  else
    k_finalize_batched<MPC_INTEG_QK21><<<n_problems, kBlock, 0, st>>>(
        part, static_cast<int>(per_robot), problems, incumbents, v_sc, beta_sc, cand_per_problem,
        n_steps, ld, out);
  return last_hip_status();
}

int mpc_select_winner(const mpc_result_t* results, int32_t n, double incumbent,
                      mpc_result_t* out, mpc_stream_t stream) {
  if (!results || !out || n < 1) return MPC_ERR_ARG;
  k_select_winner<<<1, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(results, n, incumbent, out);
  return last_hip_status();
}

int mpc_sample_controls(const double* v_grid, int32_t n_v, const double* beta_grid,
                        int32_t n_beta, int64_t n_cand, int32_t n_steps, uint64_t seed,
                        int64_t index_base, int32_t const_prefix, double* v_sc,
                        double* beta_sc, int64_t ld, mpc_stream_t stream) {
  if (!v_grid || !beta_grid || !v_sc || !beta_sc || n_v < 1 || n_beta < 1 || n_cand < 1 ||
      n_steps < 1 || index_base < 0 || ld < n_cand)
    return MPC_ERR_ARG;
  if (static_cast<int64_t>(n_v) * n_beta > 0xFFFFFFFFll) return MPC_ERR_ARG;
  const int pairs = (n_cand % 2 == 0) && (ld % 2 == 0) && aligned16(v_sc) && aligned16(beta_sc);
  const int64_t items = pairs ? n_cand / 2 : n_cand;
  const int64_t grid = std::min<int64_t>(cdiv(items, kBlock), 4096);
  k_sample_controls<<<grid, kBlock, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      v_grid, n_v, beta_grid, n_beta, n_cand, n_steps, seed, index_base, const_prefix, v_sc,
      beta_sc, ld, pairs);
  return last_hip_status();
}

}  // extern "C"
