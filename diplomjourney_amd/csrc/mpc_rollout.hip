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

// KDEV: the problem constants come from device memory (the device-resident
// episode writes them; no host round-trip) instead of the kernel arguments.
template <int NS, int CPL, int INTEG, bool STATES, bool KDEV = false>
__global__ __launch_bounds__(kBlock, MPC_MIN_WAVES) void k_rollout_argmin(
    Consts Karg, const Consts* __restrict__ Kdev, const double* __restrict__ v,
    const double* __restrict__ b, int64_t n_cand, int n_steps, int64_t n_tiles,
    Rec* __restrict__ part, double* __restrict__ states) {
  const Consts K = KDEV ? *Kdev : Karg;
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

struct EpisodeState;
struct EpisodeHook {           // single-GPU episode: finalize also advances it
  EpisodeState* S;             // nullptr: no hook
  mpc_episode_log_t* log;
  int cap;
};
__device__ void episode_hook(const mpc_episode_config_t& c, const EpisodeHook& h,
                             const mpc_result_t& r);

template <int INTEG, bool KDEV = false>
__global__ __launch_bounds__(kFinBlock) void k_finalize(
    const Rec* __restrict__ part, int n_part, Consts Karg, const Consts* __restrict__ Kdev,
    const double* __restrict__ v, const double* __restrict__ b, int64_t n_cand, int n_steps,
    int64_t index_base, double incumbent_arg, const double* __restrict__ incumbent_dev,
    mpc_result_t* __restrict__ out, mpc_episode_config_t ecfg = {}, EpisodeHook hook = {}) {
  const Consts K = KDEV ? *Kdev : Karg;
  const double incumbent = KDEV ? *incumbent_dev : incumbent_arg;
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
  if (KDEV && hook.S && threadIdx.x == 0) episode_hook(ecfg, hook, *out);
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
// ds_read_b128 instead of a division by |B| and two loads.
__device__ void sample_items(const double2* s_grid, const double* vg, int nb, uint32_t n_grid,
                             int64_t n_cand, int n_steps, uint64_t seed, int64_t base,
                             int cprefix, double* __restrict__ v, double* __restrict__ b,
                             int64_t ld, int pairs) {
  auto lookup = [&](uint32_t k) -> double2 {
    return s_grid ? s_grid[k] : make_double2(vg[k / nb], 0.0);
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

__global__ __launch_bounds__(kBlock) void k_sample_controls(
    const double* __restrict__ vg, int nv, const double* __restrict__ bg, int nb, int64_t n_cand,
    int n_steps, uint64_t seed, int64_t base, int cprefix, double* __restrict__ v,
    double* __restrict__ b, int64_t ld, int pairs) {
  __shared__ double2 s_grid[kSampleLdsEntries];
  const uint32_t n_grid = static_cast<uint32_t>(nv) * static_cast<uint32_t>(nb);
  if (n_grid > kSampleLdsEntries) {
    // large grids: direct lookups (one division per element)
    const int cpt = pairs ? 2 : 1;
    for (int64_t it = blockIdx.x * static_cast<int64_t>(kBlock) + threadIdx.x; it < n_cand / cpt;
         it += static_cast<int64_t>(gridDim.x) * kBlock) {
      const int64_t c = it * cpt;
      for (int st = 0; st < n_steps; ++st)
        for (int j = 0; j < cpt; ++j) {
          const uint32_t k = grid_entry(seed, st, base + c + j, n_grid, cprefix);
          v[st * ld + c + j] = vg[k / nb];
          b[st * ld + c + j] = bg[k % nb];
        }
    }
    return;
  }
  for (uint32_t k = threadIdx.x; k < n_grid; k += kBlock)
    s_grid[k] = make_double2(vg[k / nb], bg[k % nb]);
  __syncthreads();
  sample_items(s_grid, vg, nb, n_grid, n_cand, n_steps, seed, base, cprefix, v, b, ld, pairs);
}

// --------------------------- device-resident episode -----------------------
constexpr int kEpMaxGrid = 64;

struct EpisodeState {
  Consts K;            // this step's problem constants (k_episode_prepare)
  double incumbent;    // optimal_criterion at the start of this step
  double x, y, phi, v, beta;
  double x_t, y_t, x_0, y_0;
  double t;
  uint64_t seed;       // this step's sampler seed
  int64_t step;
  int32_t p, m, steps_for_slowing, episodes;
  int32_t nv, nb;
  double grid_v[kEpMaxGrid];
  double grid_b[kEpMaxGrid];
};

__device__ Consts episode_consts(const EpisodeState& S, double x, double y, double phi, double L,
                                 double t_a, double t_b) {
  mpc_problem_t p;
  p.x = x;
  p.y = y;
  p.phi = phi;
  p.x_t = S.x_t;
  p.y_t = S.y_t;
  p.x_0 = S.x_0;
  p.y_0 = S.y_0;
  p.L = L;
  p.t_a = t_a;
  p.t_b = t_b;
  return consts_from_problem(p);
}

// Episode.reset() / math_mpc's prologue (:521-541): start pose, target, line
// origin at the start, t = 0, p = 1, m = 0, incumbent = control_criterion of
// the origin (the reference's first optimal_criterion, :676).
__device__ void episode_restart(const mpc_episode_config_t& c, EpisodeState& S) {
  S.x = c.start_x;
  S.y = c.start_y;
  S.phi = c.start_phi;
  S.v = c.start_v;
  S.beta = c.start_beta;
  S.x_t = c.target_x;
  S.y_t = c.target_y;
  S.x_0 = c.start_x;
  S.y_0 = c.start_y;
  S.t = 0.0;
  S.p = 1;
  S.m = 0;
  S.steps_for_slowing = 0;
  S.episodes += 1;
  const Consts K0 = episode_consts(S, S.x_0, S.y_0, 0.0, c.L, 0.0, c.delta_t);
  S.incumbent = cost(S.x_0, S.y_0, K0);
}

__global__ void k_episode_reset(mpc_episode_config_t c, EpisodeState* __restrict__ S) {
  if (threadIdx.x != 0) return;
  S->step = 0;
  S->episodes = 0;
  episode_restart(c, *S);
}

// Grids (:239-256) with the reference's expressions and the slow-down
// override (:312-316), computed by one wave: lane i evaluates grid point i,
// a ballot compacts the accepted points in order.  Writes s_v[nv], s_b[nb].
__device__ void episode_grids(const mpc_episode_config_t& c, const EpisodeState& S,
                              double* s_v, double* s_b, int& nv_out, int& nb_out) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int n_v = 1 + 2 * static_cast<int>(c.ratio_v);
  int nv = 0;
  double vmin = __builtin_inf();
  for (int base = 0; base < n_v; base += 64) {
    const int i = base + lane;
    const double cand = S.v + c.delta_v * (static_cast<double>(i) - c.ratio_v);
    const bool ok = i < n_v && !(cand < 0.0) && cand < c.v_max;
    const uint64_t m = __ballot(ok);
    const int pos = nv + __popcll(m & below);
    if (ok && pos < kEpMaxGrid) s_v[pos] = cand;
    double mn = ok ? cand : __builtin_inf();
    for (int off = 32; off > 0; off >>= 1) mn = fmin(mn, __shfl_xor(mn, off, 64));
    vmin = fmin(vmin, mn);
    nv += __popcll(m);
  }
  nv = nv < kEpMaxGrid ? nv : kEpMaxGrid;
  if (S.steps_for_slowing > 0 && nv > 0) {
    const double vel = vmin > c.v_min ? vmin : c.v_min;
    for (int i = lane; i < nv; i += 64) s_v[i] = vel;
  }
  const int n_b = 1 + 2 * static_cast<int>(c.ratio_beta);
  int nb = 0;
  for (int base = 0; base < n_b; base += 64) {
    const int i = base + lane;
    const double cand = S.beta + c.delta_beta * (static_cast<double>(i) - c.ratio_beta);
    const bool ok = i < n_b && fabs(cand) <= c.beta_bound;
    const uint64_t m = __ballot(ok);
    const int pos = nb + __popcll(m & below);
    if (ok && pos < kEpMaxGrid) s_b[pos] = cand;
    nb += __popcll(m);
  }
  nv_out = nv;
  nb_out = nb < kEpMaxGrid ? nb : kEpMaxGrid;
}

__device__ __forceinline__ uint64_t episode_seed(const mpc_episode_config_t& c,
                                                 const EpisodeState& S) {
  return c.seed + 0x9E3779B9ull * static_cast<uint64_t>(S.p + 1000 * S.episodes);
}

// _turn_target (math_model_tree.py:142-215 sectors; sign = +1 left, -1 right).
__device__ void turn_target(double ax, double ay, double aphi, double d, double R, double sign,
                            double& tx, double& ty) {
  const double pi = 3.141592653589793;
  double sn, cs;
  if (pi / 2 <= aphi && aphi <= 3 * pi / 2) {
    if (aphi <= pi) {
      trig::sincos_fast(aphi - pi / 2, &sn, &cs);
      tx = ax - sign * d * cs - R * sn;
      ty = ay - sign * d * sn + R * cs;
    } else {
      trig::sincos_fast(aphi - pi, &sn, &cs);
      tx = ax + sign * d * sn - R * cs;
      ty = ay - sign * d * cs - R * sn;
    }
  } else if (aphi <= 2 * pi) {
    trig::sincos_fast(aphi - 3 * pi / 2, &sn, &cs);
    tx = ax + sign * d * cs + R * sn;
    ty = ay + sign * d * sn - R * cs;
  } else {
    trig::sincos_fast(aphi, &sn, &cs);
    tx = ax - sign * d * sn + R * cs;
    ty = ay + sign * d * cs + R * sn;
  }
}

// Episode._advance: finishing logic (:392-414), events (:564-569), restart.
__device__ void episode_advance(const mpc_episode_config_t& c, EpisodeState* __restrict__ S,
                                const mpc_result_t& r, mpc_episode_log_t* __restrict__ log,
                                int cap) {
  S->steps_for_slowing -= 1;
  S->incumbent = 9223372036854775808.0;  // float(sys.maxsize), :428
  if (log && cap > 0) {
    mpc_episode_log_t& L = log[S->step % cap];
    L.step = S->step;
    L.index = r.found ? r.index : -1;
    L.p = S->p;
    L.episode = S->episodes;
    L.cost = r.cost;
  }
  S->step += 1;
  if (r.found) {
    const int last = r.n_steps - 1;
    const int probe = last < 2 ? last : 2;
    int k = 0;
    if (S->m == 2) {
      k = 2;
    } else if (S->m == 1) {
      k = 1;
      S->m += 1;
    } else {
      const double ex = S->x_t - r.traj[probe][0], ey = S->y_t - r.traj[probe][1];
      if (ex * ex + ey * ey <= c.eps) S->m += 1;
    }
    k = k < last ? k : last;
    S->x = r.traj[k][0];
    S->y = r.traj[k][1];
    S->phi = r.traj[k][2];
    S->v = r.v;
    S->beta = r.beta;
    double tx, ty;
    if (S->p == c.p_turn_right) {
      turn_target(S->x, S->y, S->phi, c.turn_distance, c.radius_u_turn, -1.0, tx, ty);
      S->x_t = tx; S->y_t = ty; S->x_0 = S->x; S->y_0 = S->y;
      S->steps_for_slowing = c.slow_turn;
    }
    if (S->p == c.p_turn_left) {
      turn_target(S->x, S->y, S->phi, c.turn_distance, c.radius_u_turn, +1.0, tx, ty);
      S->x_t = tx; S->y_t = ty; S->x_0 = S->x; S->y_0 = S->y;
      S->steps_for_slowing = c.slow_turn;
    }
    if (S->p == c.p_new_target) {
      S->x_t = c.event_target_x; S->y_t = c.event_target_y; S->x_0 = S->x; S->y_0 = S->y;
      S->steps_for_slowing = c.slow_new_target;
    }
    S->p += 1;
    const double ex = S->x_t - S->x, ey = S->y_t - S->y;
    if (ex * ex + ey * ey <= c.eps || S->p > c.max_steps) episode_restart(c, *S);
  }
  if (log && cap > 0) {
    mpc_episode_log_t& L = log[(S->step - 1) % cap];
    L.x = S->x;
    L.y = S->y;
    L.phi = S->phi;
    L.v = S->v;
    L.beta = S->beta;
  }
}


__device__ void episode_hook(const mpc_episode_config_t& c, const EpisodeHook& h,
                             const mpc_result_t& r) {
  episode_advance(c, h.S, r, h.log, h.cap);
}

// Multi-GPU: lexicographic (cost, global index) selection over the gathered
// per-rank winners (the all-reduce(min+index)), then the episode update.
__global__ void k_episode_advance(mpc_episode_config_t c, EpisodeState* __restrict__ S,
                                  const mpc_result_t* __restrict__ res, int n,
                                  mpc_episode_log_t* __restrict__ log, int cap) {
  if (threadIdx.x != 0) return;
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
  mpc_result_t w = res[best];
  w.found = (bk != ~0ull && w.cost < S->incumbent) ? 1 : 0;
  episode_advance(c, S, w, log, cap);
}

// Device-resident episode, sampler + step prologue in one launch: every block
// derives this step's grid (one wave, ballot compaction) into LDS and samples
// its candidates; block 0 also publishes t += dt, the problem constants and
// the seed for the rollout/finalize launches that follow on the stream.
__global__ __launch_bounds__(kBlock) void k_episode_sample(
    mpc_episode_config_t c, EpisodeState* __restrict__ S, int64_t n_cand, int n_steps,
    int64_t base, double* __restrict__ v, double* __restrict__ b, int pairs) {
  __shared__ double s_v[kEpMaxGrid], s_b[kEpMaxGrid];
  __shared__ double2 s_grid[kSampleLdsEntries];
  __shared__ int s_nv, s_nb;
  if (threadIdx.x < 64) {
    int nv, nb;
    episode_grids(c, *S, s_v, s_b, nv, nb);
    if (threadIdx.x == 0) {
      s_nv = nv;
      s_nb = nb;
    }
  }
  __syncthreads();
  const int nv = s_nv, nb = s_nb;
  const uint64_t seed = episode_seed(c, *S);
  const uint32_t n_grid = static_cast<uint32_t>(nv) * static_cast<uint32_t>(nb);
  const bool in_lds = n_grid <= kSampleLdsEntries;
  if (in_lds)
    for (uint32_t k = threadIdx.x; k < n_grid; k += kBlock)
      s_grid[k] = make_double2(s_v[k / nb], s_b[k % nb]);
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const double t = S->t + c.delta_t;                                      // :302
    S->K = episode_consts(*S, S->x, S->y, S->phi, c.L, t, t + c.delta_t);
    S->t = t;
    S->seed = seed;
    S->nv = nv;
    S->nb = nb;
    for (int i = 0; i < nv; ++i) S->grid_v[i] = s_v[i];
    for (int i = 0; i < nb; ++i) S->grid_b[i] = s_b[i];
  }
  if (n_grid == 0) return;
  sample_items(in_lds ? s_grid : nullptr, s_v, nb, n_grid, n_cand, n_steps, seed, base, 1, v, b,
               n_cand, pairs);
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

template <int NS, int CPL, int INTEG, bool KDEV>
void launch_fixed(dim3 grid, hipStream_t st, const Consts& K, const Consts* Kdev, const double* v,
                  const double* b, int64_t n_cand, int n_steps, int64_t tiles, Rec* part) {
  k_rollout_argmin<NS, CPL, INTEG, false, KDEV>
      <<<grid, kBlock, 0, st>>>(K, Kdev, v, b, n_cand, n_steps, tiles, part, nullptr);
}

template <int CPL, int INTEG, bool KDEV = false>
void launch_by_steps(dim3 grid, hipStream_t st, const Consts& K, const double* v, const double* b,
                     int64_t n_cand, int n_steps, int64_t tiles, Rec* part,
                     const Consts* Kdev = nullptr) {
  switch (n_steps) {
    case 3: launch_fixed<3, CPL, INTEG, KDEV>(grid, st, K, Kdev, v, b, n_cand, n_steps, tiles, part); break;
    case 8: launch_fixed<8, CPL, INTEG, KDEV>(grid, st, K, Kdev, v, b, n_cand, n_steps, tiles, part); break;
    case 10: launch_fixed<10, CPL, INTEG, KDEV>(grid, st, K, Kdev, v, b, n_cand, n_steps, tiles, part); break;
    case 12: launch_fixed<12, CPL, INTEG, KDEV>(grid, st, K, Kdev, v, b, n_cand, n_steps, tiles, part); break;
    default: launch_fixed<0, CPL, INTEG, KDEV>(grid, st, K, Kdev, v, b, n_cand, n_steps, tiles, part); break;
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
          <<<grid, kBlock, 0, st>>>(K, nullptr, v_sc, beta_sc, n_cand, n_steps, tiles, part, states_out);
    else
      k_rollout_argmin<0, 1, MPC_INTEG_QK21, true>
          <<<grid, kBlock, 0, st>>>(K, nullptr, v_sc, beta_sc, n_cand, n_steps, tiles, part, states_out);
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
    k_finalize<MPC_INTEG_RECT><<<1, kFinBlock, 0, st>>>(part, n_part, K, nullptr, v_sc, beta_sc,
                                                        n_cand, n_steps, index_base, incumbent,
                                                        nullptr, out);
  else
    k_finalize<MPC_INTEG_QK21><<<1, kFinBlock, 0, st>>>(part, n_part, K, nullptr, v_sc, beta_sc,
                                                        n_cand, n_steps, index_base, incumbent,
                                                        nullptr, out);
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


size_t mpc_episode_state_bytes(void) { return sizeof(EpisodeState); }

static int check_episode_cfg(const mpc_episode_config_t* c) {
  if (!c) return MPC_ERR_ARG;
  if (!(c->ratio_v >= 0) || !(c->ratio_beta >= 0) || 1 + 2 * static_cast<int>(c->ratio_v) > 4 * kEpMaxGrid ||
      1 + 2 * static_cast<int>(c->ratio_beta) > 4 * kEpMaxGrid || c->max_steps < 1 || !(c->delta_t > 0))
    return MPC_ERR_ARG;
  return MPC_OK;
}

int mpc_episode_reset(const mpc_episode_config_t* cfg, void* state, mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK || !state) return MPC_ERR_ARG;
  k_episode_reset<<<1, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      *cfg, static_cast<EpisodeState*>(state));
  return last_hip_status();
}

static int check_expand_args(const mpc_episode_config_t* cfg, void* state, double* v_sc,
                             double* beta_sc, int64_t n_cand, int32_t n_steps, int64_t index_base,
                             int32_t integrator, void* ws, size_t ws_bytes) {
  if (check_episode_cfg(cfg) != MPC_OK || !state || !v_sc || !beta_sc || n_cand < 1 ||
      n_steps < 1 || n_steps > MPC_MAX_STEPS || index_base < 0)
    return MPC_ERR_ARG;
  if (integrator != MPC_INTEG_QK21 && integrator != MPC_INTEG_RECT) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  return MPC_OK;
}

int mpc_episode_sample(const mpc_episode_config_t* cfg, void* state, double* v_sc,
                       double* beta_sc, int64_t n_cand, int32_t n_steps, int64_t index_base,
                       mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK || !state || !v_sc || !beta_sc || n_cand < 1 ||
      n_steps < 1 || n_steps > MPC_MAX_STEPS || index_base < 0)
    return MPC_ERR_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  EpisodeState* S = static_cast<EpisodeState*>(state);
  const int pairs = (n_cand % 2 == 0) && aligned16(v_sc) && aligned16(beta_sc);
  const int64_t items = pairs ? n_cand / 2 : n_cand;
  k_episode_sample<<<std::min<int64_t>(cdiv(items, kBlock), 4096), kBlock, 0, st>>>(
      *cfg, S, n_cand, n_steps, index_base, v_sc, beta_sc, pairs);
  return last_hip_status();
}

int mpc_episode_partials(void* state, const double* v_sc, const double* beta_sc, int64_t n_cand,
                         int32_t n_steps, int32_t integrator, void* ws, size_t ws_bytes,
                         mpc_stream_t stream) {
  if (!state || !v_sc || !beta_sc || n_cand < 1 || n_steps < 1 || n_steps > MPC_MAX_STEPS)
    return MPC_ERR_ARG;
  if (integrator != MPC_INTEG_QK21 && integrator != MPC_INTEG_RECT) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  EpisodeState* S = static_cast<EpisodeState*>(state);
  Rec* part = static_cast<Rec*>(ws);
  const bool rect = integrator == MPC_INTEG_RECT;
  const bool wide = wide_ok(v_sc, beta_sc, n_cand);
  const int64_t tiles = cdiv(n_cand, kBlock * (wide ? kCplWide : 1));
  const int64_t grid = std::min<int64_t>(tiles, kMaxBlocks);
  const Consts Kdummy{};
  if (wide) {
    if (rect) launch_by_steps<kCplWide, MPC_INTEG_RECT, true>(grid, st, Kdummy, v_sc, beta_sc, n_cand, n_steps, tiles, part, &S->K);
    else launch_by_steps<kCplWide, MPC_INTEG_QK21, true>(grid, st, Kdummy, v_sc, beta_sc, n_cand, n_steps, tiles, part, &S->K);
  } else {
    if (rect) launch_by_steps<1, MPC_INTEG_RECT, true>(grid, st, Kdummy, v_sc, beta_sc, n_cand, n_steps, tiles, part, &S->K);
    else launch_by_steps<1, MPC_INTEG_QK21, true>(grid, st, Kdummy, v_sc, beta_sc, n_cand, n_steps, tiles, part, &S->K);
  }
  return last_hip_status();
}

int mpc_episode_finalize(void* state, const double* v_sc, const double* beta_sc, int64_t n_cand,
                         int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                         size_t ws_bytes, mpc_result_t* out, const mpc_episode_config_t* advance,
                         mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream) {
  if (!state || !v_sc || !beta_sc || !out || n_cand < 1 || n_steps < 1 ||
      n_steps > MPC_MAX_STEPS || index_base < 0)
    return MPC_ERR_ARG;
  if (integrator != MPC_INTEG_QK21 && integrator != MPC_INTEG_RECT) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  EpisodeState* S = static_cast<EpisodeState*>(state);
  const Rec* part = static_cast<const Rec*>(ws);
  const int n_part = static_cast<int>(partial_count(v_sc, beta_sc, n_cand, false));
  const Consts Kdummy{};
  if (advance && (check_episode_cfg(advance) != MPC_OK || log_capacity < 0)) return MPC_ERR_ARG;
  const mpc_episode_config_t ecfg = advance ? *advance : mpc_episode_config_t{};
  const EpisodeHook hook{advance ? S : nullptr, log, log_capacity};
  if (integrator == MPC_INTEG_RECT)
    k_finalize<MPC_INTEG_RECT, true><<<1, kFinBlock, 0, st>>>(
        part, n_part, Kdummy, &S->K, v_sc, beta_sc, n_cand, n_steps, index_base, 0.0,
        &S->incumbent, out, ecfg, hook);
  else
    k_finalize<MPC_INTEG_QK21, true><<<1, kFinBlock, 0, st>>>(
        part, n_part, Kdummy, &S->K, v_sc, beta_sc, n_cand, n_steps, index_base, 0.0,
        &S->incumbent, out, ecfg, hook);
  return last_hip_status();
}

int mpc_episode_expand(const mpc_episode_config_t* cfg, void* state, double* v_sc,
                       double* beta_sc, int64_t n_cand, int32_t n_steps, int64_t index_base,
                       int32_t integrator, void* ws, size_t ws_bytes, mpc_result_t* out,
                       mpc_stream_t stream) {
  int a = check_expand_args(cfg, state, v_sc, beta_sc, n_cand, n_steps, index_base, integrator,
                            ws, ws_bytes);
  if (a != MPC_OK) return a;
  if (!out) return MPC_ERR_ARG;
  if ((a = mpc_episode_sample(cfg, state, v_sc, beta_sc, n_cand, n_steps, index_base, stream)))
    return a;
  if ((a = mpc_episode_partials(state, v_sc, beta_sc, n_cand, n_steps, integrator, ws, ws_bytes,
                                stream)))
    return a;
  return mpc_episode_finalize(state, v_sc, beta_sc, n_cand, n_steps, index_base, integrator, ws,
                              ws_bytes, out, nullptr, nullptr, 0, stream);
}

int mpc_episode_advance(const mpc_episode_config_t* cfg, void* state, const mpc_result_t* results,
                        int32_t n_results, mpc_episode_log_t* log, int32_t log_capacity,
                        mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK || !state || !results || n_results < 1 ||
      log_capacity < 0)
    return MPC_ERR_ARG;
  k_episode_advance<<<1, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      *cfg, static_cast<EpisodeState*>(state), results, n_results, log, log_capacity);
  return last_hip_status();
}

}  // extern "C"
