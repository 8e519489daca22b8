// mpc_ftepisodes.h — run_math_model.py's episode loop (:231-280) over its own
// FULL-TREE MPC step (:133-228), R episodes device-resident.
//
// Two forms.  The default (mpc_fulltree_episodes_run) is the load-balanced
// lockstep form at the end of this file: per call, the leaves of every robot
// still running spread over the whole GPU.  k_ft_episodes_run (build with
// -DMPC_FT_LOCKSTEP=0) is the round-5 form, kept as its A/B reference:
// one block per robot runs its episode's MPC steps back to back in ONE launch
// (the structure of mpc_episodes.h, with the full tree as the step):
//
//   per MPC step of robot r (block r):
//     stop rules    on target (:261) / the caller's call limit, checked before
//                   the step as the script's `while` and run_batched do
//     window        t += delta_t (:156); the step's constants from the pose,
//                   the episode's target and line origin (consts_from_problem)
//     controls      the S1 = |V|*|B| per-control factors (FtCtl: v*h, dphi of
//                   the quad window, rotation factors) into LDS, one thread per
//                   control; a step with some |dphi| > kRotMax runs the direct
//                   sin/cos form (as k_ft_controls' launch-wide flag)
//     leaves        the S1^3 leaves (:158-197) as k_ft_leaves scores them
//                   (ft_leaves_body: lane = (k0, k1) pair, k2 wave-uniform),
//                   spread over the block's 4 waves; lexicographic (cost, j)
//                   block minimum; found = cost < the robot's never-reset
//                   optimal_criterion (:193-196)
//     update        a winner's first layer (re-derived with ft_apply) + its
//                   control becomes optimal_trajectory[0][0]; without a winner
//                   the stale one is returned again (the script re-reads it);
//                   the two-non-move stop (:266-272); one log record
//
// The state: FtEpisode[R] (the robots' episode globals, copied from the
// host-built mpc_fulltree_episode_config_t by mpc_fulltree_episodes_reset).
#pragma once

#include "mpc_episodes.h"
#include "mpc_fulltree.h"

namespace mpc {

// One robot's run_math_model.py episode (the script's module globals).
struct FtEpisode {
  double x, y, phi, v, beta;       // the pose and control the next call starts from
  double x_0, y_0, x_t, y_t;       // start (line origin) and target (:235-239)
  double atan_t;                   // numpy arctan(x_t / y_t) (:83), from the host
  double crit;                     // optimal_criterion, never reset in an episode
  double t;                        // t after the last call (:156)
  double stale[5];                 // optimal_trajectory[0][0]: x, y, phi, v, beta
  double prev_x, prev_y;           // x_previous / y_previous (:266-272)
  int32_t has_stale, k, calls, stop, max_calls, pad_;
  int64_t leaves;                  // leaves scored so far
};

// Largest S1 whose control table (48 B per control) fits the LDS: 24 KiB per
// block, so the LDS never limits the 4 blocks per CU below.
constexpr int kFtEpMaxS1 = 512;
// 4 waves per SIMD: 4 robots per CU at a time (1024 resident blocks), <= 128
// VGPRs for the leaf loop (both heading forms instantiated).
constexpr int kFtEpWaves = 4;

__global__ void k_ft_episodes_reset(const mpc_fulltree_episode_config_t* __restrict__ cfgs,
                                    int n, FtEpisode* __restrict__ eps) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const mpc_fulltree_episode_config_t c = cfgs[r];
  FtEpisode E = {};
  E.x = c.x_0;                      // :243-246: the episode starts at its start,
  E.y = c.y_0;                      // v = 0 (:233), t = 0 (:234)
  E.phi = c.phi_0;
  E.x_0 = c.x_0;
  E.y_0 = c.y_0;
  E.x_t = c.x_t;
  E.y_t = c.y_t;
  E.atan_t = c.atan_target;
  E.crit = c.incumbent0;            // control_criterion([x_0, y_0, phi_0]) (:252)
  E.prev_x = c.x_0;
  E.prev_y = c.y_0;
  E.max_calls = c.max_calls;
  eps[r] = E;
}

// Block r = robot r: up to max_calls MPC steps of its episode (fewer if it
// stops).  log: [n][cap] ring per robot; progress: {calls, stop, leaves}.
template <int INTEG, bool ROT>
__global__ __launch_bounds__(kBlock, kFtEpWaves) void k_ft_episodes_run(
    FtEpisode* __restrict__ eps, const double* __restrict__ V, int nv,
    const double* __restrict__ B, int nb, double L, double delta_t, double eps_target,
    int max_calls, mpc_episode_log_t* __restrict__ log, int cap,
    mpc_episodes_progress_t* __restrict__ progress) {
  const int r = blockIdx.x;
  __shared__ __attribute__((aligned(16))) FtCtl s_ctl[kFtEpMaxS1];
  __shared__ FtEpisode s_e;
  __shared__ mpc_episode_log_t s_log;
  __shared__ int s_run;
  if (threadIdx.x == 0) s_e = eps[r];
  const int64_t s1 = static_cast<int64_t>(nv) * nb;
  const int64_t n_items = ft_units(s1);
  const int64_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int call = 0; call < max_calls; ++call) {
    if (threadIdx.x == 0) {   // the loop's head (:261) and the caller's limit
      if (s_e.stop == 0) {
        const double ex = s_e.x_t - s_e.x, ey = s_e.y_t - s_e.y;
        if (ex * ex + ey * ey <= eps_target)
          s_e.stop = MPC_EP_ARRIVED;
        else if (s_e.max_calls > 0 && s_e.calls >= s_e.max_calls)
          s_e.stop = MPC_EP_LIMIT;
      }
      s_run = s_e.stop == 0;
    }
    __syncthreads();
    if (!s_run) break;   // uniform
    const double t_a = s_e.t + delta_t;                        // t += delta_t (:156)
    mpc_problem_t q;
    q.x = s_e.x;
    q.y = s_e.y;
    q.phi = s_e.phi;
    q.x_t = s_e.x_t;
    q.y_t = s_e.y_t;
    q.x_0 = s_e.x_0;
    q.y_0 = s_e.y_0;
    q.L = L;
    q.t_a = t_a;
    q.t_b = t_a + delta_t;
    const Consts K = uniform_consts(consts_from_problem(q));
    const double atan_t = s_e.atan_t;
    // the step's control table (k_ft_controls' arithmetic), in LDS
    bool wide = false;
    for (int64_t k = threadIdx.x; k < s1; k += kBlock) {
      FtCtl u;
      u.v = V[k / nb];
      u.beta = B[k % nb];
      u.vh = u.v * K.h;
      const double w = K.L_pow2 ? u.v * K.inv_L : u.v / K.L;
      u.dphi = heading_incr<INTEG>(w, trig::tan_fast(u.beta), K);
      if (fabs(u.dphi) <= trig::kRotMax) {
        trig::rotation_sc(u.dphi, u.sd, u.cd);
      } else {
        u.sd = u.cd = 0.0;
        wide = true;
      }
      s_ctl[k] = u;
    }
    // (the barrier that publishes the table: evaluated in every instantiation,
    // not short-circuited away by a false ROT)
    const bool any_wide = __syncthreads_or(wide);
    const bool rot = ROT && !any_wide;
    uint64_t best_k = ~0ull;
    int64_t best_i = INT64_MAX;
    const FtCrit F = ft_crit(K, atan_t);
    if (rot)
      ft_leaves_body<INTEG, true>(K, F, s_ctl, s1, 0, n_items, best_k, best_i, wave, kWaves);
    else
      ft_leaves_body<INTEG, false>(K, F, s_ctl, s1, 0, n_items, best_k, best_i, wave, kWaves);
    block_argmin(best_k, best_i);
    if (threadIdx.x == 0) {   // the update of run_batched (run_math_model.py)
      FtEpisode& E = s_e;
      mpc_episode_log_t& Lg = s_log;
      const double c = key_cost(best_k);
      const bool found = best_k != ~0ull && c < E.crit;
      int32_t status = 0;
      E.t = t_a;
      if (found) {
        E.crit = c;
        const int64_t k0 = best_i / (s1 * s1);
        const FtCtl u = s_ctl[k0];
        const FtState s0{K.x, K.y, K.phi, K.s0, K.c0};
        const FtState l0 = rot ? ft_apply<INTEG, true>(s0, u, K) : ft_apply<INTEG, false>(s0, u, K);
        E.stale[0] = l0.x;
        E.stale[1] = l0.y;
        E.stale[2] = l0.ph;
        E.stale[3] = u.v;
        E.stale[4] = u.beta;
        E.has_stale = 1;
      } else {
        status |= MPC_EP_STALE;
      }
      if (!E.has_stale) {
        // optimal_trajectory is still the script's [0]: its first call raises
        // TypeError ('int' object is not subscriptable) — the episode stops
        status |= MPC_EP_NO_TRAJ;
        E.stop = status;
      } else {
        E.x = E.stale[0];
        E.y = E.stale[1];
        E.phi = E.stale[2];
        E.v = E.stale[3];
        E.beta = E.stale[4];
        if (E.x == E.prev_x && E.y == E.prev_y) {   // :266-270
          E.k += 1;
          status |= MPC_EP_STUCK;
        }
        if (E.k == 2) {
          status |= MPC_EP_BREAK;
          E.stop = status;
        }
        E.prev_x = E.x;
        E.prev_y = E.y;
      }
      Lg.step = E.calls;
      Lg.index = found ? best_i : -1;
      Lg.p = E.calls + 1;
      Lg.episode = 1;
      Lg.found = found ? 1 : 0;
      Lg.status = status;
      Lg.cost = E.crit;
      Lg.x = E.x;
      Lg.y = E.y;
      Lg.phi = E.phi;
      Lg.v = E.v;
      Lg.beta = E.beta;
      E.calls += 1;
      E.leaves += s1 * s1 * s1;
    }
    __syncthreads();
    if (log && cap > 0 && threadIdx.x < kLogWords)
      reinterpret_cast<uint64_t*>(&log[static_cast<int64_t>(r) * cap + s_log.step % cap])
          [threadIdx.x] = reinterpret_cast<const uint64_t*>(&s_log)[threadIdx.x];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    eps[r] = s_e;
    if (progress) {
      progress[r].calls = s_e.calls;
      progress[r].stop = s_e.stop;
      progress[r].candidates = s_e.leaves;
    }
  }
}

// ---------------------------------------------------------------------------
// Load-balanced lockstep form of the same episodes (the default of
// mpc_fulltree_episodes_run).  One block per robot leaves a robot's CU idle
// once its episode has stopped: at workload G (1000 episodes, 50 calls) 40 %
// of the lockstep slots were idle (30,257 robot-calls of 50,000), and the
// last calls ran a few long episodes on a few CUs.  Here every call is three
// launches over the robots still running:
//   k_ftl_prepare  one block: the stop rules of every robot (the loop head,
//                  :261, and the call limit), the live robots compacted in
//                  ascending order, their step constants (FtRobot), and the
//                  call's control table — ONE table for all of them: every
//                  live robot has run the same number of calls, so its window
//                  [t, t + dt] is the same sum of the same dt's
//   k_ftl_leaves   a fixed grid spread over the live robots: bpr = grid /
//                  n_live blocks per robot (its S1^3 leaves in bpr x 4
//                  equal contiguous wave shares, ft_leaves_body, the control
//                  table read as wave-uniform scalar loads as in k_ft_leaves)
//   k_ftl_update   one block per live robot: its bpr records -> the first
//                  strict minimum, then exactly k_ft_episodes_run's update.
// The leaves' costs are the per-robot kernel's (same table, same constants,
// same ft_leaf); the lexicographic (cost, leaf) minimum does not depend on
// how the leaves were split, so the two forms log the same bits.
struct FtLockstep {
  int32_t n_live, bpr, no_rot, pad_;
};

// Scratch of the lockstep form, after FtEpisode[R] in the episodes' state.
__host__ __device__ inline size_t ftl_align(size_t n) { return (n + 255) & ~size_t{255}; }
__host__ __device__ inline size_t ftl_ls_offset(int n) {
  return ftl_align(static_cast<size_t>(n) * sizeof(FtEpisode));
}
__host__ __device__ inline size_t ftl_ctl_offset(int n) {
  return ftl_ls_offset(n) + ftl_align(sizeof(FtLockstep));
}
__host__ __device__ inline size_t ftl_live_offset(int n) {
  return ftl_ctl_offset(n) + ftl_align(kFtEpMaxS1 * sizeof(FtCtl));
}
__host__ __device__ inline size_t ftl_robots_offset(int n) {
  return ftl_live_offset(n) + ftl_align(static_cast<size_t>(n) * sizeof(int32_t));
}
__host__ __device__ inline size_t ftl_part_offset(int n) {
  return ftl_robots_offset(n) + ftl_align(static_cast<size_t>(n) * sizeof(FtRobot));
}
constexpr int kFtlMaxGrid = 2048;
__host__ __device__ inline size_t ftl_bytes(int n) {
  return ftl_part_offset(n) + ftl_align(kFtlMaxGrid * sizeof(Rec));
}

constexpr int kFtlPrepBlock = 1024;
template <int INTEG>
__global__ __launch_bounds__(kFtlPrepBlock) void k_ftl_prepare(
    FtEpisode* __restrict__ eps, int n, const double* __restrict__ V, int nv,
    const double* __restrict__ B, int nb, double L, double delta_t, double eps_target, int grid,
    FtLockstep* __restrict__ ls, FtCtl* __restrict__ ctl, int32_t* __restrict__ live,
    FtRobot* __restrict__ robots) {
  __shared__ int s_wave[kFtlPrepBlock / 64];
  __shared__ int s_total;
  __shared__ double s_ta;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_ta = __builtin_nan("");
  int base_out = 0;
  for (int base = 0; base < n; base += kFtlPrepBlock) {
    const int r = base + threadIdx.x;
    bool run = false;
    if (r < n) {
      FtEpisode& E = eps[r];
      if (E.stop == 0) {   // the loop's head (:261) and the caller's limit
        const double ex = E.x_t - E.x, ey = E.y_t - E.y;
        if (ex * ex + ey * ey <= eps_target)
          E.stop = MPC_EP_ARRIVED;
        else if (E.max_calls > 0 && E.calls >= E.max_calls)
          E.stop = MPC_EP_LIMIT;
      }
      run = E.stop == 0;
    }
    const uint64_t m = __ballot(run);
    if (lane == 0) s_wave[wave] = __popcll(m);
    __syncthreads();
    int before = 0, total = 0;
    for (int w = 0; w < kFtlPrepBlock / 64; ++w) {
      before += w < wave ? s_wave[w] : 0;
      total += s_wave[w];
    }
    if (run) {
      const int j = base_out + before + __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
      live[j] = r;
      const FtEpisode& E = eps[r];
      const double t_a = E.t + delta_t;                        // t += delta_t (:156)
      mpc_problem_t q;
      q.x = E.x;
      q.y = E.y;
      q.phi = E.phi;
      q.x_t = E.x_t;
      q.y_t = E.y_t;
      q.x_0 = E.x_0;
      q.y_0 = E.y_0;
      q.L = L;
      q.t_a = t_a;
      q.t_b = t_a + delta_t;
      robots[r].K = consts_from_problem(q);
      robots[r].atan_t = E.atan_t;
      if (j == 0) s_ta = t_a;   // every live robot's window (lockstep)
    }
    base_out += total;
    __syncthreads();   // (s_wave reuse)
  }
  if (threadIdx.x == 0) {
    s_total = base_out;
    ls->n_live = base_out;
    ls->bpr = base_out > 0 ? (grid / base_out > 1 ? grid / base_out : 1) : 0;
  }
  __syncthreads();
  if (s_total == 0) return;
  // the call's control table (k_ft_controls' arithmetic, with the constants
  // of the shared window)
  mpc_problem_t q = {};
  q.x_t = 1.0;   // (the table reads only L, h, hlgth, inv_L, L_pow2)
  q.L = L;
  q.t_a = s_ta;
  q.t_b = s_ta + delta_t;
  const Consts K = consts_from_problem(q);
  const int64_t s1 = static_cast<int64_t>(nv) * nb;
  bool wide = false;
  for (int64_t k = threadIdx.x; k < s1; k += kFtlPrepBlock) {
    FtCtl u;
    u.v = V[k / nb];
    u.beta = B[k % nb];
    u.vh = u.v * K.h;
    const double w = K.L_pow2 ? u.v * K.inv_L : u.v / K.L;
    u.dphi = heading_incr<INTEG>(w, trig::tan_fast(u.beta), K);
    if (fabs(u.dphi) <= trig::kRotMax) {
      trig::rotation_sc(u.dphi, u.sd, u.cd);
    } else {
      u.sd = u.cd = 0.0;
      wide = true;
    }
    ctl[k] = u;
  }
  const bool any_wide = __syncthreads_or(wide);
  if (threadIdx.x == 0) ls->no_rot = any_wide ? 1 : 0;
}

template <int INTEG, bool ROT>
__global__ __launch_bounds__(kBlock, kFtWaves) void k_ftl_leaves(
    const FtLockstep* __restrict__ ls, const FtCtl* __restrict__ ctl,
    const int32_t* __restrict__ live, const FtRobot* __restrict__ robots, int64_t s1,
    Rec* __restrict__ part) {
  const int n_live = ls->n_live, bpr = ls->bpr;
  const int j = static_cast<int>(blockIdx.x) / (bpr > 0 ? bpr : 1);
  if (n_live == 0 || j >= n_live) return;   // (uniform)
  const int share = static_cast<int>(blockIdx.x) - j * bpr;
  const int r = live[j];
  const Consts K = uniform_consts(robots[r].K);
  const FtCrit F = ft_crit(K, robots[r].atan_t);
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  const int64_t wave = static_cast<int64_t>(share) * kWaves +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n_waves = static_cast<int64_t>(bpr) * kWaves;
  if (ROT && ls->no_rot == 0)
    ft_leaves_body<INTEG, true>(K, F, ctl, s1, 0, ft_units(s1), best_k, best_i, wave, n_waves);
  else
    ft_leaves_body<INTEG, false>(K, F, ctl, s1, 0, ft_units(s1), best_k, best_i, wave, n_waves);
  block_argmin(best_k, best_i);
  if (threadIdx.x == 0) part[blockIdx.x] = Rec{best_k, best_i};
}

template <int INTEG, bool ROT>
__global__ __launch_bounds__(kBlock) void k_ftl_update(
    FtEpisode* __restrict__ eps, const FtLockstep* __restrict__ ls,
    const FtCtl* __restrict__ ctl, const int32_t* __restrict__ live,
    const FtRobot* __restrict__ robots, const Rec* __restrict__ part, int64_t s1,
    double delta_t, mpc_episode_log_t* __restrict__ log, int cap) {
  __shared__ mpc_episode_log_t s_log;
  const int n_live = ls->n_live, bpr = ls->bpr;
  const int j = blockIdx.x;
  if (j >= n_live) return;   // (uniform)
  const int r = live[j];
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  for (int p = threadIdx.x; p < bpr; p += kBlock) {
    const Rec rec = part[static_cast<int64_t>(j) * bpr + p];
    if (rec_less(rec.key, rec.idx, best_k, best_i)) {
      best_k = rec.key;
      best_i = rec.idx;
    }
  }
  block_argmin(best_k, best_i);
  if (threadIdx.x == 0) {   // k_ft_episodes_run's update (run_batched, run_math_model.py)
    FtEpisode E = eps[r];
    const Consts& K = robots[r].K;
    const bool rot = ROT && ls->no_rot == 0;
    mpc_episode_log_t& Lg = s_log;
    const double c = key_cost(best_k);
    const bool found = best_k != ~0ull && c < E.crit;
    int32_t status = 0;
    E.t = E.t + delta_t;
    if (found) {
      E.crit = c;
      const int64_t k0 = best_i / (s1 * s1);
      const FtCtl u = ctl[k0];
      const FtState s0{K.x, K.y, K.phi, K.s0, K.c0};
      const FtState l0 = rot ? ft_apply<INTEG, true>(s0, u, K) : ft_apply<INTEG, false>(s0, u, K);
      E.stale[0] = l0.x;
      E.stale[1] = l0.y;
      E.stale[2] = l0.ph;
      E.stale[3] = u.v;
      E.stale[4] = u.beta;
      E.has_stale = 1;
    } else {
      status |= MPC_EP_STALE;
    }
    if (!E.has_stale) {
      status |= MPC_EP_NO_TRAJ;
      E.stop = status;
    } else {
      E.x = E.stale[0];
      E.y = E.stale[1];
      E.phi = E.stale[2];
      E.v = E.stale[3];
      E.beta = E.stale[4];
      if (E.x == E.prev_x && E.y == E.prev_y) {   // :266-270
        E.k += 1;
        status |= MPC_EP_STUCK;
      }
      if (E.k == 2) {
        status |= MPC_EP_BREAK;
        E.stop = status;
      }
      E.prev_x = E.x;
      E.prev_y = E.y;
    }
    Lg.step = E.calls;
    Lg.index = found ? best_i : -1;
    Lg.p = E.calls + 1;
    Lg.episode = 1;
    Lg.found = found ? 1 : 0;
    Lg.status = status;
    Lg.cost = E.crit;
    Lg.x = E.x;
    Lg.y = E.y;
    Lg.phi = E.phi;
    Lg.v = E.v;
    Lg.beta = E.beta;
    E.calls += 1;
    E.leaves += s1 * s1 * s1;
    eps[r] = E;
  }
  __syncthreads();
  if (log && cap > 0 && threadIdx.x < kLogWords)
    reinterpret_cast<uint64_t*>(&log[static_cast<int64_t>(r) * cap + s_log.step % cap])
        [threadIdx.x] = reinterpret_cast<const uint64_t*>(&s_log)[threadIdx.x];
}

__global__ void k_ftl_progress(const FtEpisode* __restrict__ eps, int n,
                               mpc_episodes_progress_t* __restrict__ progress) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  progress[r].calls = eps[r].calls;
  progress[r].stop = eps[r].stop;
  progress[r].candidates = eps[r].leaves;
}

}  // namespace mpc
