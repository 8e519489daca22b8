// mpc_episode.h — device-resident MPC episode: the reference's math_mpc loop
// (math_model_tree.py:515-635) with its state in HBM, so that an MPC step is
// enqueued without a host round-trip.
//
//   k_episode_sample   every block derives this step's grids (:239-256,
//                      slow-down :312-316) with one wave and samples its
//                      candidates; block 0 publishes the grids.  (t += dt
//                      (:302), the step's problem constants and seed are
//                      prepared by reset / the previous advance.)
//   k_finalize<..., KDEV> + episode_hook   (one GPU) winner -> episode update
//   k_episode_advance  (multi-GPU) selection over the gathered per-rank
//                      winners, then the episode update
//
// The episode update mirrors diplomjourney_amd/episode.py Episode._advance:
// finishing logic (:392-414), operator events (:564-569), arrival restart.
#pragma once

#include "mpc_kernels.h"

namespace mpc {

constexpr int kEpMaxGrid = 64;

// EpisodeHead (mpc_kernels.h): the scalars; the grids only feed the sampler.
struct EpisodeState {
  EpisodeHead h;
  double grid_v[kEpMaxGrid];
  double grid_b[kEpMaxGrid];
  uint32_t done;       // blocks of the running fused launch that have finished
  uint32_t pad_;
};

__device__ inline Consts episode_consts(const EpisodeHead& S, double x, double y, double phi,
                                        double L, double t_a, double t_b) {
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
// the line origin (the reference's first optimal_criterion, :676).
__device__ inline void episode_restart(const mpc_episode_config_t& c, EpisodeHead& S) {
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

__device__ __forceinline__ uint64_t episode_seed(const mpc_episode_config_t& c,
                                                 const EpisodeHead& S) {
  return c.seed + 0x9E3779B9ull * static_cast<uint64_t>(S.p + 1000 * S.episodes);
}

// Start of an MPC step (math_mpc :302): t += dt, this step's problem
// constants (quad window [t, t+dt]) and sampler seed.  Run by reset and at
// the end of every advance, so a step's rollout needs no preparation launch.
__device__ inline void episode_prepare(const mpc_episode_config_t& c, EpisodeHead& S) {
  const double t = S.t + c.delta_t;
  S.K = episode_consts(S, S.x, S.y, S.phi, c.L, t, t + c.delta_t);
  S.t = t;
  S.seed = episode_seed(c, S);
}

__global__ void k_episode_reset(mpc_episode_config_t c, EpisodeState* __restrict__ S) {
  if (threadIdx.x != 0) return;
  EpisodeHead H = {};
  episode_restart(c, H);
  episode_prepare(c, H);
  S->h = H;
  S->done = 0u;
}

// Grids (:239-256) with the reference's expressions and the slow-down
// override (:312-316), computed by one wave: lane i evaluates grid point i,
// a ballot compacts the accepted points in order.  Writes s_v[nv], s_b[nb].
__device__ inline void episode_grids(const mpc_episode_config_t& c, const EpisodeHead& S,
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

__global__ __launch_bounds__(kBlock) void k_episode_sample(
    mpc_episode_config_t c, EpisodeState* __restrict__ S, int64_t n_cand, int n_steps,
    int64_t base, double* __restrict__ v, double* __restrict__ b, int pairs) {
  __shared__ double s_v[kEpMaxGrid], s_b[kEpMaxGrid];
  __shared__ double2 s_grid[kSampleLdsEntries];
  __shared__ int s_nv, s_nb;
  if (threadIdx.x < 64) {
    int nv, nb;
    episode_grids(c, S->h, s_v, s_b, nv, nb);
    if (threadIdx.x == 0) {
      s_nv = nv;
      s_nb = nb;
    }
  }
  __syncthreads();
  const int nv = s_nv, nb = s_nb;
  const uint64_t seed = S->h.seed;
  const uint32_t n_grid = static_cast<uint32_t>(nv) * static_cast<uint32_t>(nb);
  for (uint32_t k = threadIdx.x; k < n_grid; k += kBlock)  // nv, nb <= 64: fits in LDS
    s_grid[k] = make_double2(s_v[k / nb], s_b[k % nb]);
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S->h.nv = nv;
    S->h.nb = nb;
    for (int i = 0; i < nv; ++i) S->grid_v[i] = s_v[i];
    for (int i = 0; i < nb; ++i) S->grid_b[i] = s_b[i];
  }
  if (n_grid == 0) return;
  sample_items(s_grid, n_grid, n_cand, n_steps, seed, base, 1, v, b, n_cand, pairs);
}

// _turn_target (math_model_tree.py:142-215 sectors; sign = +1 left, -1 right).
__device__ inline void turn_target(double ax, double ay, double aphi, double d, double R,
                                   double sign, double& tx, double& ty) {
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

// r.tr[k][q] for a runtime k in {0, 1, 2} by selects: a dynamically indexed
// local array would live in scratch memory (a ~µs round trip per access).
__device__ __forceinline__ double tr_at(const Winner& r, int k, int q) {
  const double a = r.tr[0][q], b = r.tr[1][q], c = r.tr[2][q];
  return k == 0 ? a : (k == 1 ? b : c);
}

// Episode._advance: finishing logic (:392-414), events (:564-569), restart.
// Operates on a register copy of the episode scalars (the caller loads it
// once and stores it back once).
__device__ inline void episode_advance(const mpc_episode_config_t& c, EpisodeHead& H,
                                       const Winner& r, mpc_episode_log_t* __restrict__ log,
                                       int cap) {
  EpisodeHead* S = &H;
  S->steps_for_slowing -= 1;
  S->incumbent = 9223372036854775808.0;  // float(sys.maxsize), :428
  mpc_episode_log_t* L = (log && cap > 0) ? &log[S->step % cap] : nullptr;
  if (L) {
    L->step = S->step;
    L->index = r.found ? r.index : -1;
    L->p = S->p;
    L->episode = S->episodes;
    L->cost = r.cost;
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
      const double ex = S->x_t - tr_at(r, probe, 0), ey = S->y_t - tr_at(r, probe, 1);
      if (ex * ex + ey * ey <= c.eps) S->m += 1;
    }
    k = k < last ? k : last;
    S->x = tr_at(r, k, 0);
    S->y = tr_at(r, k, 1);
    S->phi = tr_at(r, k, 2);
    S->v = r.v;
    S->beta = r.beta;
    double tx, ty;
    if (S->p == c.p_turn_right) {
      turn_target(S->x, S->y, S->phi, c.turn_distance, c.radius_u_turn, -1.0, tx, ty);
      S->x_t = tx;
      S->y_t = ty;
      S->x_0 = S->x;
      S->y_0 = S->y;
      S->steps_for_slowing = c.slow_turn;
    }
    if (S->p == c.p_turn_left) {
      turn_target(S->x, S->y, S->phi, c.turn_distance, c.radius_u_turn, +1.0, tx, ty);
      S->x_t = tx;
      S->y_t = ty;
      S->x_0 = S->x;
      S->y_0 = S->y;
      S->steps_for_slowing = c.slow_turn;
    }
    if (S->p == c.p_new_target) {
      S->x_t = c.event_target_x;
      S->y_t = c.event_target_y;
      S->x_0 = S->x;
      S->y_0 = S->y;
      S->steps_for_slowing = c.slow_new_target;
    }
    S->p += 1;
    const double ex = S->x_t - S->x, ey = S->y_t - S->y;
    if (ex * ex + ey * ey <= c.eps || S->p > c.max_steps) episode_restart(c, *S);
  }
  episode_prepare(c, *S);
  if (L) {
    L->x = S->x;
    L->y = S->y;
    L->phi = S->phi;
    L->v = S->v;
    L->beta = S->beta;
  }
}

__device__ void episode_hook(const mpc_episode_config_t& c, const EpisodeHook& h,
                             const Winner& r, EpisodeHead& H) {
  episode_advance(c, H, r, h.log, h.cap);
}

// Multi-GPU: lexicographic (cost, global index) selection over the gathered
// per-rank winners (the all-reduce(min+index)), then the episode update.
__global__ void k_episode_advance(mpc_episode_config_t c, EpisodeState* __restrict__ S,
                                  const mpc_result_t* __restrict__ res, int n,
                                  mpc_episode_log_t* __restrict__ log, int cap) {
  if (threadIdx.x != 0) return;
  EpisodeHead H = S->h;
  uint64_t bk;
  const int best = select_index(res, n, bk);
  const mpc_result_t& r = res[best];
  Winner w;
  w.cost = r.cost;
  w.index = r.index;
  w.found = (bk != ~0ull && r.cost < H.incumbent) ? 1 : 0;
  w.n_steps = r.n_steps;
  w.v = r.v;
  w.beta = r.beta;
  for (int k = 0; k < 3; ++k)
    for (int q = 0; q < 3; ++q) w.tr[k][q] = r.traj[k < r.n_steps ? k : 0][q];
  episode_advance(c, H, w, log, cap);
  S->h = H;
}

}  // namespace mpc
