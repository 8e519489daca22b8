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

#include <stddef.h>

#include "mpc_kernels.h"

namespace mpc {

constexpr int kEpMaxGrid = 64;

// Bounded device waits, measured on the GPU's constant-rate wall clock
// (wall_clock64: s_memrealtime, 100 MHz on gfx950) rather than in poll passes,
// so that waits of different loops compare: a wait that runs out sets
// chain_error instead of hanging the GPU.
//   kChainWaitTicks   one GPU: a chained launch's tiles wait for block 0,
//                     which waits for nothing outside the launch
//   kPeerWaitTicks    block 0 waits for other ranks (P2P mailbox, error 5) or
//                     for a collective beside the launch (error 4); ranks are
//                     not barrier-aligned between steps, so a peer may start
//                     the same step a host hiccup later
//   kXchgWaitTicks    an exchange launch's tiles wait for THAT block 0: longer
//                     than its peer wait, so a late peer surfaces as block 0's
//                     error (or not at all), never as tiles scoring the step on
//                     speculated constants (error 1)
constexpr uint64_t kWallHz = 100000000ull;
constexpr uint64_t kChainWaitTicks = kWallHz / 5;        // 0.2 s
constexpr uint64_t kPeerWaitTicks = 2 * kWallHz;         // 2 s
constexpr uint64_t kXchgWaitTicks = 3 * kWallHz;         // 3 s
static_assert(kXchgWaitTicks > kPeerWaitTicks, "tiles outwait their block 0");

// 32-bit deadlines (one register; the low word wraps after 42 s, far beyond
// any budget here, and the comparison is wrap-safe)
__device__ __forceinline__ uint32_t wall_deadline(uint64_t ticks) {
  return static_cast<uint32_t>(wall_clock64()) + static_cast<uint32_t>(ticks);
}
__device__ __forceinline__ bool wall_passed(uint32_t deadline) {
  return static_cast<int32_t>(static_cast<uint32_t>(wall_clock64()) - deadline) > 0;
}
// Block-wide (all threads, same pass): has the deadline passed?  Thread 0's
// clock decides, so every wave leaves a __syncthreads_* poll on the same pass.
__device__ __forceinline__ bool block_wall_passed(uint32_t deadline) {
  // (readfirstlane: the compiler sees a uniform value, so a loop that leaves
  // on it stays uniform and its loop-invariant pointers stay in SGPRs)
  return __builtin_amdgcn_readfirstlane(
             __syncthreads_or(threadIdx.x == 0 && wall_passed(deadline))) != 0;
}
constexpr int kConstsWords = static_cast<int>(sizeof(Consts) / 4);
constexpr int kPubWords = kConstsWords + 2;   // Consts, then t
static_assert(sizeof(Consts) % 4 == 0 && kPubWords <= 64, "published words: one wave");

// EpisodeHead (mpc_kernels.h): the scalars; the grids only feed the sampler.
// The stale trajectory follows the head (staged and stored with it as one
// run of kStoredWords words), then the early-publication inputs (staged with
// both by a chained step's block 0: kStagedWords).
struct EpisodeState {
  EpisodeHead h;
  StaleTraj st;        // right after the head: staged and stored with it
  EarlyPub early;      // right after the stale trajectory: staged with both
  double grid_v[kEpMaxGrid];
  double grid_b[kEpMaxGrid];
  uint32_t done;       // blocks of the running fused launch that have finished
  uint32_t chain_error;   // a chained step's wait timed out (k_episode_chain)
  // P2P exchange: completions so far; completion c uses mailbox slot c & 1.
  // Counted on the device (every rank completes the same steps), not taken
  // from the launch's epoch: a replayed HIP graph repeats its epochs, and a
  // captured sequence of odd length would start its next replay in the slot
  // its flush was still reading on a slower rank.
  uint32_t p2p_seq;
  // Constants published by a chained launch's block 0 (k_episode_chain): the
  // dwords of the step's Consts and of t, each in a 64-bit word tagged with
  // the launch's epoch ((dword << 32) | epoch), so one coherent load per word
  // says whether its value is this step's.  Tag 0: none.
  alignas(128) uint64_t chain_pub[kPubWords];
  // Overlapped exchange (mpc_episode_exchange_step2 with wait_tag): the epoch
  // of the step whose candidates the last all_gather delivered, stored by
  // k_exchange_mark on the collective's stream after the collective; block 0
  // of the next launch polls it instead of the launch waiting on a stream edge.
  alignas(128) uint64_t gathered_tag;
};
static_assert(offsetof(EpisodeState, st) == sizeof(EpisodeHead), "stale trajectory follows the head");
static_assert(offsetof(EpisodeState, early) == kStoredWords * 8, "EarlyPub follows the stale trajectory");

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
// origin at the start, t = 0, p = 1, m = 0 (the script resets m between its
// two runs, :737), recursive = False;
// incumbent = cfg.incumbent0, or control_criterion of the line origin with
// the episode's target (the reference's first optimal_criterion is that of
// config.py's target, :676).  optimal_trajectory / result_v / result_beta
// are module globals the reference never resets: they carry over.
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
  S.recursive = 0;
  if (c.incumbent0 != 0.0) {
    S.incumbent = c.incumbent0;
  } else {
    const Consts K0 = episode_consts(S, S.x_0, S.y_0, 0.0, c.L, 0.0, c.delta_t);
    S.incumbent = cost(S.x_0, S.y_0, K0);
  }
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

// The head's early_* fields (EpisodeHead): the next step's early-publication
// inputs that do not depend on its winner — episode_advance's decisions
// (:559-569, :542 and the step limit) as far as the head alone fixes them,
// with st the stale trajectory the step will return without a winner.
__device__ inline void episode_early_prepare(const mpc_episode_config_t& c, const EpisodeHead& S,
                                             const StaleTraj& st, EarlyPub& E) {
  E.step = S.step;
  E.t = S.t + c.delta_t;
  E.h = (E.t + c.delta_t) - E.t;             // consts_from_problem
  E.hl = 0.5 * ((E.t + c.delta_t) - E.t);
  const bool common = !(c.stop_rule == 0 && S.recursive) && S.p != c.p_turn_right &&
                      S.p != c.p_turn_left && S.p != c.p_new_target &&
                      !(c.max_steps > 0 && S.p + 1 > c.max_steps);
  const int k = S.m == 2 ? 2 : (S.m == 1 ? 1 : 0);
  E.k = common ? k : -1;
  E.x = S.has_traj ? st.ot[k][0] : S.x;
  E.y = S.has_traj ? st.ot[k][1] : S.y;
  E.ph = S.has_traj ? st.ot[k][2] : S.phi;
  E.alt = early_pose_ok(c, S, E.x, E.y) ? 1 : 0;
}

__global__ void k_episode_reset(mpc_episode_config_t c, EpisodeState* __restrict__ S) {
  if (threadIdx.x != 0) return;
  EpisodeHead H = {};
  episode_restart(c, H);
  episode_prepare(c, H);
  EarlyPub E;
  episode_early_prepare(c, H, S->st, E);
  S->early = E;
  S->h = H;
  S->done = 0u;
  S->chain_error = 0u;
  S->p2p_seq = 0u;
  for (int q = 0; q < kPubWords; ++q) S->chain_pub[q] = 0ull;
  S->gathered_tag = 0ull;
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
    if (S.steps_for_slowing > 0) {   // (uniform) min(V) only for the slow-down
      double mn = ok ? cand : __builtin_inf();
      for (int off = 32; off > 0; off >>= 1) mn = fmin(mn, __shfl_xor(mn, off, 64));
      vmin = fmin(vmin, mn);
    }
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
  if (n_grid == 0 && !c.enumerate) return;
  sample_items(s_grid, n_grid, n_cand, n_steps, seed, base, c.enumerate ? 2 : 1, v, b, n_cand,
               pairs);
}

// ---------------------------------------------------------------------------
// Generated controls (inputs "generated", mpc_episode_generate_step): the
// sampler of k_episode_sample and the rollout of k_rollout_argmin_stream in
// ONE kernel — every block builds the step's grid (episode_grids) in LDS and
// each lane draws its candidates' (v, beta) per step from it with the same
// splitmix64 -> multiply-shift map (grid_entry, constant prefix included),
// so the controls never touch HBM.  Per lane two candidates, the same
// operations in the same order as the streaming kernel's lane
// (rollout_lane_glds_k), so results equal the sampled path's bit for bit.
// Each block also writes its best candidate's controls to part_v / part_b
// [block][MPC_MAX_STEPS] for the selection's winner re-roll (k_finalize_gen).
template <int INTEG, int ROT, bool PL2>
__device__ __forceinline__ void generated_lane(const Consts& K, const double2* s_grid,
                                               uint32_t n_grid, uint64_t seed, uint64_t g0,
                                               int n_steps, double (&cst)[2]) {
  double x[2], y[2], ph[2], sn[2], cs[2];
  bool bad[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    step_start<ROT>(K, x[j], y[j], ph[j], sn[j], cs[j]);
    bad[j] = false;
  }
  trig::Leads lead = trig::const_leads();
#pragma unroll 1
  for (int st = 0; st < n_steps; ++st) {
    const double2 e0 = s_grid[grid_entry(seed, st, g0, n_grid, 1)];
    const double2 e1 = s_grid[grid_entry(seed, st, g0 + 1, n_grid, 1)];
    double ph0 = ROT ? 0.0 : ph[0], ph1 = ROT ? 0.0 : ph[1];
    step_core<INTEG, ROT, PL2>(x[0], y[0], ph0, sn[0], cs[0], e0.x, e0.y, K, bad[0], &lead);
    step_core<INTEG, ROT, PL2>(x[1], y[1], ph1, sn[1], cs[1], e1.x, e1.y, K, bad[1], &lead);
    if (!ROT) {
      ph[0] = ph0;
      ph[1] = ph1;
    }
  }
  if constexpr (ROT == kRotCum) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (!bad[j]) cum_pose<PL2>(K, x[j], y[j], x[j], y[j]);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (bad[j]) {
      x[j] = K.x;
      y[j] = K.y;
      ph[j] = K.phi;
      for (int sr = 0; sr < n_steps; ++sr) {
        const double2 e = s_grid[grid_entry(seed, sr, g0 + j, n_grid, 1)];
        step_safe<INTEG>(x[j], y[j], ph[j], e.x, e.y, K);
      }
    }
    cst[j] = cost(x[j], y[j], K);
  }
}

constexpr int kGenWaves = 4;   // launch bound of the generated-controls rollout (5 spills)
// PL2 (wheelbase a power of two) is a template parameter picked by the host
// from cfg, as in the chained step (one rollout variant per kernel).
template <int INTEG, int ROT, bool PL2>
__global__ __launch_bounds__(kBlock, kGenWaves) void k_rollout_generated(
    mpc_episode_config_t c, EpisodeState* __restrict__ S, int64_t n_cand, int n_steps,
    int64_t base, Rec* __restrict__ part, double* __restrict__ part_v,
    double* __restrict__ part_b) {
  extern __shared__ double2 s_gen_grid[];   // the expanded grid (dynamic: nv x nb entries)
  __shared__ double s_v[kEpMaxGrid], s_b[kEpMaxGrid];
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
  const uint32_t n_grid = static_cast<uint32_t>(nv) * static_cast<uint32_t>(nb);
  for (uint32_t k = threadIdx.x; k < n_grid; k += kBlock)
    s_gen_grid[k] = make_double2(s_v[k / nb], s_b[k % nb]);
  if (blockIdx.x == 0 && threadIdx.x == 0) {   // as k_episode_sample: the step's grid
    // a state reset with another wheelbase form than cfg's: flag it (chain error 2)
    if ((S->h.K.L_pow2 != 0) != PL2) S->chain_error = 2u;
    S->h.nv = nv;
    S->h.nb = nb;
    for (int i = 0; i < nv; ++i) S->grid_v[i] = s_v[i];
    for (int i = 0; i < nb; ++i) S->grid_b[i] = s_b[i];
  }
  __syncthreads();
  const uint64_t seed = S->h.seed;
  const Consts K = S->h.K;
  const int64_t n_tiles = (n_cand + kBlock * 2 - 1) / (kBlock * 2);
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  if (n_grid > 0) {
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
      const int64_t c0 = tile * (kBlock * 2) + threadIdx.x * 2;
      if (c0 < n_cand) {   // n_cand even (host check): the pair is valid
        double cst[2];
        const uint64_t g0 = static_cast<uint64_t>(base + c0);
        generated_lane<INTEG, ROT, PL2>(K, s_gen_grid, n_grid, seed, g0, n_steps, cst);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const uint64_t kk = cost_key_nonneg(cst[j]);
          if (kk < best_k) {   // ascending index per lane: strict < keeps the first
            best_k = kk;
            best_i = c0 + j;
          }
        }
      }
    }
  }
  block_argmin(best_k, best_i);
  if (threadIdx.x == 0) part[blockIdx.x] = Rec{best_k, best_i};
  // the block's best candidate's controls, one step per lane
  __shared__ int64_t s_best;
  if (threadIdx.x == 0) s_best = best_k == ~0ull ? -1 : best_i;
  __syncthreads();
  const int64_t bi = s_best;
  if (bi >= 0 && threadIdx.x < n_steps) {
    const double2 e =
        s_gen_grid[grid_entry(seed, threadIdx.x, static_cast<uint64_t>(base + bi), n_grid, 1)];
    part_v[blockIdx.x * MPC_MAX_STEPS + threadIdx.x] = e.x;
    part_b[blockIdx.x * MPC_MAX_STEPS + threadIdx.x] = e.y;
  }
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


// Episode._advance = the rest of math_mpc's loop body after predictive_control
// (:542-574 with :351-429): the returned pose is the winner's layer state
// picked by the finishing logic (:392-414) — or, when no candidate beat the
// incumbent, the STALE optimal_trajectory / result_v / result_beta of the
// last improving step (the globals :351-359 did not touch), with the same
// finishing logic; then the stuck detector (:559-563: a pose equal to the
// previous one sets `recursive`, the next step with it set ends the episode
// before the events), the operator events (:564-569), p += 1, and the loop
// condition (:542: on target ends the episode).  An ended episode restarts
// (the bench's episode stream; the reference's loop returns).
// Operates on a register copy of the episode scalars (the caller loads it
// once and stores it back once).  The step's log record is filled in `L`
// (LDS); the caller stores it (log_slot) together with the head.
// RESTART = false (the batched robots of mpc_episodes.h): an ended episode
// stays ended (the caller stops the robot) instead of restarting.
// c.stop_rule 1: run_math_model.py's stuck detector instead of math_mpc's —
// `recursive` counts the episode's non-moving steps and the second one ends
// it at once (:266-272, before the on-target test of the loop head).
// early (a chained step's block 0 that published early, finalize_block):
// the next step's Consts and t as published (8-B aligned LDS words) — the
// step cannot end then, and the update takes t from them and leaves H.K to
// the caller (it stores the published words as the head's constants); a
// step that ends anyway sets *early_bad (chain error 6) and is prepared in
// full.
template <bool RESTART = true>
__device__ inline void episode_advance(const mpc_episode_config_t& c, EpisodeHead& H,
                                       StaleTraj& st, const Winner& r, mpc_episode_log_t& L,
                                       const uint32_t* early = nullptr,
                                       bool* early_bad = nullptr) {
  EpisodeHead* S = &H;
  S->steps_for_slowing -= 1;
  S->incumbent = 9223372036854775808.0;  // float(sys.maxsize), :428
  L.step = S->step;
  L.index = r.found ? r.index : -1;
  L.p = S->p;
  L.episode = S->episodes;
  L.found = r.found;
  L.cost = r.cost;
  int32_t status = 0;
  S->step += 1;
  if (r.found) {   // :352-359: the globals take the winner
    const int last = r.n_steps - 1;
    for (int k = 0; k < 3; ++k)
      for (int q = 0; q < 3; ++q) st.ot[k][q] = tr_at(r, k < last ? k : last, q);
    st.v = r.v;
    st.beta = r.beta;
    S->has_traj = 1;
  } else {
    status |= MPC_EP_STALE;
    if (!S->has_traj) {
      // the reference's initial optimal_trajectory [[[0]]] has no layer
      // states (it would raise IndexError): stay at the pose
      for (int k = 0; k < 3; ++k) {
        st.ot[k][0] = S->x;
        st.ot[k][1] = S->y;
        st.ot[k][2] = S->phi;
      }
      st.v = S->v;
      st.beta = S->beta;
    }
  }
  // finishing logic on optimal_trajectory[0] (:388-414): probe layer 2 (the
  // last layer for horizons < 3), return layer k
  int k = 0;
  if (S->m == 2) {
    k = 2;
  } else if (S->m == 1) {
    k = 1;
    S->m += 1;
  } else {
    const double ex = S->x_t - st.ot[2][0], ey = S->y_t - st.ot[2][1];
    if (ex * ex + ey * ey <= c.eps) S->m += 1;
  }
  const double x_prev = S->x, y_prev = S->y;   // x_previous / y_previous (:570-571)
  S->x = st.ot[k][0];   // (st lives in LDS: a dynamic index is an LDS address)
  S->y = st.ot[k][1];
  S->phi = st.ot[k][2];
  S->v = st.v;
  S->beta = st.beta;
  bool ended = false;
  if (c.stop_rule == 0 && S->recursive) {   // :559-561 "Recursive error." -> break
    status |= MPC_EP_BREAK;
    ended = true;
  } else if (S->x == x_prev && S->y == y_prev && c.stop_rule == 1 && S->recursive >= 1) {
    S->recursive += 1;                      // run_math_model.py:266-272: k == 2
    status |= MPC_EP_STUCK | MPC_EP_BREAK;
    ended = true;
  } else {
    if (S->x == x_prev && S->y == y_prev) {   // :562-563 (stop_rule 1: k += 1)
      S->recursive += 1;
      status |= MPC_EP_STUCK;
    }
    double tx, ty;
    if (S->p == c.p_turn_right) {
      turn_target(S->x, S->y, S->phi, c.turn_distance, c.radius_u_turn, -1.0, tx, ty);
      S->x_t = tx;
      S->y_t = ty;
      S->x_0 = S->x;
      S->y_0 = S->y;
      S->steps_for_slowing = c.slow_turn;
      status |= MPC_EP_EVENT;
    }
    if (S->p == c.p_turn_left) {
      turn_target(S->x, S->y, S->phi, c.turn_distance, c.radius_u_turn, +1.0, tx, ty);
      S->x_t = tx;
      S->y_t = ty;
      S->x_0 = S->x;
      S->y_0 = S->y;
      S->steps_for_slowing = c.slow_turn;
      status |= MPC_EP_EVENT;
    }
    if (S->p == c.p_new_target) {
      S->x_t = c.event_target_x;
      S->y_t = c.event_target_y;
      S->x_0 = S->x;
      S->y_0 = S->y;
      S->steps_for_slowing = c.slow_new_target;
      status |= MPC_EP_EVENT;
    }
    S->p += 1;
    const double ex = S->x_t - S->x, ey = S->y_t - S->y;
    if (ex * ex + ey * ey <= c.eps) {                   // :542
      status |= MPC_EP_ARRIVED;
      ended = true;
    } else if (c.max_steps > 0 && S->p > c.max_steps) {
      status |= MPC_EP_LIMIT;
      ended = true;
    }
  }
  L.x = S->x;
  L.y = S->y;
  L.phi = S->phi;
  L.v = S->v;
  L.beta = S->beta;
  L.status = status;
  if (ended) {
    if constexpr (!RESTART) return;
    episode_restart(c, *S);
  }
  if (early && (ended || reinterpret_cast<const Consts*>(early)->x != S->x ||
                reinterpret_cast<const Consts*>(early)->y != S->y ||
                reinterpret_cast<const Consts*>(early)->phi != S->phi))
    *early_bad = true;   // (never expected: the early decisions are this update's)
  if (early && !ended) {
    // K: the published words (= episode_prepare's; the caller stores them)
    S->t = *reinterpret_cast<const double*>(early + sizeof(Consts) / 4);
    S->seed = episode_seed(c, *S);
  } else {
    episode_prepare(c, *S);
  }
}

__device__ void episode_hook(const mpc_episode_config_t& c, const EpisodeHook& h,
                             const Winner& r, EpisodeHead& H, StaleTraj& st,
                             mpc_episode_log_t& L, mpc_episode_log_t*& slot,
                             const uint32_t* early, bool* early_bad) {
  slot = log_slot(h.log, h.cap, H.step);
  episode_advance(c, H, st, r, L, early, early_bad);
}

// Multi-GPU: lexicographic (cost, global index) selection over the gathered
// per-rank winners (the all-reduce(min+index)), then the episode update.
// Called by every thread of a block (>= 64 threads): thread 0 updates a
// register copy of the head, which goes back to HBM through LDS one word per
// lane (a single lane's stores serialise); end_chain clears the chain tags.
__device__ inline void advance_from_results(const mpc_episode_config_t& c, EpisodeState* S,
                                            const mpc_result_t* __restrict__ res, int n,
                                            mpc_episode_log_t* __restrict__ log, int cap,
                                            bool end_chain = true) {
  __shared__ uint64_t s_head[kStoredWords];
  __shared__ mpc_episode_log_t s_log;
  __shared__ mpc_episode_log_t* s_slot;
  if (threadIdx.x < kStaleWords)   // the stale trajectory, staged beside the head
    s_head[kHeadWords + threadIdx.x] = reinterpret_cast<const uint64_t*>(&S->st)[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
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
    s_slot = log_slot(log, cap, H.step);
    episode_advance(c, H, *reinterpret_cast<StaleTraj*>(&s_head[kHeadWords]), w, s_log);
    __builtin_memcpy(s_head, &H, sizeof(EpisodeHead));
  }
  __syncthreads();
  store_update(&S->h, s_head, s_slot, reinterpret_cast<const uint64_t*>(&s_log),
               end_chain ? S->chain_pub : nullptr, kPubWords);
}

// Multi-GPU chained exchange: the global winner of a step among the gathered
// per-rank candidates (lexicographic (cost, global index)), re-rolled from its
// gathered controls with the step's constants (emit_winner: the same
// operations as the rollout that scored it) into `out`, then the episode
// update.  Every thread of a block of kFinBlock threads.
template <int INTEG, int ROT>
__device__ void advance_from_candidates(const mpc_episode_config_t& c, EpisodeState* S,
                                        const mpc_candidate_t* __restrict__ g, int n,
                                        mpc_result_t* __restrict__ out,
                                        mpc_episode_log_t* __restrict__ log, int cap,
                                        uint32_t publish_epoch, EmitLds* lds) {
  __shared__ uint64_t s_head[kStoredWords];
  __shared__ mpc_episode_log_t s_log;
  __shared__ mpc_episode_log_t* s_slot;
  __shared__ int s_best;
  __shared__ uint64_t s_bk;
  if (threadIdx.x < kStoredWords)
    s_head[threadIdx.x] = reinterpret_cast<const uint64_t*>(&S->h)[threadIdx.x];
  if (threadIdx.x == 0) {
    int best = 0;
    uint64_t bk = ~0ull;
    int64_t bi = INT64_MAX;
    for (int r = 0; r < n; ++r) {
      const uint64_t k = g[r].index < 0 ? ~0ull : cost_key(g[r].cost);
      const int64_t i = g[r].index < 0 ? INT64_MAX : g[r].index;
      if (r == 0 || rec_less(k, i, bk, bi)) {
        best = r;
        bk = k;
        bi = i;
      }
    }
    s_best = best;
    s_bk = bk;
  }
  __syncthreads();
  const mpc_candidate_t* w = &g[s_best];
  const EpisodeHead* Hs = reinterpret_cast<const EpisodeHead*>(s_head);
  const Consts K = Hs->K;                // the step's constants (before the update)
  Winner win;
  emit_winner<INTEG, ROT>(K, nullptr, nullptr, 0, w->n_steps, s_bk, 0, w->index, Hs->incumbent,
                          out, lds, &win, w->v, w->beta, true);
  if (threadIdx.x == 0) {   // emit_winner ended with a barrier; lane 0 holds `win`
    EpisodeHead H;
    __builtin_memcpy(&H, s_head, sizeof(EpisodeHead));
    s_slot = log_slot(log, cap, H.step);
    episode_advance(c, H, *reinterpret_cast<StaleTraj*>(&s_head[kHeadWords]), win, s_log);
    __builtin_memcpy(s_head, &H, sizeof(EpisodeHead));
  }
  __syncthreads();
  // publish_epoch 0: the update ends the chain (tags cleared); else it
  // publishes the next step's constants (a chained exchange step's block 0)
  store_update(&S->h, s_head, s_slot, reinterpret_cast<const uint64_t*>(&s_log), S->chain_pub,
               kPubWords, publish_epoch);
  emit_winner_tail<INTEG, ROT>(K, w->n_steps, lds, out);   // the rest of the record
}

template <int INTEG, int ROT>
__global__ __launch_bounds__(kFinBlock) void k_episode_advance_cand(
    mpc_episode_config_t c, EpisodeState* __restrict__ S, const mpc_candidate_t* __restrict__ g,
    int n, mpc_result_t* __restrict__ out, mpc_episode_log_t* __restrict__ log, int cap) {
  __shared__ EmitLds lds;
  advance_from_candidates<INTEG, ROT>(c, S, g, n, out, log, cap, 0u, &lds);
}

// A tile block's record in an exchange step: ONE 16-B `sc1` store that block
// 0 of the same launch polls for (no counter, no wait in the tile block).
// Freshness must not rest on the 16-B store and load being single-copy
// atomic (the memory model promises that only up to 8 B), so EACH 8-B half
// carries the launch's 16-bit tag in its low bits and block 0 accepts the
// record only when both halves show it:
//   word 0 = key[63:16] << 16 | tag
//   word 1 = key[15:0] << 48 | index[31:0] << 16 | tag
// (the 64-bit cost key and a 32-bit local index; no candidate: index
// 0xffffffff).  A half torn from an older record carries another tag (or the
// 0 of a consumed record) and is polled again.
__device__ __forceinline__ uint32_t rec_tag(uint32_t epoch) {
  return epoch % 0xffffu + 1u;   // in [1, 0xffff]; consecutive epochs differ, 0 = untagged
}

__device__ __forceinline__ void store_tagged_rec(Rec* dst, uint64_t key, int64_t idx,
                                                 uint32_t epoch) {
  const uint64_t ix = idx == INT64_MAX ? 0xffffffffull
                                       : static_cast<uint64_t>(static_cast<uint32_t>(idx));
  const uint64_t tag = rec_tag(epoch);
  const uint64_t w0 = (key & ~0xffffull) | tag;
  const uint64_t w1 = (key << 48) | (ix << 16) | tag;
  // (s_nop 1: the store must read its data registers before the compiler's
  // next instruction may overwrite them)
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1"
               :
               : "v"(dst), "v"(u64x2{w0, w1})
               : "memory");
}

__device__ __forceinline__ bool tagged_rec_fresh(const u64x2& r, uint32_t tag) {
  return static_cast<uint32_t>(r.x & 0xffffu) == tag && static_cast<uint32_t>(r.y & 0xffffu) == tag;
}

__device__ __forceinline__ uint64_t tagged_rec_key(const u64x2& r) {
  return (r.x & ~0xffffull) | (r.y >> 48);
}

__device__ __forceinline__ uint32_t tagged_rec_index(const u64x2& r) {
  return static_cast<uint32_t>(r.y >> 16);
}

// Block 0 of an exchange step, after publishing: wait until every tile
// block's record of THIS launch has landed (tags == epoch; `sc1` loads, a
// bounded poll), reduce them and write this rank's best candidate — its
// (cost, global index) and its controls, one step per lane — to `out`.
__device__ void collect_local_candidate(const Rec* __restrict__ part, int n_part, uint32_t epoch,
                                        const double* __restrict__ v,
                                        const double* __restrict__ b, int64_t n_cand,
                                        int n_steps, int64_t index_base,
                                        mpc_candidate_t* __restrict__ out, uint32_t* err) {
  static_assert(kMaxBlocks <= 8 * kBlock, "eight records per thread");
  uint32_t off[8];   // byte offsets from the (uniform) record base
  u64x2 r[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int p = threadIdx.x + q * kBlock;
    off[q] = static_cast<uint32_t>(p < n_part ? p : n_part - 1) * sizeof(Rec);
  }
  bool timed_out = false;
  const uint32_t tag = rec_tag(epoch);
  // Bounded in passes (~1-2 us each: 2^20 passes, >= 1 s; the tiles may share
  // the GPU with other processes' launches).  A clock check here (a second
  // block-wide barrier per check) kept 52 B of VGPR spills in this form.
  for (uint32_t it = 0;; ++it) {
    load8_rec_sc1_sbase(part, off, r);
    bool ok = true;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (threadIdx.x + q * kBlock < n_part) ok = ok && tagged_rec_fresh(r[q], tag);
    if (__syncthreads_and(ok)) break;
    if (it >= (1u << 20)) {   // uniform: every thread counts the same passes
      timed_out = true;
      break;
    }
    __builtin_amdgcn_s_sleep(16);
  }
  uint64_t k = ~0ull;
  int64_t i = INT64_MAX;
  if (!timed_out) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint32_t lo = tagged_rec_index(r[q]);
      const int64_t idx = lo == 0xffffffffu ? INT64_MAX : static_cast<int64_t>(lo);
      const uint64_t key = tagged_rec_key(r[q]);
      if (threadIdx.x + q * kBlock < n_part) {
        if (rec_less(key, idx, k, i)) {
          k = key;
          i = idx;
        }
        // consumed: untag both halves.  A replayed HIP graph repeats its
        // launches' epochs, so a record left tagged would pass for the
        // replay's own before that launch's tile block stores it.  Coherent
        // (`sc1`) stores: a plain store could stay dirty in this XCD's L2 and
        // be written back over a later record stored there by a block on
        // another XCD with no kernel boundary in between (measured: a
        // persistent multi-step variant of this collection timed out so).
        uint64_t* h = reinterpret_cast<uint64_t*>(
            const_cast<char*>(reinterpret_cast<const char*>(part)) + off[q]);
        __hip_atomic_store(h, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(h + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else if (threadIdx.x == 0) {
    *err = 3u;
  }
  block_argmin(k, i);
  __shared__ uint64_t s_k;
  __shared__ int64_t s_i;
  if (threadIdx.x == 0) {
    s_k = k;
    s_i = i;
  }
  __syncthreads();
  k = s_k;
  i = s_i;
  const bool valid = k != ~0ull;
  const int q = threadIdx.x;
  if (q < MPC_MAX_STEPS) {   // one value per lane
    out->v[q] = (valid && q < n_steps) ? v[q * n_cand + i] : 0.0;
    out->beta[q] = (valid && q < n_steps) ? b[q * n_cand + i] : 0.0;
  }
  if (q == 0) {
    out->cost = valid ? key_cost(k) : __builtin_inf();
    out->index = valid ? index_base + i : -1;
    out->n_steps = n_steps;
    out->reserved_ = 0;
  }
}

// The overlapped exchange's hand-off: after the all_gather of step `tag`'s
// candidates (same stream, so the collective's stores are complete), publish
// the tag.  One coherent 8-B store (relaxed, agent scope: `sc1`).
__global__ void k_exchange_mark(EpisodeState* __restrict__ S, uint32_t tag) {
  if (threadIdx.x == 0) __hip_atomic_store(&S->gathered_tag, static_cast<uint64_t>(tag),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kXchgLdsRanks = 32;   // gathered candidates staged in the ring's LDS
static_assert(kXchgLdsRanks * sizeof(mpc_candidate_t) + sizeof(EmitLds) <= sizeof(g_ring),
              "staged candidates + the re-roll's LDS fit in the control ring");

// Block 0 of an overlapped exchange step, all threads: wait (bounded) until
// the all_gather of step `tag` has been marked, then copy the n gathered
// candidates into LDS with coherent 8-B loads (the collective wrote them
// while this launch was already running: no stream edge orders them for
// it).  Returns the LDS copy, or nullptr if the wait timed out (error 4).
__device__ const mpc_candidate_t* wait_gathered(EpisodeState* S, uint32_t tag,
                                                const mpc_candidate_t* __restrict__ g, int n) {
  __shared__ int s_ok;
  if (threadIdx.x < 64) {   // one wave: its clock reads are uniform
    bool ok = false;
    const uint32_t deadline = wall_deadline(kPeerWaitTicks);
    for (;;) {
      const uint64_t w = __hip_atomic_load(&S->gathered_tag, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      if (static_cast<uint32_t>(w) == tag) {
        ok = true;
        break;
      }
      if (wall_passed(deadline)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (threadIdx.x == 0) {
      s_ok = ok;
      if (!ok) S->chain_error = 4u;
    }
  }
  __syncthreads();
  if (!s_ok) return nullptr;
  mpc_candidate_t* dst = reinterpret_cast<mpc_candidate_t*>(
      reinterpret_cast<char*>(ring_lds()) + ((sizeof(EmitLds) + 15) & ~size_t{15}));
  const int words = n * static_cast<int>(sizeof(mpc_candidate_t) / 8);
  for (int q = threadIdx.x; q < words; q += blockDim.x)
    reinterpret_cast<uint64_t*>(dst)[q] =
        __hip_atomic_load(reinterpret_cast<const uint64_t*>(g) + q, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return dst;
}

__global__ __launch_bounds__(64) void k_episode_advance(mpc_episode_config_t c,
                                                        EpisodeState* __restrict__ S,
                                                        const mpc_result_t* __restrict__ res,
                                                        int n, mpc_episode_log_t* __restrict__ log,
                                                        int cap) {
  advance_from_results(c, S, res, n, log, cap);
}

// ---------------------------------------------------------------------------
// Chained episode step (heading mode kRotCum): ONE launch = this step's
// streaming rollout + the completion of the PREVIOUS step.  Block 0 completes
// step k-1 — kChainFin (one GPU): k_finalize's record reduction, winner
// re-roll and episode update; kChainXchg (multi-GPU): the selection over the
// gathered per-rank candidates, the winner's re-roll and the update — and
// publishes step k's constants as epoch-tagged words (EpisodeState::chain_pub);
// kChainXchg's block 0 then collects this launch's tagged block records into
// the rank's candidate (collect_local_candidate), which the caller gathers.
// The other blocks do not wait for it: in kRotCum mode a candidate's rollout
// needs no start pose, only the step size h (and the constant wheelbase
// terms).  A block reads the published words once, right after its first
// control loads are in flight: if all carry this launch's epoch (block 0 is
// done: every block after the first round) the constants are final; else it
// speculates h as the next step of the same episode (from the previous
// step's published t, + dt, as episode_prepare forms it) and reads the words
// again after its loop, for the final pose transform and the criterion.  If h
// turns out different (the previous step restarted the episode and reset t)
// the lane recomputes with the published constants (rollout_lane_glds).
// Records of tile-block b go to part[b - 1].  Consecutive chained launches
// carry different epochs and the update that ends a chain (k_finalize's hook,
// k_episode_advance) clears the tags.  The wait is bounded: if the words
// never came, chain_error is set instead of hanging the GPU.
// kChainP2P (multi-GPU, no collective): kChainFin's structure (records to
// part, the next launch's block 0 reduces them) with the per-rank candidates
// exchanged through the mailboxes by block 0 (p2p_complete).
constexpr int kChainFin = 1, kChainXchg = 3, kChainP2P = 4;

// LDS dwords (Consts layout) -> wave-uniform Consts, field by field (no
// memory view of the struct: it stays in SGPRs).
__device__ __forceinline__ Consts consts_from_words(const uint32_t* w) {
  auto d = [&](size_t off) {
    const int q = static_cast<int>(off / 4);
    // (readfirstlane returns int: through uint32_t, not sign-extended)
    const uint64_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(w[q]));
    const uint64_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(w[q + 1]));
    return __longlong_as_double(static_cast<long long>((hi << 32) | lo));
  };
  auto i32 = [&](size_t off) {
    return static_cast<int32_t>(__builtin_amdgcn_readfirstlane(w[off / 4]));
  };
  Consts K;
  K.x = d(offsetof(Consts, x));
  K.y = d(offsetof(Consts, y));
  K.phi = d(offsetof(Consts, phi));
  K.x_t = d(offsetof(Consts, x_t));
  K.y_t = d(offsetof(Consts, y_t));
  K.x_0 = d(offsetof(Consts, x_0));
  K.y_0 = d(offsetof(Consts, y_0));
  K.A = d(offsetof(Consts, A));
  K.B = d(offsetof(Consts, B));
  K.C1 = d(offsetof(Consts, C1));
  K.C2 = d(offsetof(Consts, C2));
  K.inv_den = d(offsetof(Consts, inv_den));
  K.L = d(offsetof(Consts, L));
  K.inv_L = d(offsetof(Consts, inv_L));
  K.h = d(offsetof(Consts, h));
  K.hlgth = d(offsetof(Consts, hlgth));
  K.s0 = d(offsetof(Consts, s0));
  K.c0 = d(offsetof(Consts, c0));
  K.L_pow2 = i32(offsetof(Consts, L_pow2));
  K.pad_ = 0;
  return K;
}

// Block 0, all threads, after the episode head is stored: publish its Consts
// and t as tagged words (relaxed agent-scope atomic stores: coherent, and each
// word validates itself).
__device__ __forceinline__ void chain_publish(EpisodeState* S, uint32_t epoch) {
  __syncthreads();   // the head (stored by thread 0) is visible to the block
  const int q = threadIdx.x;
  if (q < kPubWords) {
    const uint32_t d = q < kConstsWords
                           ? reinterpret_cast<const uint32_t*>(&S->h.K)[q]
                           : reinterpret_cast<const uint32_t*>(&S->h.t)[q - kConstsWords];
    __hip_atomic_store(&S->chain_pub[q], (static_cast<uint64_t>(d) << 32) | epoch,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Wave 0 of a tile block: one coherent load of every published word into
// s_w / s_tag; returns (wave-uniform) whether all carry `epoch`.
__device__ __forceinline__ bool chain_read(const EpisodeState* S, uint32_t epoch,
                                           uint32_t* s_w, uint32_t* s_tag) {
  const int q = threadIdx.x;
  bool ok = true;
  if (q < kPubWords) {
    const uint64_t w = __hip_atomic_load(const_cast<uint64_t*>(&S->chain_pub[q]),
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_w[q] = static_cast<uint32_t>(w >> 32);
    s_tag[q] = static_cast<uint32_t>(w);
    ok = static_cast<uint32_t>(w) == epoch;
  }
  return __ballot(!ok) == 0;
}

// ---------------------------------------------------------------------------
// Peer-to-peer exchange (mpc_episode_p2p_step): no collective launch.  Every
// rank owns a MAILBOX in its HBM (uncached device memory, mpc_mailbox_alloc:
// each access goes to HBM, so stores a peer GPU makes over xGMI are what this
// GPU's loads see).  Block 0 of rank q's launch with epoch e+1 — the launch
// that completes step e — reduces step e's block records (the previous
// launch's, stream-ordered: plain loads) into q's candidate and stores it into
// slot c&1 (c = the episode's P2P completions so far, EpisodeState::p2p_seq),
// row q, of EVERY rank's mailbox (its own included); it then waits
// until the world's candidates of step e are complete in its own mailbox,
// stages them in LDS, clears them, selects the global winner and updates the
// episode.  The tile blocks meanwhile stream step e+1 (its constants are
// speculated until block 0 publishes them, as in the one-GPU chain): the
// exchange runs beside the rollout, not between launches.
// Self-validating granules: each 8-B word of a candidate travels as one 16-B
// granule whose two 8-B halves both carry the step's 16-bit tag (word[63:16]
// | tag, word[15:0] << 48 | tag — the tagged block records' encoding), so a
// reader accepts a word only when both halves are this step's, never relying
// on store ordering, on a fence or on 16-B single-copy atomicity: the writer
// issues its stores and goes on (no completion wait, no flag store), the
// reader polls the granules themselves.  Only the words a step needs move:
// cost, index, (n_steps, reserved), v[0..n_steps), beta[0..n_steps).
// A consumed granule is zeroed by its reader.  Two slots suffice: rank q
// writes slot c&1 again only for completion c+2, after it has read every
// rank's completion-(c+1) candidate — each posted in a launch that began after
// the launch whose zeroing stores had completed (a kernel boundary).  This
// holds across graph replays whatever the captured length (the count lives on
// the device; the epochs only tag the granules).
//   layout: MailHdr (the peers' mailbox pointers as mapped in this process,
//           this rank, the world size, ping words), then granule
//           [2][world][kCandWords] of 16 B
constexpr int kMailMaxRanks = kXchgLdsRanks;
struct MailHdr {
  uint64_t peers[kMailMaxRanks];
  int32_t rank, world;
  uint64_t ping[kMailMaxRanks];   // mpc_mailbox_ping: rank r's ping word
};
constexpr size_t kMailHdrBytes = (sizeof(MailHdr) + 255) & ~size_t{255};
constexpr int kCandWords = static_cast<int>(sizeof(mpc_candidate_t) / 8);
constexpr size_t kMailRecBytes = kCandWords * sizeof(u64x2);
static_assert(sizeof(mpc_candidate_t) % 8 == 0, "candidates move as 8-B words");
static_assert(offsetof(mpc_candidate_t, v) == 24 && offsetof(mpc_candidate_t, beta) ==
                  24 + 8 * MPC_MAX_STEPS, "candidate word map (cand_word)");
// Peers' launches are not stream-ordered with this one: a rank may start its
// step a host-side hiccup later.  kPeerWaitTicks (2 s) before chain error 5.

__host__ __device__ inline size_t mailbox_bytes(int world) {
  return kMailHdrBytes + 2 * static_cast<size_t>(world) * kMailRecBytes;
}

__device__ __forceinline__ u64x2* mail_rec(void* mb, uint32_t slot, int rank, int world) {
  return reinterpret_cast<u64x2*>(static_cast<char*>(mb) + kMailHdrBytes +
                                  (static_cast<size_t>(slot) * world + rank) * kMailRecBytes);
}

// The j-th posted word of a candidate of n_steps steps: its word index in
// mpc_candidate_t (3 header words, then v[0..n), then beta[0..n)).
__device__ __forceinline__ int cand_word(int j, int n_steps) {
  return j < 3 + n_steps ? j : j + (MPC_MAX_STEPS - n_steps);
}

// Where block 0 stages candidates: the control ring's LDS after the re-roll's
// EmitLds (the ring is idle in block 0).
__device__ __forceinline__ mpc_candidate_t* cand_lds() {
  return reinterpret_cast<mpc_candidate_t*>(reinterpret_cast<char*>(ring_lds()) +
                                            ((sizeof(EmitLds) + 15) & ~size_t{15}));
}

// Block 0, all threads: this rank's best candidate of the previous launch —
// the lexicographic (cost, local index) minimum of its n_part block records
// (plain 16-B records of a stream-ordered earlier launch), its global index
// and its controls — into `out` (LDS).  Each wave loads its own best's
// controls while the waves' minima are combined (finalize_block's prefetch:
// no dependent load after the block's winner is known).
template <bool TILED = false>
__device__ void records_candidate(const Rec* __restrict__ part, int n_part,
                                  const double* __restrict__ v, const double* __restrict__ b,
                                  int64_t n_cand, int n_steps, int64_t index_base,
                                  mpc_candidate_t* out) {
  constexpr int kPer = static_cast<int>((kMaxBlocks + kBlock - 1) / kBlock);
  Rec r[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {   // every load issued before any compare
    const int p = threadIdx.x + q * kBlock;
    r[q] = p < n_part ? part[p] : Rec{~0ull, INT64_MAX};
  }
  uint64_t k = ~0ull;
  int64_t i = INT64_MAX;
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if (rec_less(r[q].key, r[q].idx, k, i)) {
      k = r[q].key;
      i = r[q].idx;
    }
  wave_argmin(k, i);   // every lane: its wave's best
  const int ln = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double pv = 0.0, pb = 0.0;
  if (k != ~0ull && ln < n_steps) {
    const int64_t o = ctl_off<TILED>(ln, i, TILED ? n_steps : n_cand);
    pv = v[o];
    pb = b[o];
  }
  __shared__ uint64_t s_k[kWaves];
  __shared__ int64_t s_i[kWaves];
  if (ln == 0) {
    s_k[wave] = k;
    s_i[wave] = i;
  }
  __syncthreads();
  int wbest = 0;
  k = s_k[0];
  i = s_i[0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w)
    if (rec_less(s_k[w], s_i[w], k, i)) {
      k = s_k[w];
      i = s_i[w];
      wbest = w;
    }
  const bool valid = k != ~0ull;
  if (wave == wbest && ln < MPC_MAX_STEPS) {   // one value per lane
    out->v[ln] = (valid && ln < n_steps) ? pv : 0.0;
    out->beta[ln] = (valid && ln < n_steps) ? pb : 0.0;
  }
  if (threadIdx.x == 0) {
    out->cost = valid ? key_cost(k) : __builtin_inf();
    out->index = valid ? index_base + i : -1;
    out->n_steps = n_steps;
    out->reserved_ = 0;
  }
}

// Block 0, all threads: post this rank's candidate (in LDS) of step `epoch`
// to every rank's mailbox as tagged granules (16-B `sc0 sc1` stores; nothing
// waits for them).
__device__ void post_candidate(const uint64_t* s_peers, int rank, int world, uint32_t epoch,
                               uint32_t slot, int n_steps, const mpc_candidate_t* cand) {
  const uint64_t tag = rec_tag(epoch);
  const int words = 3 + 2 * n_steps;
  __syncthreads();   // the candidate is complete in LDS
  const uint64_t* src = reinterpret_cast<const uint64_t*>(cand);
  for (int q = threadIdx.x; q < world * words; q += blockDim.x) {
    const int r = q / words, j = q - r * words;
    const uint64_t w = src[cand_word(j, n_steps)];
    u64x2* dst = mail_rec(reinterpret_cast<void*>(s_peers[r]), slot, rank, world) + j;
    // (s_nop 1: the store reads its data registers before hipcc's next
    // instruction may overwrite them)
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1"
                 :
                 : "v"(dst), "v"(u64x2{(w & ~0xffffull) | tag, (w << 48) | tag})
                 : "memory");
  }
}

// Block 0, all threads: wait (bounded; chain error 5) until every rank's
// candidate of step `epoch` is complete in this rank's mailbox, decode them
// into LDS (cand_lds) and zero the granules.  Returns the LDS copy, or nullptr
// on a timeout.
__device__ const mpc_candidate_t* wait_mailbox(EpisodeState* S, void* mb, uint32_t epoch,
                                               uint32_t slot, int world, int n_steps,
                                               uint64_t ticks) {
  const uint32_t tag = rec_tag(epoch);
  const int words = 3 + 2 * n_steps, total = world * words;
  mpc_candidate_t* dst = cand_lds();
  const uint32_t deadline = wall_deadline(ticks);
  uint32_t it = 0;
  // one granule per thread and pass (world * words <= 256 in one pass: up to
  // 11 ranks at N = 10); a later chunk is polled after the earlier is in
#pragma unroll 1
  for (int base = 0; base < total; base += kBlock) {
    const int q = base + static_cast<int>(threadIdx.x);
    const int r = q / words, j = q - r * words;
    uint64_t* h = q < total ? reinterpret_cast<uint64_t*>(mail_rec(mb, slot, r, world) + j)
                            : nullptr;
    u64x2 g = {0, 0};
    for (;; ++it) {
      bool ok = true;
      if (h) {
        g.x = __hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        g.y = __hip_atomic_load(h + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = tagged_rec_fresh(g, tag);
      }
      if (__syncthreads_and(ok)) break;
      // uniform: every thread counts the same passes, thread 0's clock decides
      if ((it & 63) == 63 && block_wall_passed(deadline)) {
        if (threadIdx.x == 0) S->chain_error = 5u;
        return nullptr;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (h) {
      reinterpret_cast<uint64_t*>(&dst[r])[cand_word(j, n_steps)] = tagged_rec_key(g);
      __hip_atomic_store(h, uint64_t{0}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(h + 1, uint64_t{0}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
  return dst;
}

// Block 0 of a P2P launch (and the flush): complete step `tag` = prev: this
// rank's candidate from the previous launch's records, posted; the world
// candidates awaited; the global winner re-rolled into out_prev and the
// episode updated, publishing `publish_epoch` (0: end of the chain).
template <int INTEG, int ROT, bool TILED = false>
__device__ void p2p_complete(const mpc_episode_config_t& c, EpisodeState* S, void* mb, int world,
                             uint32_t prev, const Rec* __restrict__ part_prev, int n_part_prev,
                             const double* __restrict__ v_prev, const double* __restrict__ b_prev,
                             int64_t n_cand, int n_steps, int64_t index_base,
                             mpc_result_t* __restrict__ out_prev,
                             mpc_episode_log_t* __restrict__ log, int cap, uint32_t publish_epoch) {
  // the header (peers, rank: uncached, so a full memory round trip) loaded
  // before the records, its values parked in LDS after them
  __shared__ uint64_t s_peers[kMailMaxRanks];
  __shared__ int s_rank;
  const MailHdr* hdr = static_cast<const MailHdr*>(mb);
  __shared__ uint32_t s_err, s_seq;
  const uint64_t my_peer = static_cast<int>(threadIdx.x) < world ? hdr->peers[threadIdx.x] : 0;
  const int my_rank = threadIdx.x == 0 ? hdr->rank : 0;
  // an earlier step of this episode already timed out waiting for its peers
  // (error 5: a peer gone): fail fast instead of waiting the full budget
  // again on every later step.  Other errors say nothing about the peers.
  const uint32_t prior_err = threadIdx.x == 0 ? S->chain_error : 0u;
  const uint32_t seq = threadIdx.x == 0 ? S->p2p_seq : 0u;
  mpc_candidate_t* lc = cand_lds();
  records_candidate<TILED>(part_prev, n_part_prev, v_prev, b_prev, n_cand, n_steps, index_base,
                           lc);
  if (static_cast<int>(threadIdx.x) < world) s_peers[threadIdx.x] = my_peer;
  if (threadIdx.x == 0) {
    s_rank = my_rank;
    s_err = prior_err;
    s_seq = seq;
  }
  __syncthreads();
  const uint32_t slot = s_seq & 1u;
  post_candidate(s_peers, s_rank, world, prev, slot, n_steps, lc);
  const mpc_candidate_t* g =
      wait_mailbox(S, mb, prev, slot, world, n_steps, s_err == 5u ? 0ull : kPeerWaitTicks);
  if (threadIdx.x == 0) S->p2p_seq = s_seq + 1u;   // read by the next launch
  if (g) {
    advance_from_candidates<INTEG, ROT>(c, S, g, world, out_prev, log, cap, publish_epoch,
                                        ring_lds());
  } else if (publish_epoch) {   // timed out (error 5): publish the unchanged head
    chain_publish(S, publish_epoch);
  } else if (threadIdx.x < kPubWords) {   // ... or still end the chain
    __hip_atomic_store(&S->chain_pub[threadIdx.x], uint64_t{0}, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The mailboxes' self-test (mpc_mailbox_ping): lane r stores `tag` into
// rank r's ping word for this rank, then every lane waits (~0.1 s at most)
// for its rank's word in this mailbox; ok[0] = 1 if all `world` arrived.
__global__ __launch_bounds__(64) void k_mailbox_ping(void* mb, uint32_t tag, int32_t* ok) {
  MailHdr* hdr = static_cast<MailHdr*>(mb);
  const int world = hdr->world, rank = hdr->rank;
  const int r = threadIdx.x;
  if (r < world)
    __hip_atomic_store(&static_cast<MailHdr*>(reinterpret_cast<void*>(hdr->peers[r]))->ping[rank],
                       static_cast<uint64_t>(tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  bool seen = r >= world;
  const uint32_t deadline = wall_deadline(kPeerWaitTicks);   // one wave: uniform clock
  while (__ballot(!seen) != 0 && !wall_passed(deadline)) {
    if (!seen)
      seen = __hip_atomic_load(&hdr->ping[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ==
             static_cast<uint64_t>(tag);
    __builtin_amdgcn_s_sleep(8);
  }
  const bool all = __ballot(!seen) == 0;
  if (r == 0) ok[0] = all ? 1 : 0;
}

template <int INTEG, int ROT, bool TILED>
__global__ __launch_bounds__(kBlock) void k_episode_p2p_flush(
    mpc_episode_config_t c, EpisodeState* __restrict__ S, void* mailbox, uint32_t tag, int world,
    const Rec* __restrict__ part, int n_part, const double* __restrict__ v,
    const double* __restrict__ b, int64_t n_cand, int n_steps, int64_t index_base,
    mpc_result_t* __restrict__ out, mpc_episode_log_t* __restrict__ log, int cap) {
  p2p_complete<INTEG, ROT, TILED>(c, S, mailbox, world, tag, part, n_part, v, b, n_cand, n_steps,
                           index_base, out, log, cap, 0u);
}

// Launch bound of the chained kernel (waves per SIMD).  The one-GPU form runs
// 5 since round 6 (87 VGPRs, no scratch): at 6 it held 80 VGPRs with 4 spilled
// (12 B of scratch per lane) and ran 0.2-0.6 us slower per launch at config C
// and 0.7 us at D (same-box A/Bs, profiles/r06/ab_chain_waves.txt); the
// exchange and P2P forms run 5
// (at 6 they keep scratch: the P2P form spilled the work-item id at entry, a
// 4-B store per lane in EVERY wave — 2 MB of writes per config-C launch, the
// round-4 traffic excess; measured, 3 interleaved pairs each: exchange 36.73
// (6 waves) vs 36.31 us, profiles/r04/exchange_waves_ab.txt; P2P 31.17-31.47
// vs 30.83-31.11 us, profiles/r05/p2p_waves_ab.txt).
#ifndef MPC_CHAIN_FIN_WAVES
#define MPC_CHAIN_FIN_WAVES 5
#endif
template <int MODE>
constexpr int chain_waves() {
  return MODE == kChainFin ? MPC_CHAIN_FIN_WAVES : 5;
}

// PL2 (wheelbase a power of two) is a template parameter, not a runtime
// branch: with both rollout variants inlined the kernel held 119 VGPRs and
// spilled 191 SGPRs; one variant per instantiation: 108-112 VGPRs, 81-86.
// The tile blocks of a chained launch (blocks 1..): stream this step's
// controls through the LDS ring, speculating the step size until block 0 has
// published the step's constants (see k_episode_chain), then the criterion
// and the block's record into part[blockIdx.x - 1] (TAGGED: the exchange
// form, whose records block 0 of the SAME launch collects).  WAIT_TICKS bounds
// the wait for block 0's constants (kChainWaitTicks on one GPU,
// kXchgWaitTicks when block 0 itself waits for peers or a collective).
template <int INTEG, int ROT, bool PL2, bool TAGGED, uint64_t WAIT_TICKS, bool TILED>
__device__ __forceinline__ void chain_tiles(EpisodeState* __restrict__ S, uint32_t epoch,
                                            const double* __restrict__ v,
                                            const double* __restrict__ b, int64_t n_cand,
                                            int n_steps, Rec* __restrict__ part, int has_prev,
                                            const mpc_episode_config_t& ecfg) {
  constexpr int CPL = 2;
  __shared__ __attribute__((aligned(16))) uint32_t s_w[kPubWords];
  __shared__ uint32_t s_tag[kPubWords];
  __shared__ int s_final;
  // The step's final constants as the tile's epilogue reads them (the pose
  // transform, the criterion, an irregular candidate's recompute): straight
  // from the published words in LDS (s_w holds Consts' dwords), as VGPR
  // operands loaded where they are used.  Formed in SGPRs (readfirstlane)
  // they did not fit beside the loop's trig coefficients and spilled to VGPR
  // lanes: ~100 v_writelane / v_readlane per wave and tile.
  static_assert(offsetof(Consts, x) == 0 && alignof(Consts) <= 16, "Consts over s_w");
  const Consts& K = *reinterpret_cast<const Consts*>(s_w);
  Consts Kl;
  bool waited = false;
  // After the block's first control loads are in flight: the loop constants.
  // (K itself is formed only after the loop, from the LDS words, so that it
  // is not live in SGPRs across the loop.)
  auto pre0 = [&]() {
    if (threadIdx.x < 64) {
      bool fin = true;
      if (has_prev) {
        fin = chain_read(S, epoch, s_w, s_tag);
      } else if (threadIdx.x < kConstsWords) {   // block 0 only republishes the head
        s_w[threadIdx.x] = reinterpret_cast<const uint32_t*>(&S->h.K)[threadIdx.x];
      }
      if (threadIdx.x == 0) s_final = fin;
    }
    __syncthreads();
    Kl = consts_from_words(s_w);
    if (s_final) return;
    // speculate h from the published t: the previous step's (+ dt) or, if
    // block 0 already published it, this step's; torn -> NaN (recompute)
    const uint32_t g0 = __builtin_amdgcn_readfirstlane(s_tag[kConstsWords]);
    const uint32_t g1 = __builtin_amdgcn_readfirstlane(s_tag[kConstsWords + 1]);
    const uint64_t tb =
        (static_cast<uint64_t>(static_cast<uint32_t>(
             __builtin_amdgcn_readfirstlane(s_w[kConstsWords + 1]))) << 32) |
        static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(s_w[kConstsWords]));
    double t = __longlong_as_double(static_cast<long long>(tb));
    if (g0 == g1 && g0 == epoch - 1u)
      t = t + ecfg.delta_t;                                   // episode_prepare
    else if (!(g0 == g1 && g0 == epoch))
      t = __builtin_nan("");
    Kl.h = (t + ecfg.delta_t) - t;                            // consts_from_problem: t_b - t_a
  };
  // Three steps before the loop ends (blocks whose constants were not final
  // at the start): wave 0 loads the published words again, in flight with
  // the last control loads, so the end of the loop normally finds them there.
  uint64_t w_pre = 0;
  bool pre_issued = false;
  auto mid = [&]() {
    if (waited || pre_issued || s_final) return;
    pre_issued = true;
    if (threadIdx.x < kPubWords)
      w_pre = __hip_atomic_load(&S->chain_pub[threadIdx.x], __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
  };
  // After the loop: the final constants (called by every thread of the block
  // at the same point, see the clamp below).
  auto wait = [&]() {
    if (waited) return;
    waited = true;
    __syncthreads();   // LDS reuse
    if (!s_final) {
      if (threadIdx.x < 64) {
        bool fin = false;
        if (pre_issued) {
          const bool ok = threadIdx.x >= kPubWords || static_cast<uint32_t>(w_pre) == epoch;
          fin = __ballot(!ok) == 0;
          if (fin && threadIdx.x < kPubWords) s_w[threadIdx.x] = static_cast<uint32_t>(w_pre >> 32);
        }
        // (wave 0 only: its clock reads are uniform)
        // Two polls in flight, issued ~0.1 us apart: a poll's answer is as of
        // when it reached memory, so the words are seen about half a round
        // trip after they land instead of up to one and a half.
        if (!fin) {
          const uint32_t deadline = wall_deadline(WAIT_TICKS);
          const int q = threadIdx.x;
          uint64_t* const pw = &S->chain_pub[q < kPubWords ? q : 0];
          auto ld = [&]() {
            return __hip_atomic_load(pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          };
          auto here = [&](uint64_t w) {
            return __ballot(q < kPubWords && static_cast<uint32_t>(w) != epoch) == 0;
          };
          uint64_t a = ld(), b = 0, got = 0;
          for (;;) {
            __builtin_amdgcn_s_sleep(2);
            b = ld();
            if (here(a)) { got = a; fin = true; break; }
            if (wall_passed(deadline)) break;
            __builtin_amdgcn_s_sleep(2);
            a = ld();
            if (here(b)) { got = b; fin = true; break; }
            if (wall_passed(deadline)) break;
          }
          if (fin && q < kPubWords) s_w[q] = static_cast<uint32_t>(got >> 32);
        }
        if (!fin && threadIdx.x == 0) S->chain_error = 1u;
      }
      __syncthreads();
    }
  };
  // 32-bit candidate indices (the aligned path's rows are < 2^28 candidates,
  // wide_ok): the clamp below is one v_min with a scalar operand, no 64-bit
  // select holding its own registers across the loop
  const int32_t n32 = static_cast<int32_t>(n_cand);
  const int32_t n_tiles = (n32 + kBlock * CPL - 1) / (kBlock * CPL);
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  for (int32_t tile = blockIdx.x - 1; tile < n_tiles; tile += gridDim.x - 1) {
    const int32_t c0 = tile * (kBlock * CPL) + static_cast<int32_t>(threadIdx.x) * CPL;
    // lanes past the end of a partial tile roll the last pair again (result
    // ignored), so every lane reaches the barriers of pre0 / wait on the same path
    const int32_t cl = min(c0, n32 - CPL);
    double cst[CPL];
    // leading trig coefficients not pinned: the fifth wave per SIMD needs the
    // registers more (as the rect+cum stream kernel)
    // TILED: the tile's rows are one contiguous run (tile base + s * 1024
    // doubles), the lane's column its offset within the tile
    const int64_t tb0 = TILED ? static_cast<int64_t>(tile) * (2 * MPC_TILE) * n_steps : 0;
    rollout_lane_glds_k<INTEG, ROT, PL2, decltype(wait), decltype(pre0), decltype(mid),
                        false>(K, Kl, v + tb0, b + tb0, TILED ? 2 * MPC_TILE : n_cand,
                               TILED ? cl - tile * MPC_TILE : cl, n_steps, cst, wait, pre0, mid);
    if (c0 < n32) {
#pragma unroll
      for (int j = 0; j < CPL; ++j) {
        const uint64_t kk = cost_key_nonneg(cst[j]);
        if (kk < best_k) {
          best_k = kk;
          best_i = c0 + j;
        }
      }
    }
  }
  block_argmin<true>(best_k, best_i);   // (indices < n_cand < 2^31)
  if (threadIdx.x == 0) {
    if constexpr (TAGGED)
      store_tagged_rec(&part[blockIdx.x - 1], best_k, best_i, epoch);
    else
      part[blockIdx.x - 1] = Rec{best_k, best_i};
  }
}

template <int INTEG, int ROT, int MODE, bool PL2, bool TILED = false>
__global__ __launch_bounds__(kBlock, chain_waves<MODE>()) void k_episode_chain(
    EpisodeState* __restrict__ S, uint32_t epoch, const double* __restrict__ v,
    const double* __restrict__ b, int64_t n_cand, int n_steps, Rec* __restrict__ part,
    int has_prev, const Rec* __restrict__ part_prev, int n_part_prev,
    const double* __restrict__ v_prev, const double* __restrict__ b_prev, int64_t index_base,
    mpc_result_t* __restrict__ out_prev, const mpc_candidate_t* __restrict__ gathered,
    int n_gathered, mpc_episode_config_t ecfg, mpc_episode_log_t* __restrict__ log, int cap,
    uint32_t wait_tag) {
  static_assert(ROT == kRotCum, "chained steps need the pose-independent recurrence");
  if (blockIdx.x == 0) {
    if (has_prev) {
      // the completion of step k-1 publishes step k's constants itself, from
      // its LDS copy of the updated head (store_update)
      if constexpr (MODE == kChainP2P) {
        // the previous launch's records -> this rank's candidate, posted to
        // every mailbox; the world's awaited; selection and update.
        // (`gathered` carries the mailbox, n_gathered the world size, wait_tag
        // the previous step's epoch)
        p2p_complete<INTEG, ROT, TILED>(ecfg, S, const_cast<mpc_candidate_t*>(gathered), n_gathered,
                                 wait_tag, part_prev, n_part_prev, v_prev, b_prev, n_cand,
                                 n_steps, index_base, out_prev, log, cap, epoch);
      } else if constexpr (MODE == kChainFin) {
        const Consts Kp = S->h.K;
        const EpisodeHook hook{&S->h, log, cap, S->chain_pub, kPubWords, epoch, &S->chain_error};
        // (block 0 never fills the control ring: its LDS holds the re-roll)
        finalize_block<INTEG, ROT, true, kBlock, false, false, TILED>(
            part_prev, n_part_prev, Kp, v_prev, b_prev, n_cand, n_steps, index_base,
            S->h.incumbent, out_prev, ecfg, hook, ring_lds());
      } else {
        // overlapped exchange: the gathered candidates come from a collective
        // that ran beside this launch — wait for its mark, stage them in LDS.
        // P2P: wait for them in this rank's mailbox (`gathered` carries it,
        // n_gathered the world size, wait_tag the previous step's epoch).
        const mpc_candidate_t* g =
            wait_tag ? wait_gathered(S, wait_tag, gathered, n_gathered) : gathered;
        if (g)
          advance_from_candidates<INTEG, ROT>(ecfg, S, g, n_gathered, out_prev, log, cap,
                                              epoch, ring_lds());
        else   // timed out (chain error 4): publish the unchanged head so no tile hangs
          chain_publish(S, epoch);
      }
      __syncthreads();   // (the wheelbase check below reads the stored head)
    } else {
      chain_publish(S, epoch);   // no previous step: the head as reset / last updated
    }
    // The host picked PL2 from the caller's cfg; the tile blocks use the
    // published head's wheelbase terms.  If those disagree (a cfg other than
    // the one the state was reset with) every dphi would be formed with the
    // wrong form: flag it (chain_error = 2) instead of returning wrong costs
    // silently.  (chain_publish ended with a barrier after the head store.)
    if (threadIdx.x == 0 && (S->h.K.L_pow2 != 0) != PL2) S->chain_error = 2u;
    // kChainXchg passes the rank's candidate record in part_prev's slot (one
    // kernel argument fewer: a further SGPR pair spilled a VGPR)
    if constexpr (MODE == kChainXchg)
      collect_local_candidate(part, gridDim.x - 1, epoch, v, b, n_cand, n_steps, index_base,
                              reinterpret_cast<mpc_candidate_t*>(const_cast<Rec*>(part_prev)),
                              &S->chain_error);
    return;
  }
  static_assert(!TILED || MODE != kChainXchg, "the all_gather form reads SoA controls");
  chain_tiles<INTEG, ROT, PL2, MODE == kChainXchg,
              MODE == kChainFin ? kChainWaitTicks : kXchgWaitTicks, TILED>(
      S, epoch, v, b, n_cand, n_steps, part, has_prev, ecfg);
}

}  // namespace mpc
