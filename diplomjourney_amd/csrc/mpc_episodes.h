// mpc_episodes.h — R robots' MPC episodes, device-resident and batched.
//
// run_math_model.py:231-280 runs one episode per robot (random start and
// target, MPC steps until on target or stuck); its MPC step, at config.py's
// resolution, is math_model_tree.py's tree expansion (SURVEY Fact 2).  Here
// every robot is one block that runs its episode's MPC steps back to back in
// ONE launch — no host round trip per step and no lockstep:
//
//   per MPC step of robot r (block r):
//     grid        episode_grids: vector_of_velocities / vector_of_beta_angles
//                 around the robot's (v, beta) (:239-256), slow-down (:312-316)
//     candidates  the reference's enumeration k = a*|B| + b of the step's
//                 |V|*|B| constant sequences (:308-350), two per lane, from
//                 the grid in LDS (never in HBM)
//     rollout     the N-step recurrence of rollout_candidate_l (the kernels'
//                 arithmetic, bitwise), the criterion (:82-87)
//     arg-min     lowest index among the minima, strict < against the robot's
//                 incumbent (:351)
//     winner      re-rolled from its controls (emit_winner: the layer states)
//     update      episode_advance without restart: finishing logic m
//                 (:392-414), the stuck detector of cfg.stop_rule, operator
//                 events (math_mpc, :564-569; off for run_math_model),
//                 arrival (:542 / run_math_model.py:261), the step limit
//     log         one mpc_episode_log_t per step in the robot's ring
//
// Per-robot configurations (mpc_episode_config_t, copied into the state by
// mpc_episodes_reset) carry the start, target and rules of each robot: the
// run_math_model episodes (stop_rule 1, no events) and math_mpc episodes
// (stop_rule 0, the operator schedule) can share one launch.
#pragma once

#include "mpc_episode.h"

namespace mpc {

// One robot's episode in HBM.
struct RobotState {
  EpisodeHead h;
  StaleTraj st;        // right after the head: staged with it
  int32_t stop;        // 0 running, else the MPC_EP_* bits of the step that ended it
                       // (MPC_EP_ARRIVED with calls == 0: on target at the start)
  int32_t calls;       // MPC steps run
  int64_t candidates;  // candidates rolled out (the steps' |V| * |B|)
};
static_assert(offsetof(RobotState, st) == sizeof(EpisodeHead), "stale trajectory follows the head");

constexpr int32_t kEpEnded = MPC_EP_ARRIVED | MPC_EP_BREAK | MPC_EP_LIMIT;

// The state of n robots: RobotState[n], then each robot's configuration
// (mpc_episodes_reset copies them in), so a run needs nothing but the state.
__host__ __device__ inline size_t episodes_cfg_offset(int n) {
  return (static_cast<size_t>(n) * sizeof(RobotState) + 255) & ~static_cast<size_t>(255);
}

__global__ void k_episodes_reset(const mpc_episode_config_t* __restrict__ cfgs, int n,
                                 RobotState* __restrict__ robots) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const mpc_episode_config_t c = cfgs[r];
  RobotState R = {};
  episode_restart(c, R.h);
  episode_prepare(c, R.h);
  // the loop's head (:542, run_math_model.py:261): an episode that starts on
  // its target runs no step
  const double ex = R.h.x_t - R.h.x, ey = R.h.y_t - R.h.y;
  R.stop = (ex * ex + ey * ey <= c.eps) ? MPC_EP_ARRIVED : 0;
  robots[r] = R;
}

// One candidate with constant control (v, b) over n_steps, exactly as the
// rollout kernels evaluate it (rollout_candidate_l without the trajectory:
// the core recurrence, and the safe one for an irregular candidate).
template <int INTEG, int ROT, bool PL2>
__device__ __forceinline__ double const_candidate_cost_l(const Consts& K, double v, double b,
                                                         int n_steps) {
  double x, y, ph, s, c;
  step_start<ROT>(K, x, y, ph, s, c);
  bool bad = false;
  for (int st = 0; st < n_steps; ++st) step_core<INTEG, ROT, PL2>(x, y, ph, s, c, v, b, K, bad);
  if constexpr (ROT == kRotCum) {
    if (!bad) cum_pose<PL2>(K, x, y, x, y);
  }
  if (bad) {
    x = K.x;
    y = K.y;
    ph = K.phi;
    for (int st = 0; st < n_steps; ++st) step_safe<INTEG>(x, y, ph, v, b, K);
  }
  return cost(x, y, K);
}

template <int INTEG, int ROT>
__device__ __forceinline__ double const_candidate_cost(const Consts& K, double v, double b,
                                                       int n_steps) {
  return K.L_pow2 ? const_candidate_cost_l<INTEG, ROT, true>(K, v, b, n_steps)
                  : const_candidate_cost_l<INTEG, ROT, false>(K, v, b, n_steps);
}

// Two candidates' recurrences in one loop — independent chains the scheduler
// interleaves — each with exactly const_candidate_cost_l's operations (the
// same bits per candidate).
// NS > 0: the horizon as a compile-time constant (the reference's N = 3):
// the loop unrolls, and the steps' sin/cos — which depend only on the heading
// chain, a sum of the candidate's constant increment — overlap.
template <int INTEG, int ROT, bool PL2, int NS = 0>
__device__ __forceinline__ void const_pair_cost_l(const Consts& K, const double (&v)[2],
                                                  const double (&b)[2], int n_steps,
                                                  double (&cst)[2]) {
  if constexpr (NS > 0) n_steps = NS;
  double x[2], y[2], ph[2], s[2], c[2];
  bool bad[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    step_start<ROT>(K, x[j], y[j], ph[j], s[j], c[j]);
    bad[j] = false;
  }
  auto one_step = [&]() {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      step_core<INTEG, ROT, PL2>(x[j], y[j], ph[j], s[j], c[j], v[j], b[j], K, bad[j]);
  };
  if constexpr (NS > 0) {
#pragma unroll
    for (int st = 0; st < NS; ++st) one_step();
  } else {
    for (int st = 0; st < n_steps; ++st) one_step();
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if constexpr (ROT == kRotCum) {
      if (!bad[j]) cum_pose<PL2>(K, x[j], y[j], x[j], y[j]);
    }
    if (bad[j]) {
      x[j] = K.x;
      y[j] = K.y;
      ph[j] = K.phi;
      for (int st = 0; st < n_steps; ++st) step_safe<INTEG>(x[j], y[j], ph[j], v[j], b[j], K);
    }
    cst[j] = cost(x[j], y[j], K);
  }
}

template <int INTEG, int ROT, int NS = 0>
__device__ __forceinline__ void const_pair_cost(const Consts& K, const double (&v)[2],
                                                const double (&b)[2], int n_steps,
                                                double (&cst)[2]) {
  if (K.L_pow2)
    const_pair_cost_l<INTEG, ROT, true, NS>(K, v, b, n_steps, cst);
  else
    const_pair_cost_l<INTEG, ROT, false, NS>(K, v, b, n_steps, cst);
}

// The step's winner (constant controls v, b) re-derived by ONE lane with the
// rollout's own per-candidate recurrence — rollout_candidate_l's operations,
// the core form or, for a flagged candidate, the safe form — its layer states
// 0..2 (clamped to the horizon) into w.tr: the same bits as emit_winner's
// block-wide re-roll for the direct and rotation heading forms, without its
// barriers (kRotCum, whose sums run scaled, keeps emit_winner).
template <int INTEG, int ROT, bool PL2>
__device__ inline void const_winner_states_l(const Consts& K, double v, double b, int n_steps,
                                             Winner& w) {
  static_assert(ROT != kRotCum, "kRotCum winners are re-rolled by emit_winner");
  auto keep = [&](int st, double x, double y, double ph) {
    // (constant indices only: a dynamically indexed w.tr would live in scratch)
    if (st == 0) {
      w.tr[0][0] = x, w.tr[0][1] = y, w.tr[0][2] = ph;
    } else if (st == 1) {
      w.tr[1][0] = x, w.tr[1][1] = y, w.tr[1][2] = ph;
    } else if (st == 2) {
      w.tr[2][0] = x, w.tr[2][1] = y, w.tr[2][2] = ph;
    }
  };
  double x, y, ph, s, c;
  step_start<ROT>(K, x, y, ph, s, c);
  bool bad = false;
  for (int st = 0; st < n_steps; ++st) {
    step_core<INTEG, ROT, PL2>(x, y, ph, s, c, v, b, K, bad);
    keep(st, x, y, ph);
  }
  if (bad) {
    x = K.x;
    y = K.y;
    ph = K.phi;
    for (int st = 0; st < n_steps; ++st) {
      step_safe<INTEG>(x, y, ph, v, b, K);
      keep(st, x, y, ph);
    }
  }
  for (int k = n_steps; k < 3; ++k)   // a horizon below 3: the last layer repeated
    for (int q = 0; q < 3; ++q) {
      const double last = n_steps == 1 ? w.tr[0][q] : w.tr[1][q];
      if (k == 1) w.tr[1][q] = last;
      if (k == 2) w.tr[2][q] = last;
    }
}

// The same states for the direct heading form (ROT = 0), lane-parallel over
// the steps, by wave 0 (all 64 lanes, n_steps <= 64): the control is constant,
// so lane s forms its step's heading phi_s = phi + dphi (+ dphi ...) with
// exactly the serial chain's additions, its sin / cos and (QK21) position
// increments; lane 0 then only sums them in the serial order (QK21: x + inc;
// RECT: the fused fma(v h, cos, x)) — the serial recurrence's bits, its
// dependent chain cut from n_steps x (sin/cos + quadratures) to one.  A
// flagged candidate (|beta| > kTanMax, |phi_s| > kFastMax) takes lane 0's
// serial path (const_winner_states_l: the core form, then the safe one).
template <int INTEG, bool PL2>
__device__ inline void wave_winner_states_l(const Consts& K, double v, double b, int n_steps,
                                            Winner& w) {
  const int lane = threadIdx.x & 63;
  double ph = K.phi, sn = 0.0, cs = 0.0, ix = 0.0, iy = 0.0;
  bool bad = !(fabs(b) <= trig::kTanMax);
  const double t = trig::tan_small(b);
  double dphi, vh = 0.0;
  if constexpr (PL2 && INTEG == MPC_INTEG_RECT) {
    vh = v * K.h;
    dphi = (vh * K.inv_L) * t;                                 // step_core's form
  } else {
    const double wv = PL2 ? v * K.inv_L : v / K.L;
    dphi = heading_incr<INTEG>(wv, t, K);
  }
  if (lane < n_steps) {
    for (int j = 0; j <= lane; ++j) ph = ph + dphi;
    bad |= !(fabs(ph) <= trig::kFastMax);
    trig::sincos_core(ph, &sn, &cs);
    if constexpr (INTEG != MPC_INTEG_RECT) {
      ix = quad_const<INTEG>(v * cs, K);                      // position_step's increment
      iy = quad_const<INTEG>(v * sn, K);
    }
  }
  const bool any_bad = __ballot(lane < n_steps && bad) != 0;
  if (lane != 0) return;
  if (any_bad) {
    const_winner_states_l<INTEG, 0, PL2>(K, v, b, n_steps, w);
    return;
  }
  auto rl = [](double val, int src) {
    const uint64_t u = static_cast<uint64_t>(__double_as_longlong(val));
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<int>(u), src);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<int>(u >> 32), src);
    return __longlong_as_double(static_cast<long long>((static_cast<uint64_t>(hi) << 32) | lo));
  };
  double x = K.x, y = K.y;
  for (int st = 0; st < n_steps; ++st) {
    if constexpr (INTEG == MPC_INTEG_RECT) {
      const double vhs = PL2 ? vh : v * K.h;                  // = position_step<RECT>
      x = fma(vhs, rl(cs, st), x);
      y = fma(vhs, rl(sn, st), y);
    } else {
      x = x + rl(ix, st);
      y = y + rl(iy, st);
    }
    const double p = rl(ph, st);
    if (st == 0) {
      w.tr[0][0] = x, w.tr[0][1] = y, w.tr[0][2] = p;
    } else if (st == 1) {
      w.tr[1][0] = x, w.tr[1][1] = y, w.tr[1][2] = p;
    } else if (st == 2) {
      w.tr[2][0] = x, w.tr[2][1] = y, w.tr[2][2] = p;
    }
  }
  for (int k = n_steps; k < 3; ++k)
    for (int q = 0; q < 3; ++q) {
      const double last = n_steps == 1 ? w.tr[0][q] : w.tr[1][q];
      if (k == 1) w.tr[1][q] = last;
      if (k == 2) w.tr[2][q] = last;
    }
}

// Block r = robot r: up to max_calls MPC steps of its episode (fewer if it
// ends).  log: [n][cap] ring per robot; progress (optional): {calls, stop,
// candidates} per robot after the launch.
// NT = 256: 4 waves per SIMD (<= 128 VGPRs), 4 robots per CU at a time; a
// robot's serial phases (grid, re-roll, update: one lane) then share their
// SIMD with three other robots' waves.
// NT = 64 (the default for N <= 21): ONE wave per robot — 1000 robots are
// ~1 wave per SIMD, so the serial phases run uncontended; a lane rolls out
// its candidates two at a time (const_pair_cost), the arg-min is one DPP
// wave reduction and the barriers are a single wave's.
// PAIR: a lane's candidates two at a time, interleaved (const_pair_cost);
// else one after the other (more waves per SIMD fit: <= 128 VGPRs).
constexpr int kEpisodesWaves = 4;
template <int INTEG, int ROT, int NT = kBlock, bool PAIR = (NT == 64)>
__global__ __launch_bounds__(NT, PAIR ? 2 : kEpisodesWaves) void k_episodes_run(
    const mpc_episode_config_t* __restrict__ cfgs, RobotState* __restrict__ robots, int n_steps,
    int max_calls, mpc_episode_log_t* __restrict__ log, int cap,
    mpc_episodes_progress_t* __restrict__ progress) {
  static_assert(NT == 64 || NT == kBlock, "one wave or one standard block per robot");
  const int r = blockIdx.x;
  const mpc_episode_config_t& c = cfgs[r];
  RobotState* __restrict__ R = &robots[r];
  __shared__ uint64_t s_head[kStoredWords];   // head + stale trajectory
  __shared__ double s_v[kEpMaxGrid], s_b[kEpMaxGrid];
  __shared__ int s_nv, s_nb, s_stop, s_calls;
  __shared__ uint64_t s_bk;
  __shared__ int64_t s_bi;
  __shared__ mpc_episode_log_t s_log;
  __shared__ mpc_result_t s_out;
  __shared__ EmitLds lds;
  for (int q = threadIdx.x; q < kStoredWords; q += NT)
    s_head[q] = reinterpret_cast<const uint64_t*>(R)[q];
  if (threadIdx.x == 0) {
    s_stop = R->stop;
    s_calls = R->calls;
  }
  int64_t cands = 0;   // (thread 0)
  for (int call = 0; call < max_calls; ++call) {
    __syncthreads();
    if (s_stop) break;   // uniform
    const EpisodeHead* Hs = reinterpret_cast<const EpisodeHead*>(s_head);
    if (threadIdx.x < 64) {
      int nv, nb;
      episode_grids(c, *Hs, s_v, s_b, nv, nb);
      if (threadIdx.x == 0) {
        s_nv = nv;
        s_nb = nb;
      }
    }
    __syncthreads();
    const Consts K = uniform_consts(Hs->K);
    const double incumbent = Hs->incumbent;
    const int nv = s_nv, nb = s_nb, n_grid = nv * nb;
    uint64_t best_k = ~0ull;
    int64_t best_i = INT64_MAX;
    if constexpr (PAIR) {
      // lane l: candidates l, l + NT, l + 2 NT, ... two per pass (ascending per
      // lane: strict < keeps the first)
      for (int k0 = threadIdx.x; k0 < n_grid; k0 += 2 * NT) {
        const int k1 = k0 + NT;
        const bool has1 = k1 < n_grid;
        const int kq = has1 ? k1 : k0;   // (a valid stand-in; its cost is not used)
        const double vv[2] = {s_v[k0 / nb], s_v[kq / nb]};
        const double bb[2] = {s_b[k0 % nb], s_b[kq % nb]};
        double cst[2];
        if (n_steps == 3)   // uniform: the reference's horizon, unrolled
          const_pair_cost<INTEG, ROT, 3>(K, vv, bb, n_steps, cst);
        else
          const_pair_cost<INTEG, ROT>(K, vv, bb, n_steps, cst);
        uint64_t kk = cost_key_nonneg(cst[0]);
        if (kk < best_k) {
          best_k = kk;
          best_i = k0;
        }
        kk = cost_key_nonneg(cst[1]);
        if (has1 && kk < best_k) {
          best_k = kk;
          best_i = k1;
        }
      }
    } else {
      for (int k0 = 2 * threadIdx.x; k0 < n_grid; k0 += 2 * kBlock) {
#pragma unroll 1
        for (int j = 0; j < 2; ++j) {
          const int k = k0 + j;   // ascending per lane: strict < keeps the first
          if (k < n_grid) {
            const uint64_t kk = cost_key_nonneg(
                const_candidate_cost<INTEG, ROT>(K, s_v[k / nb], s_b[k % nb], n_steps));
            if (kk < best_k) {
              best_k = kk;
              best_i = k;
            }
          }
        }
      }
    }
    if constexpr (NT == 64)
      wave_argmin32(best_k, best_i);   // (every lane holds the minimum)
    else
      block_argmin<true>(best_k, best_i);
    if (threadIdx.x == 0) {
      s_bk = best_k;
      s_bi = best_i;
      cands += n_grid;
    }
    __syncthreads();
    const uint64_t bk = s_bk;
    const int64_t bi = s_bi;
    // (in LDS: thread 0's private copy spilled to scratch, a memory round
    // trip per field on the step's serial path)
    __shared__ Winner s_win;
    Winner& win = s_win;
    if constexpr (ROT != kRotCum) {
      // wave 0 re-derives the winner itself (wave_winner_states_l for the
      // direct heading form, one lane's const_winner_states_l for the
      // rotation form): no block barriers
      if (threadIdx.x < 64) {
        if (threadIdx.x == 0) {
          win.n_steps = n_steps;
          win.cost = bk == ~0ull ? __builtin_inf() : key_cost(bk);
          win.index = bk == ~0ull ? -1 : bi;
          win.found = bk != ~0ull && key_cost(bk) < incumbent ? 1 : 0;
        }
        if (bk != ~0ull) {
          const double wv = s_v[bi / nb], wb = s_b[bi % nb];
          if (threadIdx.x == 0) {
            win.v = wv;
            win.beta = wb;
          }
          if constexpr (ROT == 0) {
            if (K.L_pow2)
              wave_winner_states_l<INTEG, true>(K, wv, wb, n_steps, win);
            else
              wave_winner_states_l<INTEG, false>(K, wv, wb, n_steps, win);
          } else if (threadIdx.x == 0) {
            if (K.L_pow2)
              const_winner_states_l<INTEG, ROT, true>(K, wv, wb, n_steps, win);
            else
              const_winner_states_l<INTEG, ROT, false>(K, wv, wb, n_steps, win);
          }
        }
      }
    } else {
      // the winner's controls (constant over the horizon) staged for its re-roll
      if (bk != ~0ull && threadIdx.x < n_steps) {
        lds.pv[threadIdx.x] = s_v[bi / nb];
        lds.pb[threadIdx.x] = s_b[bi % nb];
      }
      // (v / b: the staged controls again, never read since pre_v / pre_b are
      // given — null constants there crash hipcc 7.2's inliner, which also
      // sees k_finalize's call of the same instantiation)
      emit_winner<INTEG, ROT>(K, lds.pv, lds.pb, 1, n_steps, bk, bi, bi, incumbent, &s_out,
                              &lds, &win, lds.pv, lds.pb, false);
    }
    if (threadIdx.x == 0) {   // (emit_winner, if it ran, ended with a barrier)
      EpisodeHead H;
      __builtin_memcpy(&H, s_head, sizeof(EpisodeHead));
      episode_advance<false>(c, H, *reinterpret_cast<StaleTraj*>(&s_head[kHeadWords]), win,
                             s_log);
      __builtin_memcpy(s_head, &H, sizeof(EpisodeHead));
      if (s_log.status & kEpEnded) s_stop = s_log.status;
      s_calls += 1;
    }
    __syncthreads();
    if (log && cap > 0 && threadIdx.x < kLogWords)
      reinterpret_cast<uint64_t*>(&log[static_cast<int64_t>(r) * cap + s_log.step % cap])
          [threadIdx.x] = reinterpret_cast<const uint64_t*>(&s_log)[threadIdx.x];
  }
  __syncthreads();
  for (int q = threadIdx.x; q < kStoredWords; q += NT) reinterpret_cast<uint64_t*>(R)[q] = s_head[q];
  if (threadIdx.x == 0) {
    R->stop = s_stop;
    R->calls = s_calls;
    R->candidates += cands;
    if (progress) {
      progress[r].calls = s_calls;
      progress[r].stop = s_stop;
      progress[r].candidates = R->candidates;
    }
  }
}

}  // namespace mpc
