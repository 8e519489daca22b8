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

// Block r = robot r: up to max_calls MPC steps of its episode (fewer if it
// ends).  log: [n][cap] ring per robot; progress (optional): {calls, stop,
// candidates} per robot after the launch.
// 4 waves per SIMD (<= 128 VGPRs): 4 robots per CU at a time.
constexpr int kEpisodesWaves = 4;
template <int INTEG, int ROT>
__global__ __launch_bounds__(kBlock, kEpisodesWaves) void k_episodes_run(
    const mpc_episode_config_t* __restrict__ cfgs, RobotState* __restrict__ robots, int n_steps,
    int max_calls, mpc_episode_log_t* __restrict__ log, int cap,
    mpc_episodes_progress_t* __restrict__ progress) {
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
  if (threadIdx.x < kStoredWords)
    s_head[threadIdx.x] = reinterpret_cast<const uint64_t*>(R)[threadIdx.x];
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
    block_argmin<true>(best_k, best_i);
    if (threadIdx.x == 0) {
      s_bk = best_k;
      s_bi = best_i;
      cands += n_grid;
    }
    __syncthreads();
    // the winner's controls (constant over the horizon) staged for its re-roll
    const uint64_t bk = s_bk;
    const int64_t bi = s_bi;
    if (bk != ~0ull && threadIdx.x < n_steps) {
      lds.pv[threadIdx.x] = s_v[bi / nb];
      lds.pb[threadIdx.x] = s_b[bi % nb];
    }
    Winner win;
    // (v / b: the staged controls again, never read since pre_v / pre_b are
    // given — null constants there crash hipcc 7.2's inliner, which also
    // sees k_finalize's call of the same instantiation)
    emit_winner<INTEG, ROT>(K, lds.pv, lds.pb, 1, n_steps, bk, bi, bi, incumbent, &s_out, &lds,
                            &win, lds.pv, lds.pb, false);
    if (threadIdx.x == 0) {   // (emit_winner ended with a barrier)
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
  if (threadIdx.x < kStoredWords) reinterpret_cast<uint64_t*>(R)[threadIdx.x] = s_head[threadIdx.x];
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
