// mpc_fulltree.h — full-tree MPC of run_math_model.py / math_model.py
// (SURVEY §8f 3): S1^3 leaves per MPC step, generated from the leaf index.
//
// predictive_control (run_math_model.py:133-228) fills leaf j = k0*S1^2 +
// k1*S1 + k2 with the controls u_k0, u_k1, u_k2 (u_k = (V[k / |B|],
// B[k % |B|]), loop order :158-160) applied in turn to the initial state, and
// scans the heading-term criterion (:82-86) with strict < against a running
// incumbent (:193-196).
//
//   k_ft_controls   per control k: v, dphi = Q((v/L) tan(beta)) (the same for
//                   all three layers: one quad window per call), the rotation
//                   factors of dphi, v*h; a launch-wide flag when some
//                   |dphi| > kRotMax (the rotation form is then not used)
//   k_ft_leaves     work units = (group of 64 consecutive (k0, k1) pairs, k2);
//                   a shard owns a contiguous unit range, each wave an equal
//                   contiguous share of it, one pair per lane: each lane derives
//                   its pair's layer-0 and layer-1 states once per group, then
//                   runs its k2 with the control WAVE-UNIFORM (scalar loads, no
//                   per-leaf vector memory traffic); lexicographic (cost, j)
//                   arg-min per lane -> wave -> block record
//   k_ft_finalize   record reduction, the winner's three layers re-derived
//                   with the same functions
#pragma once

#include "mpc_kernels.h"

namespace mpc {

struct FtCtl {
  double v, beta, dphi, sd, cd;   // sd, cd = sin / cos of dphi (ROT)
  double vh;   // v * h (RECT's position increment factor, formed once per control)
};

struct FtState {
  double x, y, ph, s, c;
};

// The criterion's per-problem terms, folded once per problem (ft_crit) so that
// a leaf spends 27 VALU on it instead of 35:
//   10000*dist_target + 10*(arctan(x_t/y_t) - phi)^2 + 100*dist_line^2
// (run_math_model.py:82-86) with dist_line = |A x - B y + C1 - C2| / hyp
// (:53-61) evaluated as lin = fma(A, x, fma(-B, y, C1 - C2)) and
// 100*dist_line^2 = (lin * K2) * lin, K2 = 100 / hyp^2; the sum as
// fma(10000, dist_target, fma(lin * K2, lin, (10 a) a)).  Other roundings than
// the script's order (a few ulps of the cost; the tests' 1e-12 bar).  The
// line-origin sentinel (:57-58, dist_line = 1000) replaces lin by
// S = sqrt(1e8 / K2): its term is 1e8 to within an ulp or two, and such a
// leaf (the state AT the line origin, cost >= 1e8) never wins.
struct FtCrit {
  double x_t, y_t, x_0, y_0, A, nB, C, K2, S, atan_t;
};

MPC_HD __forceinline__ FtCrit ft_crit(const Consts& K, double atan_t) {
  FtCrit F;
  F.x_t = K.x_t;
  F.y_t = K.y_t;
  F.x_0 = K.x_0;
  F.y_0 = K.y_0;
  F.A = K.A;
  F.nB = -K.B;
  F.C = K.C1 - K.C2;
  F.K2 = 100.0 * (K.inv_den * K.inv_den);
  F.S = sqrt(1e8 / F.K2);
  F.atan_t = atan_t;
  return F;
}

MPC_HD __forceinline__ double cost_fulltree(double x, double y, double ph, const FtCrit& F) {
  const double a = F.atan_t - ph;
  const double ex = F.x_t - x, ey = F.y_t - y;
  const double dist_target = crit_sqrt(fma(ex, ex, ey * ey));
  const double lin0 = fma(F.A, x, fma(F.nB, y, F.C));
  const double lin = (x == F.x_0 && y == F.y_0) ? F.S : lin0;
  return fma(10000.0, dist_target, fma(lin * F.K2, lin, (a * 10.0) * a));
}

// iteration_of_predict (:111-115) with a precomputed control: heading first,
// then the position with the new heading.  ROT: (s, c) rotated by the
// control's sin / cos (the candidate rollout's complex product, 4 VALU).
template <int INTEG, bool ROT>
MPC_HD __forceinline__ FtState ft_apply(const FtState& in, const FtCtl& u, const Consts& K) {
  FtState o;
  o.ph = in.ph + u.dphi;
  if constexpr (ROT) {
    o.s = in.s;
    o.c = in.c;
    trig::rotate_sc(u.sd, u.cd, o.s, o.c);
  } else {
    trig::sincos_fast(o.ph, &o.s, &o.c);
  }
  if constexpr (INTEG == MPC_INTEG_RECT) {   // = position_step: fma(v * h, trig, p)
    o.x = fma(u.vh, o.c, in.x);
    o.y = fma(u.vh, o.s, in.y);
  } else {
    o.x = position_step<INTEG>(in.x, u.v, o.c, K);
    o.y = position_step<INTEG>(in.y, u.v, o.s, K);
  }
  return o;
}

template <int INTEG>
__global__ __launch_bounds__(kBlock) void k_ft_controls(Consts K, const double* __restrict__ V,
                                                        const double* __restrict__ B, int nb,
                                                        int64_t s1, FtCtl* __restrict__ ctl,
                                                        uint32_t* __restrict__ no_rot) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= s1) return;
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
    atomicOr(no_rot, 1u);
  }
  ctl[k] = u;
}

constexpr int kFtWaves = 7;    // launch bound (waves per SIMD): <= 72 VGPRs, no scratch

// Work units: u = g * S1 + k2 — group g of 64 consecutive (k0, k1) pairs (one
// per lane), control k2 of the last layer.  A launch (or shard, or robot) owns
// the contiguous range [u_lo, u_hi); wave `wave` of `n_waves` takes an equal
// contiguous share of it (+-1 unit).  Round 4 dealt whole (group, 256-k2
// chunk) items round-robin: at S1 = 451 that was one item per wave with the
// 256- and 195-k2 chunks landing on alternate SIMDs and 6 or 7 waves per
// SIMD — the launch waited on its most loaded SIMDs.
__host__ __device__ __forceinline__ int64_t ft_units(int64_t s1) {
  return ((s1 * s1 + 63) / 64) * s1;
}

// The leaf (k0, k1, k2) of lane-pair mm and control k2 from the layer-1 state.
template <int INTEG, bool ROT>
__device__ __forceinline__ double ft_leaf(const FtState& l1, const FtCtl& u, const Consts& K,
                                          const FtCrit& F) {
  const FtState lf = ft_apply<INTEG, ROT>(l1, u, K);
  return cost_fulltree(lf.x, lf.y, lf.ph, F);
}

// wave / n_waves: this wave's rank among the waves that share [u_lo, u_hi)
// (the launch's waves; a block's own in the device-resident episodes).
// Each lane keeps the first strict minimum of its leaves — which ascend in
// leaf index (units ascend: (k0, k1) with g, k2 within a group) — in three
// steps, so that the per-leaf bookkeeping is 1.5 VALU instead of 3:
//   * per 4 consecutive k2 (a quad): the quad minimum (3 fmin); if it is
//     strictly below the lane's best, the quad's first k2 (one compare, one
//     32-bit select) — the first quad reaching a value keeps it, as the scan
//     would;
//   * per piece (the wave's run of k2 within one group): the group of the best
//     quad, if the piece improved it;
//   * once per wave: the winning quad re-evaluated (the same operations, so the
//     same bits) to find its first leaf at the minimum.
// Costs are compared as doubles: the criterion is >= 0, where the double order
// is the cost keys' (+-0 equal, +inf and NaN never below a best; fmin ignores
// a NaN), so the key is formed once per lane.
template <int INTEG, bool ROT>
__device__ __forceinline__ void ft_leaves_body(const Consts& K, const FtCrit& F,
                                               const FtCtl* __restrict__ ctl, int64_t s1,
                                               int64_t u_lo, int64_t u_hi,
                                               uint64_t& best_k, int64_t& best_i, int64_t wave,
                                               int64_t n_waves) {
  const int lane = threadIdx.x & 63;
  const int64_t n_pairs = s1 * s1;
  const int64_t total = u_hi - u_lo, share = total / n_waves, rem = total % n_waves;
  int64_t u = u_lo + wave * share + (wave < rem ? wave : rem);
  const int64_t u_end = u + share + (wave < rem ? 1 : 0);
  const FtState s0{K.x, K.y, K.phi, K.s0, K.c0};
  double best_c = key_cost(best_k);   // (+inf: none yet)
  int64_t best_mm = -1;               // the pair of the lane's best quad (-1: best_i stands)
  int32_t best_q = 0;                 // ... and its first k2
  while (u < u_end) {   // wave-uniform
    const int64_t g = u / s1;
    const int64_t k2_lo = u - g * s1;
    const int64_t k2_hi = (s1 - k2_lo < u_end - u) ? s1 : k2_lo + (u_end - u);
    u += k2_hi - k2_lo;
    const int64_t m = g * 64 + lane;           // this lane's (k0, k1) pair
    const int64_t mm = m < n_pairs ? m : n_pairs - 1;
    const int64_t k0 = mm / s1, k1 = mm - k0 * s1;
    const FtState l0 = ft_apply<INTEG, ROT>(s0, ctl[k0], K);
    const FtState l1 = ft_apply<INTEG, ROT>(l0, ctl[k1], K);
    int32_t q = -1;   // the piece's best quad (first k2; -1: none)
    int64_t k2 = k2_lo;
    for (; k2 + 4 <= k2_hi; k2 += 4) {   // wave-uniform controls
      const double c0 = ft_leaf<INTEG, ROT>(l1, ctl[k2], K, F);
      const double c1 = ft_leaf<INTEG, ROT>(l1, ctl[k2 + 1], K, F);
      const double c2 = ft_leaf<INTEG, ROT>(l1, ctl[k2 + 2], K, F);
      const double c3 = ft_leaf<INTEG, ROT>(l1, ctl[k2 + 3], K, F);
      const double cm = fmin(fmin(c0, c1), fmin(c2, c3));
      if (cm < best_c) q = static_cast<int32_t>(k2);
      best_c = fmin(best_c, cm);
    }
    for (; k2 < k2_hi; ++k2) {   // the piece's last < 4 leaves: quads of one
      const double c = ft_leaf<INTEG, ROT>(l1, ctl[k2], K, F);
      if (c < best_c) q = static_cast<int32_t>(k2);
      best_c = fmin(best_c, c);
    }
    if (q >= 0) {
      best_mm = mm;
      best_q = q;
    }
  }
  if (__ballot(best_mm >= 0) != 0) {   // the winning quad's first leaf at best_c
    if (best_mm >= 0) {
      const int64_t k0 = best_mm / s1, k1 = best_mm - k0 * s1;
      const FtState l0 = ft_apply<INTEG, ROT>(s0, ctl[k0], K);
      const FtState l1 = ft_apply<INTEG, ROT>(l0, ctl[k1], K);
      // (a quad of one — a piece's last leaves — matches at j = 0: the scan
      // never reaches past its quad)
      int32_t hit = -1;
      for (int32_t j = 0; j < 4 && hit < 0 && best_q + j < s1; ++j)
        if (ft_leaf<INTEG, ROT>(l1, ctl[best_q + j], K, F) == best_c) hit = best_q + j;
      best_i = best_mm * s1 + (hit >= 0 ? hit : best_q);   // (hit >= 0: same bits)
    }
  }
  best_k = cost_key_nonneg(best_c);   // (+inf: ~0, no finite leaf)
}

template <int INTEG, bool ROT>
__global__ __launch_bounds__(kBlock, kFtWaves) void k_ft_leaves(Consts K, double atan_t,
                                                      const FtCtl* __restrict__ ctl,
                                                      const uint32_t* __restrict__ no_rot,
                                                      int64_t s1, int64_t u_lo,
                                                      int64_t u_hi, Rec* __restrict__ part) {
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * kWaves +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n_waves = static_cast<int64_t>(gridDim.x) * kWaves;
  const FtCrit F = ft_crit(K, atan_t);
  if (ROT && *no_rot == 0u)
    ft_leaves_body<INTEG, true>(K, F, ctl, s1, u_lo, u_hi, best_k, best_i, wave, n_waves);
  else
    ft_leaves_body<INTEG, false>(K, F, ctl, s1, u_lo, u_hi, best_k, best_i, wave, n_waves);
  block_argmin(best_k, best_i);
  if (threadIdx.x == 0) part[blockIdx.x] = Rec{best_k, best_i};
}

template <int INTEG, bool ROT>
__global__ __launch_bounds__(kFinBlock) void k_ft_finalize(
    const Rec* __restrict__ part, int n_part, Consts K, const FtCtl* __restrict__ ctl,
    const uint32_t* __restrict__ no_rot, int64_t s1, double incumbent,
    mpc_fulltree_result_t* __restrict__ out) {
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
  if (threadIdx.x != 0) return;
  for (int w = 1; w < kFinBlock / 64; ++w)
    if (rec_less(s_key[w], s_idx[w], k, i)) {
      k = s_key[w];
      i = s_idx[w];
    }
  out->s1 = static_cast<int32_t>(s1);
  if (k == ~0ull) {
    out->cost = __builtin_inf();
    out->leaf = -1;
    out->found = 0;
    return;
  }
  const double c = key_cost(k);
  out->cost = c;
  out->leaf = i;
  out->found = c < incumbent ? 1 : 0;
  const int64_t kk[3] = {i / (s1 * s1), (i / s1) % s1, i % s1};
  const bool rot = ROT && *no_rot == 0u;
  FtState st{K.x, K.y, K.phi, K.s0, K.c0};
  for (int l = 0; l < 3; ++l) {
    const FtCtl u = ctl[kk[l]];
    st = rot ? ft_apply<INTEG, true>(st, u, K) : ft_apply<INTEG, false>(st, u, K);
    out->k[l] = kk[l];
    out->v[l] = u.v;
    out->beta[l] = u.beta;
    out->traj[l][0] = st.x;
    out->traj[l][1] = st.y;
    out->traj[l][2] = st.ph;
  }
}

// ---------------------------------------------------------------------------
// Robot-batched full tree (the run_math_model.py:231-280 episodes run side by
// side, one robot per episode, in lockstep: every robot's MPC step k uses the
// same quad window, so the per-control table is shared).  blockIdx.y = robot.

struct FtRobot {
  Consts K;
  double atan_t;
};

__global__ void k_ft_robots(const mpc_fulltree_problem_t* __restrict__ probs, int n,
                            double L, double t_a, double t_b, FtRobot* __restrict__ robots) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  mpc_problem_t q;
  q.x = probs[r].x;
  q.y = probs[r].y;
  q.phi = probs[r].phi;
  q.x_t = probs[r].x_t;
  q.y_t = probs[r].y_t;
  q.x_0 = probs[r].x_0;
  q.y_0 = probs[r].y_0;
  q.L = L;
  q.t_a = t_a;
  q.t_b = t_b;
  robots[r].K = consts_from_problem(q);
  robots[r].atan_t = probs[r].atan_target;
}

template <int INTEG, bool ROT>
__global__ __launch_bounds__(kBlock, kFtWaves) void k_ft_leaves_batched(
    const FtRobot* __restrict__ robots, const FtCtl* __restrict__ ctl,
    const uint32_t* __restrict__ no_rot, int64_t s1, Rec* __restrict__ part) {
  const int r = blockIdx.y;
  const Consts K = robots[r].K;
  const double atan_t = robots[r].atan_t;
  const int64_t n_items = ft_units(s1);
  uint64_t best_k = ~0ull;
  int64_t best_i = INT64_MAX;
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * kWaves +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n_waves = static_cast<int64_t>(gridDim.x) * kWaves;
  const FtCrit F = ft_crit(K, atan_t);
  if (ROT && *no_rot == 0u)
    ft_leaves_body<INTEG, true>(K, F, ctl, s1, 0, n_items, best_k, best_i, wave, n_waves);
  else
    ft_leaves_body<INTEG, false>(K, F, ctl, s1, 0, n_items, best_k, best_i, wave, n_waves);
  block_argmin(best_k, best_i);
  if (threadIdx.x == 0) part[static_cast<int64_t>(r) * gridDim.x + blockIdx.x] =
      Rec{best_k, best_i};
}

template <int INTEG, bool ROT>
__global__ __launch_bounds__(kBlock) void k_ft_finalize_batched(
    const Rec* __restrict__ part, int n_part, const FtRobot* __restrict__ robots,
    const FtCtl* __restrict__ ctl, const uint32_t* __restrict__ no_rot, int64_t s1,
    const double* __restrict__ incumbents, mpc_fulltree_result_t* __restrict__ outs) {
  const int r = blockIdx.x;
  uint64_t k = ~0ull;
  int64_t i = INT64_MAX;
  for (int p = threadIdx.x; p < n_part; p += kBlock) {
    const Rec rec = part[static_cast<int64_t>(r) * n_part + p];
    if (rec_less(rec.key, rec.idx, k, i)) {
      k = rec.key;
      i = rec.idx;
    }
  }
  block_argmin(k, i);
  if (threadIdx.x != 0) return;
  mpc_fulltree_result_t* out = outs + r;
  const Consts& K = robots[r].K;
  out->s1 = static_cast<int32_t>(s1);
  if (k == ~0ull) {
    out->cost = __builtin_inf();
    out->leaf = -1;
    out->found = 0;
    return;
  }
  const double c = key_cost(k);
  out->cost = c;
  out->leaf = i;
  out->found = c < (incumbents ? incumbents[r] : __builtin_inf()) ? 1 : 0;
  const int64_t kk[3] = {i / (s1 * s1), (i / s1) % s1, i % s1};
  const bool rot = ROT && *no_rot == 0u;
  FtState st{K.x, K.y, K.phi, K.s0, K.c0};
  for (int l = 0; l < 3; ++l) {
    const FtCtl u = ctl[kk[l]];
    st = rot ? ft_apply<INTEG, true>(st, u, K) : ft_apply<INTEG, false>(st, u, K);
    out->k[l] = kk[l];
    out->v[l] = u.v;
    out->beta[l] = u.beta;
    out->traj[l][0] = st.x;
    out->traj[l][1] = st.y;
    out->traj[l][2] = st.ph;
  }
}

}  // namespace mpc
