// mpc_device.h — device-side arithmetic of the MPC candidate expansion (gfx950).
//
// Every function here states one piece of ShittyWizard/DiplomJourney's
// math_model_tree.py in IEEE fp64 with the reference's operation order.  The
// translation unit is compiled with -ffp-contract=off so each + - * / is one
// rounding, exactly as in CPython; tan/sincos/sqrt are the ROCm device
// kernel's own fp64 routines (mpc_trig.h; faithfully rounded, <= 1 ulp from
// glibc's).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mpc_rollout.h"
#include "mpc_trig.h"

namespace mpc {

// Per-problem constants, derived once on the host (or per robot on device).
struct Consts {
  double x, y, phi;        // s0 = initial_coordinates (math_model_tree.py:294)
  double x_t, y_t;         // target globals (:65-66)
  double x_0, y_0;         // line origin globals (:57)
  double A, B, C1, C2;     // (y_t-y_0), (x_t-x_0), x_t*y_0, y_t*x_0   (:60)
  double inv_den;          // 1 / sqrt((y_t-y_0)**2 + (x_t-x_0)**2)    (:61): the line
                           // distance's division as a multiply (one rounding apart)
  double L, inv_L;         // wheelbase; 1/L when L is a power of two
  double h;                // (t+dt) - t, the quad interval length (RECT)
  double hlgth;            // 0.5*((t+dt) - t), QUADPACK's half length (QK21)
  double s0, c0;            // sin/cos of phi (heading-rotation mode)
  int32_t L_pow2;          // v/L == v*inv_L exactly
  int32_t pad_;
};

// QUADPACK dqk21 Kronrod weights wgk(1..11).
constexpr double kWGK[11] = {
    0.011694638867371874278064396062192, 0.032558162307964727478818972459390,
    0.054755896574351996031381300244580, 0.075039674810919952767043140916190,
    0.093125454583697605535065465083366, 0.109387158802297641899210590325805,
    0.123491976262065851077208698889469, 0.134709217311473325928054001771707,
    0.142775938577060080797094273138717, 0.147739104901338491374841515972068,
    0.149445554002916905664936468389821};

// sp.quad(f, t, t+dt) of a constant integrand (math_model_tree.py:91-96).
template <int INTEG>
MPC_HD __forceinline__ double quad_const(double f, const Consts& K) {
  if constexpr (INTEG == MPC_INTEG_RECT) {
    return f * K.h;
  } else {
    double resk = kWGK[10] * f;
    const double fsum = f + f;
#pragma unroll
    for (int j = 1; j <= 9; j += 2) resk = resk + kWGK[j] * fsum;
#pragma unroll
    for (int j = 0; j <= 8; j += 2) resk = resk + kWGK[j] * fsum;
    return resk * K.hlgth;
  }
}

// The three integrals of one step.  QK21: the reference's quad() (bitwise
// dqk21 on the constant integrand).  RECT: the same integrals of the constant
// integrands evaluated directly, h * f, with one rounding fewer per position
// update: dphi = ((v/L) * h) * tan(beta), x' = fma(v * h, cos phi', x).  (For
// L a power of two (v * inv_L) * h == (v * h) * inv_L exactly, so both forms of
// v/L give the same dphi.)
template <int INTEG>
MPC_HD __forceinline__ double heading_incr(double w, double t, const Consts& K) {
  if constexpr (INTEG == MPC_INTEG_RECT)
    return (w * K.h) * t;
  else
    return quad_const<INTEG>(w * t, K);
}

template <int INTEG>
MPC_HD __forceinline__ double position_step(double p, double v, double trig, const Consts& K) {
  if constexpr (INTEG == MPC_INTEG_RECT)
    return fma(v * K.h, trig, p);
  else
    return p + quad_const<INTEG>(v * trig, K);
}

// iteration_of_predict (math_model_tree.py:111-115): heading first, then
// position with the updated heading (semi-implicit bicycle step).
//
// step_core is the hot-loop form.  It uses the range-limited trig cores and
// flags the candidate `bad` when an argument leaves their range (|beta| >
// kTanMax; in direct mode |phi| > kFastMax; in rotation mode |dphi| > kRotMax;
// NaN).
// A bad candidate is recomputed with step_safe (direct sin/cos, library
// fallbacks), so every candidate gets a well-defined, correct result while the
// hot loop carries no fallback code.
//   ROT = false: sin/cos of the new heading evaluated directly (the reference's
//                formula, :113-114)
//   ROT = 1:     (s, c) carry sin/cos of the heading and are rotated by the
//                increment (mpc_trig.h rotation_factors / rotate_by)
//   ROT = 2:     (kRotCum) the same recurrence started from the identity
//                rotation (s, c) = (0, 1) and positions (x, y) = (0, 0): it
//                accumulates the pose-independent sums A = sum vh cos(Phi_k),
//                B = sum vh sin(Phi_k) of the heading increments Phi_k since
//                the start; cum_pose() turns them into the pose.  The work
//                per step is ROT = 1's; only the start state and the final
//                transform differ, and nothing before the transform needs the
//                start pose (the chained episode step, k_episode_chain).
//   PL2:         L is a power of two (v / L == v * inv_L exactly).  A template
//                parameter, not a branch: a branch inside the step would split
//                the loop into basic blocks and stop the scheduler from
//                interleaving the lane's independent candidate chains.
//   PL2 + RECT:  (v * inv_L) * h is formed as (v * h) * inv_L — the same
//                value (scaling by a power of two commutes with rounding in the
//                normal range) — so v * h is shared with the position update.
//                kRotCum goes one step further: v * (h * inv_L) serves both, the
//                sums A, B are accumulated scaled by 1/L (every rounding scales
//                exactly) and cum_pose<true> scales them back: the same bits
//                as the unscaled sums, one multiply fewer per step.
//   ld:          VGPR-resident leading coefficients (trig::Leads), or nullptr.
constexpr int kRotCum = 2;

template <int INTEG, int ROT, bool PL2>
MPC_HD __forceinline__ void step_core(double& x, double& y, double& ph, double& s, double& c,
                                      double v, double beta, const Consts& K, bool& bad,
                                      const trig::Leads* ld = nullptr) {
  bad |= !(fabs(beta) <= trig::kTanMax);
  const double t = trig::tan_small(beta, ld);
  double dphi, vh = 0.0;
  if constexpr (PL2 && INTEG == MPC_INTEG_RECT && ROT == kRotCum) {
    vh = v * (K.h * K.inv_L);                                  // the sums scaled by 1/L
    dphi = vh * t;                                             // angle_phi (:107)
  } else if constexpr (PL2 && INTEG == MPC_INTEG_RECT) {
    vh = v * K.h;
    dphi = (vh * K.inv_L) * t;                                 // angle_phi (:107)
  } else {
    const double w = PL2 ? v * K.inv_L : v / K.L;              // _velocity / L   (:78)
    dphi = heading_incr<INTEG>(w, t, K);                       // angle_phi (:107)
  }
  ph = ph + dphi;                                              // phi + _phi      (:113)
  if constexpr (ROT) {
    bad |= !(fabs(dphi) <= trig::kRotMax);
    double sd, cd;
    trig::rotation_sc(dphi, sd, cd, ld);
    trig::rotate_sc(sd, cd, s, c);
  } else {
    bad |= !(fabs(ph) <= trig::kFastMax);
    trig::sincos_core(ph, &s, &c);
  }
  if constexpr (PL2 && INTEG == MPC_INTEG_RECT) {
    x = fma(vh, c, x);                                         // coordinate_x    (:99)
    y = fma(vh, s, y);                                         // coordinate_y    (:103)
  } else {
    x = position_step<INTEG>(x, v, c, K);                      // coordinate_x    (:99)
    y = position_step<INTEG>(y, v, s, K);                      // coordinate_y    (:103)
  }
}

// Start state of the step recurrence: the pose (ROT 0 / 1) or the identity
// rotation and empty sums (kRotCum).
template <int ROT>
MPC_HD __forceinline__ void step_start(const Consts& K, double& x, double& y, double& ph,
                                       double& s, double& c) {
  ph = K.phi;
  if constexpr (ROT == kRotCum) {
    x = 0.0;
    y = 0.0;
    s = 0.0;
    c = 1.0;
  } else {
    x = K.x;
    y = K.y;
    s = K.s0;
    c = K.c0;
  }
}

// kRotCum: position from the sums, x = x0 + (c0 A - s0 B), y = y0 + (s0 A + c0 B).
// SCALED: the sums of step_core<RECT, kRotCum, PL2 = true>, i.e. A/L and B/L.
template <bool SCALED>
MPC_HD __forceinline__ void cum_pose(const Consts& K, double A, double B, double& x, double& y) {
  if constexpr (SCALED) {
    A = A * K.L;
    B = B * K.L;
  }
  x = K.x + fma(K.c0, A, -(K.s0 * B));
  y = K.y + fma(K.s0, A, K.c0 * B);
}

template <int INTEG>
MPC_HD __forceinline__ void step_safe(double& x, double& y, double& ph, double v, double beta,
                                      const Consts& K) {
  const double w = K.L_pow2 ? v * K.inv_L : v / K.L;
  const double dphi = heading_incr<INTEG>(w, trig::tan_fast(beta), K);
  ph = ph + dphi;
  double s, c;
  trig::sincos_fast(ph, &s, &c);
  x = position_step<INTEG>(x, v, c, K);
  y = position_step<INTEG>(y, v, s, K);
}

// IEEE sqrt for the criteria: on the device, the rsq + Newton sequence hipcc
// emits for sqrt(double) (correctly rounded: the same bits as sqrt) without
// its input scaling and special-case selects, 11 instead of 18 VALU.  Exact
// for 0 and for every input >= 2^-767; below that (a terminal
// state closer to the target than 1e-115) and for +inf / NaN it returns NaN,
// which never wins the strict < of an arg-min (+inf and NaN never do either).
MPC_HD __forceinline__ double crit_sqrt(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  // (the estimate of max(x, 2^-767): x itself in the exact range; for x = 0 a
  // finite estimate, so the sequence yields 0 exactly without a select; a NaN
  // x still propagates through the products)
  const double y = __builtin_amdgcn_rsq(fmax(x, 0x1p-767));
  double g = x * y, h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  return fma(d, h, g);
#else
  return sqrt(x);
#endif
}

// control_criterion (math_model_tree.py:82-87) on the layer-N state.
MPC_HD __forceinline__ double cost(double x, double y, const Consts& K) {
  const double ex = K.x_t - x, ey = K.y_t - y;
  const double dist_target = crit_sqrt(ex * ex + ey * ey);     // :66
  // :60-61, the division by the hypotenuse as a multiply by its reciprocal
  // (formed once per problem): <= 1 ulp from the quotient, and ~10 VALU
  // fewer per candidate than the IEEE division sequence.  Both sides of the
  // sentinel test are formed and one selected (no divergent branch).
  const double dl = fabs(K.A * x - K.B * y + K.C1 - K.C2) * K.inv_den;
  const double d = (x == K.x_0 && y == K.y_0) ? 1000.0 : dl;  // :57-58
  return 10000.0 * dist_target + 10000.0 * (d * d);            // :62, :87
}

// One candidate, exactly as the kernels evaluate it (the host replica in
// tests/replica_harness.cpp calls this): the core recurrence, and if that
// flags the candidate, the safe recurrence.  traj (optional) gets the
// per-step (x, y, phi).  Returns the cost.
template <int INTEG, int ROT, bool PL2>
MPC_HD inline double rollout_candidate_l(const Consts& K, const double* v, const double* b,
                                         int64_t ld, int64_t col, int n_steps, double* traj) {
  double x, y, ph, s, c;
  step_start<ROT>(K, x, y, ph, s, c);
  bool bad = false;
  for (int st = 0; st < n_steps; ++st) {
    step_core<INTEG, ROT, PL2>(x, y, ph, s, c, v[st * ld + col], b[st * ld + col], K, bad);
    if (traj) {
      if constexpr (ROT == kRotCum) {
        cum_pose<PL2>(K, x, y, traj[3 * st + 0], traj[3 * st + 1]);
      } else {
        traj[3 * st + 0] = x;
        traj[3 * st + 1] = y;
      }
      traj[3 * st + 2] = ph;
    }
  }
  if constexpr (ROT == kRotCum) {
    if (!bad) cum_pose<PL2>(K, x, y, x, y);
  }
  if (bad) {
    x = K.x;
    y = K.y;
    ph = K.phi;
    for (int st = 0; st < n_steps; ++st) {
      step_safe<INTEG>(x, y, ph, v[st * ld + col], b[st * ld + col], K);
      if (traj) {
        traj[3 * st + 0] = x;
        traj[3 * st + 1] = y;
        traj[3 * st + 2] = ph;
      }
    }
  }
  return cost(x, y, K);
}

template <int INTEG, int ROT>
MPC_HD inline double rollout_candidate(const Consts& K, const double* v, const double* b,
                                       int64_t ld, int64_t col, int n_steps, double* traj) {
  return K.L_pow2 ? rollout_candidate_l<INTEG, ROT, true>(K, v, b, ld, col, n_steps, traj)
                  : rollout_candidate_l<INTEG, ROT, false>(K, v, b, ld, col, n_steps, traj);
}

// Total order on costs for the arg-min: non-finite costs (NaN, +inf) map to
// the largest key and never win; -0 is folded into +0.
__device__ __forceinline__ uint64_t cost_key(double c) {
  if (!(c < __builtin_inf())) return ~0ull;
  c = c + 0.0;
  const uint64_t u = static_cast<uint64_t>(__double_as_longlong(c));
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// cost_key for a criterion value, which is never negative (a sum of
// 10000 * sqrt(.) and squares: +0 at least, or NaN / +inf): the same key
// without the sign fold — 2 VALU per candidate instead of ~6.
__device__ __forceinline__ uint64_t cost_key_nonneg(double c) {
  const uint64_t u = static_cast<uint64_t>(__double_as_longlong(c));
  return c < __builtin_inf() ? (u | 0x8000000000000000ull) : ~0ull;
}

__device__ __forceinline__ double key_cost(uint64_t k) {
  if (k == ~0ull) return __builtin_inf();
  const uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double(static_cast<long long>(u));
}

// Lexicographic (key, index) order: lowest cost, then lowest index — the
// first strict minimum of the reference's ascending scan (:351).
__device__ __forceinline__ bool rec_less(uint64_t ka, int64_t ia, uint64_t kb, int64_t ib) {
  return ka < kb || (ka == kb && ia < ib);
}

// One level of the wave reduction: every lane combines its (key, index) with
// the lane the DPP pattern CTRL names.  DPP moves run on the VALU: a level is
// a few cycles instead of an LDS round trip per 32-bit half (ds_bpermute).
// Lanes of rows outside RM receive an undefined value (no copy of the old
// one): the reduction below reads only lane 63, whose inputs are all defined.
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ void argmin_dpp_level(uint64_t& k, int64_t& i) {
  auto mv = [](uint64_t x) {
    const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(x), CTRL, RM, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(x >> 32), CTRL, RM, 0xf, true);
    return (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo);
  };
  const uint64_t ok = mv(k);
  const int64_t oi = static_cast<int64_t>(mv(static_cast<uint64_t>(i)));
  const bool lt = rec_less(ok, oi, k, i);
  k = lt ? ok : k;
  i = lt ? oi : i;
}

// Lexicographic (key, index) minimum over the 64 lanes of a wave (all lanes
// active), returned in every lane.  quad_perm [1,0,3,2] and [2,3,0,1], then
// row_half_mirror and row_mirror leave each row of 16 lanes holding its
// minimum in every lane; row_bcast:15 (into rows 1, 3: lane 31 then holds
// rows 0-1, lane 63 rows 2-3) and row_bcast:31 (lane 31 into row 3) fold the
// rows into lane 63, which is broadcast.  The minimum of a total order does
// not depend on the combination order: the same result as any other
// reduction tree.
__device__ __forceinline__ void wave_argmin(uint64_t& k, int64_t& i) {
  argmin_dpp_level<0xB1>(k, i);
  argmin_dpp_level<0x4E>(k, i);
  argmin_dpp_level<0x141>(k, i);
  argmin_dpp_level<0x140>(k, i);
  argmin_dpp_level<0x142, 0xA>(k, i);
  argmin_dpp_level<0x143, 0xC>(k, i);
  auto lane63 = [](uint64_t x) {
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<int>(x), 63);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<int>(x >> 32), 63);
    return (static_cast<uint64_t>(hi) << 32) | lo;
  };
  k = lane63(k);
  i = static_cast<int64_t>(lane63(static_cast<uint64_t>(i)));
}

// Minimum of a 32-bit value over the 64 lanes of a wave (all lanes active),
// returned in every lane: the DPP pattern of wave_argmin with v_min_u32
// (lanes a pattern does not feed get the identity 0xffffffff).
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
  auto lvl = [](uint32_t v, auto ctrl, auto rm) {
    constexpr int C = decltype(ctrl)::value, M = decltype(rm)::value;
    const uint32_t o = static_cast<uint32_t>(
        __builtin_amdgcn_update_dpp(-1, static_cast<int>(v), C, M, 0xf, false));
    return v < o ? v : o;
  };
  using std::integral_constant;
  x = lvl(x, integral_constant<int, 0xB1>{}, integral_constant<int, 0xf>{});
  x = lvl(x, integral_constant<int, 0x4E>{}, integral_constant<int, 0xf>{});
  x = lvl(x, integral_constant<int, 0x141>{}, integral_constant<int, 0xf>{});
  x = lvl(x, integral_constant<int, 0x140>{}, integral_constant<int, 0xf>{});
  x = lvl(x, integral_constant<int, 0x142>{}, integral_constant<int, 0xA>{});
  x = lvl(x, integral_constant<int, 0x143>{}, integral_constant<int, 0xC>{});
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), 63));
}

// wave_argmin for 31-bit indices (a lane without a candidate holds the
// sentinel (~0, INT64_MAX)): three 32-bit minima — the key's high word, its
// low word among the lanes holding that high word, the index among the lanes
// holding the whole key — give the same lexicographic minimum with ~40 VALU
// instead of ~70 (two 64-bit compares and four selects per level).
__device__ __forceinline__ void wave_argmin32(uint64_t& k, int64_t& i) {
  const uint32_t hi = static_cast<uint32_t>(k >> 32), lo = static_cast<uint32_t>(k);
  const uint32_t ix = k == ~0ull ? 0xffffffffu : static_cast<uint32_t>(i);
  const uint32_t m1 = wave_min_u32(hi);
  const uint32_t m2 = wave_min_u32(hi == m1 ? lo : 0xffffffffu);
  const uint32_t m3 = wave_min_u32(hi == m1 && lo == m2 ? ix : 0xffffffffu);
  k = (static_cast<uint64_t>(m1) << 32) | m2;
  i = k == ~0ull ? INT64_MAX : static_cast<int64_t>(m3);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace mpc
