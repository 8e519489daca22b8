// mpc_rollout.hip — C ABI (include/mpc_rollout.h) over the MI355X kernels of
// the MPC candidate expansion (ShittyWizard/DiplomJourney
// math_model_tree.py:278-362).  Kernels: mpc_kernels.h (rollout, arg-min,
// selection, sampler) and mpc_episode.h (device-resident episode).
//
// HBM traffic of k_rollout_argmin: 16 B per candidate-step read once
// (v, beta fp64 SoA), 16 B per block written.  See DESIGN.md for the roofline.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <type_traits>

#include "../../include/mpc_rollout.h"
#include "mpc_comm.h"
#include "mpc_episode.h"
#include "mpc_ftepisodes.h"
#include "mpc_episodes.h"
#include "mpc_fulltree.h"
#include "mpc_kernels.h"
#include "mpc_run.h"

namespace mpc {
namespace {

// libm through volatile pointers: the compiler must not fold pow(x, 2.0) into
// x*x (Python's `a ** 2` is libm pow, which is not always x*x).
double (*volatile g_libm_pow)(double, double) = pow;
double (*volatile g_libm_sin)(double) = sin;
double (*volatile g_libm_cos)(double) = cos;

// Problem constants derived on the host with the reference's libm calls.
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
  K.inv_den = 1.0 / sqrt(g_libm_pow(K.A, 2.0) + g_libm_pow(K.B, 2.0));
  K.L = p.L;
  int e;
  K.L_pow2 = (frexp(p.L, &e) == 0.5) ? 1 : 0;
  K.inv_L = K.L_pow2 ? 1.0 / p.L : 0.0;
  K.h = p.t_b - p.t_a;
  K.hlgth = 0.5 * (p.t_b - p.t_a);
  K.s0 = g_libm_sin(p.phi);
  K.c0 = g_libm_cos(p.phi);
  return K;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline int64_t rollout_blocks(int64_t n_cand) {
  // Upper bound on the rollout grid (the workspace is sized for it).
  return std::max<int64_t>(1, std::min<int64_t>(cdiv(n_cand, kBlock), kMaxBlocks));
}

int last_hip_status() { return hipGetLastError() == hipSuccess ? MPC_OK : MPC_ERR_HIP; }

// The LDS-DMA path addresses a control row as SGPR base + 32-bit lane byte
// offset (glds_pair): rows of leading dimension `ld` must stay below 2 GiB.
bool wide_ok(const double* v_sc, const double* beta_sc, int64_t n, int64_t ld = 0) {
  return (n % kCplWide == 0) && (ld > 0 ? ld : n) < (int64_t{1} << 28) && aligned16(v_sc) &&
         aligned16(beta_sc);
}

// Tile-strided grid: one block per tile of kBlock*CPL candidates, at most
// kMaxBlocks (blocks then stride over the tiles).
template <int CPL>
int64_t rollout_grid(int64_t n_cand) {
  return std::max<int64_t>(1, std::min<int64_t>(cdiv(n_cand, kBlock * CPL), kMaxBlocks));
}

template <int V>
using IC = std::integral_constant<int, V>;
template <bool V>
using BC = std::integral_constant<bool, V>;

// integrator = MPC_INTEG_* [| MPC_HEADING_ROTATE | MPC_HEADING_CUMULATIVE]
//   -> f(IC<INTEG>, IC<ROT>), ROT 0 direct heading, 1 rotation, 2 (kRotCum)
//   rotation from the identity with the pose applied last (rect only).
// allow_cum = false for the full-tree entry points (their own recurrence).
// allow_tiled: the entry accepts MPC_LAYOUT_TILED controls.
int mode_ok(int32_t integrator, bool allow_cum = true, bool allow_tiled = false) {
  if (integrator & ~(0xff | MPC_HEADING_ROTATE | MPC_HEADING_CUMULATIVE |
                     (allow_tiled ? MPC_LAYOUT_TILED : 0)))
    return MPC_ERR_UNSUPPORTED;
  const int integ = integrator & 0xff;
  if (integ != MPC_INTEG_QK21 && integ != MPC_INTEG_RECT) return MPC_ERR_UNSUPPORTED;
  if ((integrator & MPC_HEADING_CUMULATIVE) && (!allow_cum || integ != MPC_INTEG_RECT))
    return MPC_ERR_UNSUPPORTED;
  return MPC_OK;
}

inline bool is_cum(int32_t integrator) { return (integrator & MPC_HEADING_CUMULATIVE) != 0; }
inline bool is_tiled(int32_t integrator) { return (integrator & MPC_LAYOUT_TILED) != 0; }

// MPC_LAYOUT_TILED controls: v = the buffer's base (16-B aligned), beta =
// v + 512, n_cand even (two candidates per lane) and below 2^31.
bool tiled_ok(const double* v, const double* b, int64_t n_cand) {
  return v && b == v + MPC_TILE && (reinterpret_cast<uintptr_t>(v) & 15) == 0 &&
         n_cand >= 2 && n_cand % 2 == 0 && n_cand < (int64_t{1} << 31);
}

// The chained entries' control check: the aligned SoA path or the tiled layout.
bool chain_ctl_ok(const double* v, const double* b, int64_t n_cand, int32_t integrator) {
  return is_tiled(integrator) ? tiled_ok(v, b, n_cand) : wide_ok(v, b, n_cand);
}

// The bounded device waits count wall_clock64 ticks at kWallHz
// (mpc_episode.h).  A device whose constant-rate clock runs at another rate
// would scale every budget silently: the entries with such waits refuse it.
// Unknown (no device / the query fails): not refused here (the launch reports).
bool wall_clock_ok() {
  static int cache[16] = {0};   // 0 unknown, 1 kWallHz, -1 another rate
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return true;
  if (cache[dev] == 0) {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
      return true;
    cache[dev] = static_cast<uint64_t>(khz) * 1000ull == kWallHz ? 1 : -1;
  }
  return cache[dev] == 1;
}

template <class F>
void dispatch_mode(int32_t integrator, F&& f) {
  const bool rot = (integrator & MPC_HEADING_ROTATE) != 0;
  if ((integrator & 0xff) == MPC_INTEG_RECT) {
    if (is_cum(integrator)) f(IC<MPC_INTEG_RECT>{}, IC<kRotCum>{});
    else if (rot) f(IC<MPC_INTEG_RECT>{}, IC<1>{});
    else f(IC<MPC_INTEG_RECT>{}, IC<0>{});
  } else {
    if (rot) f(IC<MPC_INTEG_QK21>{}, IC<1>{});
    else f(IC<MPC_INTEG_QK21>{}, IC<0>{});
  }
}

// The full-tree kernels: direct or rotation heading only.
template <class F>
void dispatch_mode2(int32_t integrator, F&& f) {
  const bool rot = (integrator & MPC_HEADING_ROTATE) != 0;
  if ((integrator & 0xff) == MPC_INTEG_RECT) {
    if (rot) f(IC<MPC_INTEG_RECT>{}, BC<true>{});
    else f(IC<MPC_INTEG_RECT>{}, BC<false>{});
  } else {
    if (rot) f(IC<MPC_INTEG_QK21>{}, BC<true>{});
    else f(IC<MPC_INTEG_QK21>{}, BC<false>{});
  }
}

// Resident blocks of one fused episode instantiation (occupancy x CUs), cached
// per instantiation and device.  The fused launch is sized to ONE resident
// round: each block's end-of-launch hand-off (sc1 store + counter atomic) is
// then paid once per block, not once per tile round.
template <int CPL, int I, int R>
int64_t fused_grid(int64_t n_cand) {
  static int64_t cache[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (cache[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, reinterpret_cast<const void*>(&k_rollout_episode<CPL, I, R>), kBlock, 0) !=
            hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
      cus = 256;
    cache[dev] = std::min<int64_t>(static_cast<int64_t>(per_cu) * cus, kMaxBlocks);
  }
  return std::max<int64_t>(1, std::min(cdiv(n_cand, kBlock * CPL), cache[dev]));
}

// Tile blocks of one run launch: one resident round of the instantiation
// (occupancy x CUs; more would only queue behind it), at most one per unit.
template <bool P, bool T>
int64_t run_tile_blocks(int64_t units) {
  static int64_t cache[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (cache[dev] == 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, reinterpret_cast<const void*>(&k_episode_run<P, T>), kBlock, 0) !=
            hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
      cus = 256;
    // block 0 (the selector) takes one of the slots
    cache[dev] = std::max<int64_t>(1, static_cast<int64_t>(per_cu) * cus - 1);
  }
  return std::max<int64_t>(1, std::min(units, cache[dev]));
}

// Number of block records the rollout launch for these arguments writes
// (= its grid); the finalize launch reduces exactly these.
int64_t partial_count(const double* v_sc, const double* beta_sc, int64_t n_cand,
                      bool with_states) {
  const bool wide = !with_states && wide_ok(v_sc, beta_sc, n_cand);
  return wide ? rollout_grid<kCplWide>(n_cand) : rollout_grid<1>(n_cand);
}

// The streaming kernel: wide (CPL = kCplWide) or scalar path.
template <bool KDEV>
void launch_rollout(hipStream_t st, int32_t integrator, const Consts& K, const Consts* Kdev,
                    const double* v, const double* b, int64_t n_cand, int n_steps, Rec* part) {
  const bool wide = wide_ok(v, b, n_cand);
  dispatch_mode(integrator, [&](auto integ, auto rot) {
    constexpr int I = decltype(integ)::value;
    constexpr int R = decltype(rot)::value;
    if (wide)
      k_rollout_argmin_stream<I, R, KDEV><<<rollout_grid<kCplWide>(n_cand), kBlock, 0, st>>>(
          K, Kdev, v, b, n_cand, n_steps, part);
    else
      k_rollout_argmin<1, I, R, false, KDEV>
          <<<rollout_grid<1>(n_cand), kBlock, 0, st>>>(
              K, Kdev, v, b, n_cand, n_steps, part, nullptr);
  });
}

template <bool KDEV>
void launch_finalize(hipStream_t st, int32_t integrator, const Rec* part, int n_part,
                     const Consts& K, const Consts* Kdev, const double* v, const double* b,
                     int64_t n_cand, int n_steps, int64_t index_base, double incumbent,
                     const double* incumbent_dev, mpc_result_t* out,
                     const mpc_episode_config_t& ecfg, const EpisodeHook& hook) {
  dispatch_mode(integrator, [&](auto integ, auto rot) {
    constexpr int I = decltype(integ)::value;
    constexpr int R = decltype(rot)::value;
    if constexpr (KDEV && R == kRotCum) {
      if (is_tiled(integrator)) {   // the flush of a tiled chained episode
        k_finalize<I, R, KDEV, true><<<1, kFinBlock, 0, st>>>(
            part, n_part, K, Kdev, v, b, n_cand, n_steps, index_base, incumbent, incumbent_dev,
            out, ecfg, hook);
        return;
      }
    }
    k_finalize<I, R, KDEV><<<1, kFinBlock, 0, st>>>(part, n_part, K, Kdev, v, b, n_cand, n_steps,
                                                    index_base, incumbent, incumbent_dev, out,
                                                    ecfg, hook);
  });
}

int check_episode_cfg(const mpc_episode_config_t* c) {
  if (!c) return MPC_ERR_ARG;
  if (!(c->ratio_v >= 0) || !(c->ratio_beta >= 0) || c->ratio_v > 1000 || c->ratio_beta > 1000 ||
      c->max_steps < 0 || !(c->delta_t > 0) || (c->enumerate != 0 && c->enumerate != 1) ||
      (c->stop_rule != 0 && c->stop_rule != 1))
    return MPC_ERR_ARG;
  return MPC_OK;
}

}  // namespace
}  // namespace mpc

using namespace mpc;

extern "C" {

const char* mpc_version(void) { return "diplomjourney_amd mpc_rollout 0.2 (gfx950)"; }

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

static int check_args(const mpc_problem_t* p, const double* v_sc, const double* beta_sc,
                      int64_t n_cand, int32_t n_steps, int32_t integrator, void* ws,
                      size_t ws_bytes) {
  if (!p || n_cand < 1 || n_steps < 1 || n_steps > MPC_MAX_STEPS || !v_sc || !beta_sc)
    return MPC_ERR_ARG;
  if (mode_ok(integrator) != MPC_OK) return MPC_ERR_UNSUPPORTED;
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
  if (states_out) {
    // CoordinateTree materialisation path: one candidate per lane, all states out.
    dispatch_mode(integrator, [&](auto integ, auto rot) {
      constexpr int I = decltype(integ)::value;
      constexpr int R = decltype(rot)::value;
      k_rollout_argmin<1, I, R, true, false>
          <<<rollout_grid<1>(n_cand), kBlock, 0, st>>>(
              K, nullptr, v_sc, beta_sc, n_cand, n_steps, part, states_out);
    });
  } else {
    launch_rollout<false>(st, integrator, K, nullptr, v_sc, beta_sc, n_cand, n_steps, part);
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
  const Consts K = host_consts(*p);
  const int n_part = static_cast<int>(partial_count(v_sc, beta_sc, n_cand, with_states != 0));
  launch_finalize<false>(reinterpret_cast<hipStream_t>(stream), integrator,
                         static_cast<const Rec*>(ws), n_part, K, nullptr, v_sc, beta_sc, n_cand,
                         n_steps, index_base, incumbent, nullptr, out, mpc_episode_config_t{},
                         EpisodeHook{});
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
  if (mode_ok(integrator) != MPC_OK) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_batched_workspace_bytes(n_problems, cand_per_problem, n_steps))
    return MPC_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t ld = static_cast<int64_t>(n_problems) * cand_per_problem;
  const bool wide = wide_ok(v_sc, beta_sc, cand_per_problem, ld);
  const int64_t tiles = cdiv(cand_per_problem, kBlock * (wide ? kCplWide : 1));
  const int64_t per_robot = std::min<int64_t>(tiles, rollout_blocks(cand_per_problem));
  const dim3 grid(static_cast<unsigned>(per_robot), static_cast<unsigned>(n_problems));
  Rec* part = static_cast<Rec*>(ws);
  dispatch_mode(integrator, [&](auto integ, auto rot) {
    constexpr int I = decltype(integ)::value;
    constexpr int R = decltype(rot)::value;
    if (wide)
      k_rollout_argmin_batched<kCplWide, I, R>
          <<<grid, kBlock, 0, st>>>(problems, v_sc, beta_sc, cand_per_problem, n_steps, ld, part);
    else
      k_rollout_argmin_batched<1, I, R>
          <<<grid, kBlock, 0, st>>>(problems, v_sc, beta_sc, cand_per_problem, n_steps, ld, part);
  });
  if (last_hip_status() != MPC_OK) return MPC_ERR_HIP;
  dispatch_mode(integrator, [&](auto integ, auto rot) {
    constexpr int I = decltype(integ)::value;
    constexpr int R = decltype(rot)::value;
    k_finalize_batched<I, R><<<n_problems, kBlock, 0, st>>>(
        part, static_cast<int>(per_robot), problems, incumbents, v_sc, beta_sc, cand_per_problem,
        n_steps, ld, out);
  });
  return last_hip_status();
}

int mpc_stream_probe(const double* v_sc, const double* beta_sc, int64_t n_cand,
                     int32_t n_steps, void* sink, size_t sink_bytes, mpc_stream_t stream) {
  if (!v_sc || !beta_sc || n_cand < 2 || n_steps < 1 || n_steps > MPC_MAX_STEPS || !sink)
    return MPC_ERR_ARG;
  if (!wide_ok(v_sc, beta_sc, n_cand)) return MPC_ERR_UNSUPPORTED;
  const int64_t grid = rollout_grid<kCplWide>(n_cand);
  if (sink_bytes < static_cast<size_t>(kMaxBlocks) * kBlock * sizeof(uint64_t))
    return MPC_ERR_WORKSPACE;
  k_stream_probe<false><<<grid, kBlock, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      v_sc, beta_sc, n_cand, n_steps, static_cast<uint64_t*>(sink));
  return last_hip_status();
}

int mpc_stream_probe_tiled(const double* tiles, int64_t n_cand, int32_t n_steps, void* sink,
                           size_t sink_bytes, mpc_stream_t stream) {
  if (!tiles || n_steps < 1 || n_steps > MPC_MAX_STEPS || !sink) return MPC_ERR_ARG;
  if (!tiled_ok(tiles, tiles + MPC_TILE, n_cand)) return MPC_ERR_UNSUPPORTED;
  if (sink_bytes < static_cast<size_t>(kMaxBlocks) * kBlock * sizeof(uint64_t))
    return MPC_ERR_WORKSPACE;
  k_stream_probe<true><<<rollout_grid<kCplWide>(n_cand), kBlock, 0,
                         reinterpret_cast<hipStream_t>(stream)>>>(
      tiles, tiles + MPC_TILE, n_cand, n_steps, static_cast<uint64_t*>(sink));
  return last_hip_status();
}

__global__ void k_rcp_estimate(const double* __restrict__ q, double* __restrict__ r, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) r[i] = trig::rcp_estimate(q[i]);
}

int mpc_rcp_estimate(const double* q, double* r, int64_t n, mpc_stream_t stream) {
  if (n < 0 || (n > 0 && (!q || !r))) return MPC_ERR_ARG;
  if (n == 0) return MPC_OK;
  k_rcp_estimate<<<static_cast<unsigned>(cdiv(n, kBlock)), kBlock, 0,
                   reinterpret_cast<hipStream_t>(stream)>>>(q, r, n);
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
      beta_sc, ld, pairs, 0);
  return last_hip_status();
}

int mpc_sample_controls_tiled(const double* v_grid, int32_t n_v, const double* beta_grid,
                              int32_t n_beta, int64_t n_cand, int32_t n_steps, uint64_t seed,
                              int64_t index_base, int32_t const_prefix, double* tiles,
                              mpc_stream_t stream) {
  if (!v_grid || !beta_grid || !tiles || n_v < 1 || n_beta < 1 || n_steps < 1 ||
      n_steps > MPC_MAX_STEPS || index_base < 0)
    return MPC_ERR_ARG;
  if (static_cast<int64_t>(n_v) * n_beta > 0xFFFFFFFFll) return MPC_ERR_ARG;
  if (!tiled_ok(tiles, tiles + MPC_TILE, n_cand)) return MPC_ERR_ARG;
  // every slot of every tile, the last tile's padding included
  const int64_t n_pad = cdiv(n_cand, MPC_TILE) * MPC_TILE;
  const int64_t grid = std::min<int64_t>(cdiv(n_pad / 2, kBlock), 4096);
  k_sample_controls<<<grid, kBlock, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      v_grid, n_v, beta_grid, n_beta, n_pad, n_steps, seed, index_base, const_prefix, tiles,
      tiles + MPC_TILE, n_steps, 1, 1);
  return last_hip_status();
}

// ----------------------------- episode -------------------------------------
size_t mpc_episode_state_bytes(void) { return sizeof(EpisodeState); }

int mpc_episode_reset(const mpc_episode_config_t* cfg, void* state, mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK || !state) return MPC_ERR_ARG;
  k_episode_reset<<<1, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      *cfg, static_cast<EpisodeState*>(state));
  return last_hip_status();
}

static int check_episode_arrays(void* state, const double* v_sc, const double* beta_sc,
                                int64_t n_cand, int32_t n_steps) {
  if (!state || !v_sc || !beta_sc || n_cand < 1 || n_steps < 1 || n_steps > MPC_MAX_STEPS)
    return MPC_ERR_ARG;
  return MPC_OK;
}

int mpc_episode_sample(const mpc_episode_config_t* cfg, void* state, double* v_sc,
                       double* beta_sc, int64_t n_cand, int32_t n_steps, int64_t index_base,
                       mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK ||
      check_episode_arrays(state, v_sc, beta_sc, n_cand, n_steps) != MPC_OK || index_base < 0)
    return MPC_ERR_ARG;
  const int pairs = (n_cand % 2 == 0) && aligned16(v_sc) && aligned16(beta_sc);
  const int64_t items = pairs ? n_cand / 2 : n_cand;
  k_episode_sample<<<std::min<int64_t>(cdiv(items, kBlock), 4096), kBlock, 0,
                     reinterpret_cast<hipStream_t>(stream)>>>(
      *cfg, static_cast<EpisodeState*>(state), n_cand, n_steps, index_base, v_sc, beta_sc, pairs);
  return last_hip_status();
}

// Generated controls: the block records, then [grid][MPC_MAX_STEPS] v and beta
// of each block's best candidate.
static int64_t gen_grid(int64_t n_cand) { return rollout_grid<2>(n_cand); }
static size_t gen_ctl_offset(int64_t n_cand) {
  return (static_cast<size_t>(gen_grid(n_cand)) * sizeof(Rec) + 255) & ~static_cast<size_t>(255);
}

size_t mpc_episode_generate_workspace_bytes(int64_t n_cand, int32_t n_steps) {
  (void)n_steps;
  if (n_cand < 2) return 0;
  return gen_ctl_offset(n_cand) +
         2 * static_cast<size_t>(gen_grid(n_cand)) * MPC_MAX_STEPS * sizeof(double);
}

int mpc_episode_generate_step(const mpc_episode_config_t* cfg, void* state, int64_t n_cand,
                              int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                              size_t ws_bytes, mpc_result_t* out, mpc_episode_log_t* log,
                              int32_t log_capacity, mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK || !state || !out || n_steps < 1 ||
      n_steps > MPC_MAX_STEPS || index_base < 0 || log_capacity < 0)
    return MPC_ERR_ARG;
  if (n_cand < 2 || n_cand % 2 != 0) return MPC_ERR_ARG;   // two candidates per lane
  if (mode_ok(integrator) != MPC_OK || cfg->enumerate) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_episode_generate_workspace_bytes(n_cand, n_steps))
    return MPC_ERR_WORKSPACE;
  // the expanded grid in LDS: at most (1 + 2 ratio_v) x (1 + 2 ratio_beta) entries
  static_assert(kEpMaxGrid * kEpMaxGrid * sizeof(double2) <= 64 * 1024, "grid LDS bound");
  const int64_t nv = std::min<int64_t>(kEpMaxGrid, 1 + 2 * static_cast<int64_t>(cfg->ratio_v));
  const int64_t nb =
      std::min<int64_t>(kEpMaxGrid, 1 + 2 * static_cast<int64_t>(cfg->ratio_beta));
  const size_t lds = static_cast<size_t>(nv * nb) * sizeof(double2);
  EpisodeState* S = static_cast<EpisodeState*>(state);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  char* w = static_cast<char*>(ws);
  Rec* part = reinterpret_cast<Rec*>(w);
  const int64_t grid = gen_grid(n_cand);
  double* part_v = reinterpret_cast<double*>(w + gen_ctl_offset(n_cand));
  double* part_b = part_v + grid * MPC_MAX_STEPS;
  const EpisodeHook hook{&S->h, log, log_capacity, S->chain_pub, kPubWords};
  int e;
  const bool pl2 = frexp(cfg->L, &e) == 0.5;   // as consts_from_problem decides
  dispatch_mode(integrator, [&](auto integ, auto rot) {
    constexpr int I = decltype(integ)::value;
    constexpr int R = decltype(rot)::value;
    if (pl2)
      k_rollout_generated<I, R, true><<<grid, kBlock, lds, st>>>(*cfg, S, n_cand, n_steps,
                                                                 index_base, part, part_v, part_b);
    else
      k_rollout_generated<I, R, false><<<grid, kBlock, lds, st>>>(*cfg, S, n_cand, n_steps,
                                                                  index_base, part, part_v, part_b);
    k_finalize_gen<I, R><<<1, kFinBlock, 0, st>>>(part, static_cast<int>(grid), &S->h.K, part_v,
                                                  part_b, n_steps, index_base, &S->h.incumbent,
                                                  out, *cfg, hook);
  });
  return last_hip_status();
}

int mpc_episode_partials(void* state, const double* v_sc, const double* beta_sc, int64_t n_cand,
                         int32_t n_steps, int32_t integrator, void* ws, size_t ws_bytes,
                         mpc_stream_t stream) {
  if (check_episode_arrays(state, v_sc, beta_sc, n_cand, n_steps) != MPC_OK) return MPC_ERR_ARG;
  if (mode_ok(integrator) != MPC_OK) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  EpisodeState* S = static_cast<EpisodeState*>(state);
  launch_rollout<true>(reinterpret_cast<hipStream_t>(stream), integrator, Consts{}, &S->h.K, v_sc,
                       beta_sc, n_cand, n_steps, static_cast<Rec*>(ws));
  return last_hip_status();
}

int mpc_episode_finalize(void* state, const double* v_sc, const double* beta_sc, int64_t n_cand,
                         int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                         size_t ws_bytes, mpc_result_t* out, const mpc_episode_config_t* advance,
                         mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream) {
  if (check_episode_arrays(state, v_sc, beta_sc, n_cand, n_steps) != MPC_OK || !out ||
      index_base < 0)
    return MPC_ERR_ARG;
  if (mode_ok(integrator, true, true) != MPC_OK) return MPC_ERR_UNSUPPORTED;
  // tiled controls: the flush of a tiled chained episode (its records are the
  // chained launch's, one per tile)
  if (is_tiled(integrator) && (!is_cum(integrator) || !advance || !tiled_ok(v_sc, beta_sc, n_cand)))
    return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  if (advance && (check_episode_cfg(advance) != MPC_OK || log_capacity < 0)) return MPC_ERR_ARG;
  EpisodeState* S = static_cast<EpisodeState*>(state);
  const int n_part = static_cast<int>(is_tiled(integrator)
                                          ? rollout_grid<kCplWide>(n_cand)
                                          : partial_count(v_sc, beta_sc, n_cand, false));
  const mpc_episode_config_t ecfg = advance ? *advance : mpc_episode_config_t{};
  const EpisodeHook hook{advance ? &S->h : nullptr, log, log_capacity,
                         advance ? S->chain_pub : nullptr, advance ? kPubWords : 0};
  launch_finalize<true>(reinterpret_cast<hipStream_t>(stream), integrator,
                        static_cast<const Rec*>(ws), n_part, Consts{}, &S->h.K, v_sc, beta_sc,
                        n_cand, n_steps, index_base, 0.0, &S->h.incumbent, out, ecfg, hook);
  return last_hip_status();
}

int mpc_episode_step(void* state, const double* v_sc, const double* beta_sc, int64_t n_cand,
                     int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                     size_t ws_bytes, mpc_result_t* out, const mpc_episode_config_t* advance,
                     mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream) {
  const int a =
      mpc_episode_partials(state, v_sc, beta_sc, n_cand, n_steps, integrator, ws, ws_bytes, stream);
  if (a != MPC_OK) return a;
  return mpc_episode_finalize(state, v_sc, beta_sc, n_cand, n_steps, index_base, integrator, ws,
                              ws_bytes, out, advance, log, log_capacity, stream);
}

int mpc_episode_rollout(void* state, const double* v_sc, const double* beta_sc, int64_t n_cand,
                        int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                        size_t ws_bytes, mpc_result_t* out, const mpc_episode_config_t* advance,
                        mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream) {
  if (check_episode_arrays(state, v_sc, beta_sc, n_cand, n_steps) != MPC_OK || !out ||
      index_base < 0)
    return MPC_ERR_ARG;
  if (mode_ok(integrator) != MPC_OK) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  if (advance && (check_episode_cfg(advance) != MPC_OK || log_capacity < 0)) return MPC_ERR_ARG;
  EpisodeState* S = static_cast<EpisodeState*>(state);
  const mpc_episode_config_t ecfg = advance ? *advance : mpc_episode_config_t{};
  const EpisodeHook hook{advance ? &S->h : nullptr, log, log_capacity,
                         advance ? S->chain_pub : nullptr, advance ? kPubWords : 0};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool wide = wide_ok(v_sc, beta_sc, n_cand);
  dispatch_mode(integrator, [&](auto integ, auto rot) {
    constexpr int I = decltype(integ)::value;
    constexpr int R = decltype(rot)::value;
    if (wide)
      k_rollout_episode<kCplWide, I, R><<<fused_grid<kCplWide, I, R>(n_cand), kBlock, 0, st>>>(
          &S->h.K, v_sc, beta_sc, n_cand, n_steps, index_base, static_cast<Rec*>(ws), &S->done,
          &S->h.incumbent, out, ecfg, hook);
    else
      k_rollout_episode<1, I, R><<<fused_grid<1, I, R>(n_cand), kBlock, 0, st>>>(
          &S->h.K, v_sc, beta_sc, n_cand, n_steps, index_base, static_cast<Rec*>(ws), &S->done,
          &S->h.incumbent, out, ecfg, hook);
  });
  return last_hip_status();
}

int mpc_episode_chain_step(const mpc_episode_config_t* cfg, void* state, int32_t mode,
                           uint32_t epoch, const double* v_sc, const double* beta_sc,
                           int64_t n_cand,
                           int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                           const void* ws_prev, size_t ws_bytes, const double* v_prev,
                           const double* beta_prev, mpc_result_t* out_prev,
                           const mpc_result_t* gathered, int32_t n_gathered,
                           mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream) {
  (void)gathered;
  (void)n_gathered;
  if (check_episode_cfg(cfg) != MPC_OK ||
      check_episode_arrays(state, v_sc, beta_sc, n_cand, n_steps) != MPC_OK || index_base < 0 ||
      log_capacity < 0 || mode != MPC_CHAIN_FINALIZE || epoch == 0)
    return MPC_ERR_ARG;
  if (mode_ok(integrator, true, true) != MPC_OK || !is_cum(integrator) ||
      !chain_ctl_ok(v_sc, beta_sc, n_cand, integrator))
    return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  int has_prev = 0;
  if (v_prev) {
    if (!beta_prev || !out_prev || !ws_prev || !chain_ctl_ok(v_prev, beta_prev, n_cand, integrator))
      return MPC_ERR_ARG;
    has_prev = 1;
  }
  if (!wall_clock_ok()) return MPC_ERR_UNSUPPORTED;
  EpisodeState* S = static_cast<EpisodeState*>(state);
  int e;
  const int pl2 = frexp(cfg->L, &e) == 0.5 ? 1 : 0;   // as consts_from_problem decides
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  constexpr int I = MPC_INTEG_RECT;
  // block 0 + one block per tile; the previous step's records are as many
  // (same n_cand), and as many as mpc_episode_finalize reduces
  const int64_t tiles = rollout_grid<kCplWide>(n_cand);
  const int n_part_prev = static_cast<int>(tiles);
  auto launch = [&](auto pl2_tag, auto tiled_tag) {
    constexpr bool P = decltype(pl2_tag)::value;
    constexpr bool T = decltype(tiled_tag)::value;
    k_episode_chain<I, kRotCum, kChainFin, P, T><<<tiles + 1, kBlock, 0, st>>>(
        S, epoch, v_sc, beta_sc, n_cand, n_steps, static_cast<Rec*>(ws), has_prev,
        static_cast<const Rec*>(ws_prev), n_part_prev, v_prev, beta_prev, index_base, out_prev,
        nullptr, 0, *cfg, log, log_capacity, 0u);
  };
  const bool tl = is_tiled(integrator);
  if (pl2)
    tl ? launch(std::true_type{}, std::true_type{}) : launch(std::true_type{}, std::false_type{});
  else
    tl ? launch(std::false_type{}, std::true_type{}) : launch(std::false_type{}, std::false_type{});
  return last_hip_status();
}

#ifdef MPC_RUN_STATS
int mpc_debug_run_stats(unsigned long long* host, int reset) {
  if (reset) {
    unsigned long long init[kRunMaxSteps][8];
    for (int j = 0; j < kRunMaxSteps; ++j)
      for (int f = 0; f < 8; ++f) init[j][f] = (f == 3) ? ~0ull : 0ull;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_run_tl), init, sizeof(init)) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_run_tl), sizeof(g_run_tl)) == hipSuccess ? 0 : -1;
}
#endif

size_t mpc_episode_run_workspace_bytes(int64_t n_cand) {
  if (n_cand < 2) return 0;
  return run_workspace_bytes(cdiv(n_cand, kBlock * kCplWide));
}

int mpc_episode_run(const mpc_episode_config_t* cfg, void* state, uint32_t epoch0,
                    const double* const* v_steps, const double* const* beta_steps, int32_t n_run,
                    int64_t n_cand, int32_t n_steps, int64_t index_base, int32_t integrator,
                    void* ws, size_t ws_bytes, mpc_result_t* out, mpc_episode_log_t* log,
                    int32_t log_capacity, mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK || !state || n_steps < 1 || n_steps > MPC_MAX_STEPS ||
      n_cand < 2 || index_base < 0 || log_capacity < 0 || epoch0 == 0 || n_run < 1 ||
      !v_steps || !beta_steps || !out)
    return MPC_ERR_ARG;
  // the run's epochs are epoch0 .. epoch0 + n_run - 1, none of them 0
  if (static_cast<uint64_t>(epoch0) + static_cast<uint64_t>(n_run) - 1u > 0xFFFFFFFFull)
    return MPC_ERR_ARG;
  if (n_cand > 0x7fffffffll) return MPC_ERR_ARG;   // 32-bit local indices in the records
  if (mode_ok(integrator, true, true) != MPC_OK || !is_cum(integrator)) return MPC_ERR_UNSUPPORTED;
  for (int32_t j = 0; j < n_run; ++j)
    if (!v_steps[j] || !beta_steps[j] || !chain_ctl_ok(v_steps[j], beta_steps[j], n_cand, integrator))
      return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_episode_run_workspace_bytes(n_cand)) return MPC_ERR_WORKSPACE;
  if (!wall_clock_ok()) return MPC_ERR_UNSUPPORTED;
  EpisodeState* S = static_cast<EpisodeState*>(state);
  int e;
  const bool pl2 = frexp(cfg->L, &e) == 0.5;   // as consts_from_problem decides
  const bool tl = is_tiled(integrator);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t tiles = cdiv(n_cand, kBlock * kCplWide);
  for (int32_t j0 = 0; j0 < n_run; j0 += kRunMaxSteps) {
    const int k = std::min<int32_t>(kRunMaxSteps, n_run - j0);
    RunArgs ra;
    memset(&ra, 0, sizeof(ra));
    for (int j = 0; j < k; ++j) {
      ra.ctl.v[j] = v_steps[j0 + j];
      ra.ctl.b[j] = beta_steps[j0 + j];
    }
    ra.S = S;
    ra.ws = ws;
    ra.out = out;
    ra.log = log;
    ra.n_cand = n_cand;
    ra.index_base = index_base;
    ra.e0 = epoch0 + static_cast<uint32_t>(j0);
    ra.K = k;
    ra.n_steps = n_steps;
    ra.T = static_cast<int>(tiles);
    ra.cap = log_capacity;
    ra.ecfg = *cfg;
    auto launch = [&](auto pl2_tag, auto tiled_tag) {
      constexpr bool P = decltype(pl2_tag)::value;
      constexpr bool T = decltype(tiled_tag)::value;
      const int64_t grid = 1 + run_tile_blocks<P, T>(tiles * k);
      k_episode_run<P, T><<<grid, kBlock, 0, st>>>(ra);
    };
    if (pl2)
      tl ? launch(std::true_type{}, std::true_type{}) : launch(std::true_type{}, std::false_type{});
    else
      tl ? launch(std::false_type{}, std::true_type{}) : launch(std::false_type{}, std::false_type{});
    if (hipPeekAtLastError() != hipSuccess) break;
  }
  return last_hip_status();
}

int mpc_episode_exchange_step(const mpc_episode_config_t* cfg, void* state, uint32_t epoch,
                              const double* v_sc, const double* beta_sc, int64_t n_cand,
                              int32_t n_steps, int64_t index_base, int32_t integrator, void* ws,
                              size_t ws_bytes, const mpc_candidate_t* gathered,
                              int32_t n_gathered, mpc_result_t* out_prev, mpc_candidate_t* local,
                              mpc_episode_log_t* log, int32_t log_capacity, mpc_stream_t stream) {
  return mpc_episode_exchange_step2(cfg, state, epoch, 0u, v_sc, beta_sc, n_cand, n_steps,
                                    index_base, integrator, ws, ws_bytes, gathered, n_gathered,
                                    out_prev, local, log, log_capacity, stream);
}

int mpc_episode_exchange_step2(const mpc_episode_config_t* cfg, void* state, uint32_t epoch,
                               uint32_t wait_tag, const double* v_sc, const double* beta_sc,
                               int64_t n_cand, int32_t n_steps, int64_t index_base,
                               int32_t integrator, void* ws, size_t ws_bytes,
                               const mpc_candidate_t* gathered, int32_t n_gathered,
                               mpc_result_t* out_prev, mpc_candidate_t* local,
                               mpc_episode_log_t* log, int32_t log_capacity,
                               mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK ||
      check_episode_arrays(state, v_sc, beta_sc, n_cand, n_steps) != MPC_OK || index_base < 0 ||
      log_capacity < 0 || epoch == 0 || !local || !out_prev)
    return MPC_ERR_ARG;
  // local indices travel in the low 32 bits of a tagged record
  if (n_cand > 0x7fffffffll || (gathered && n_gathered < 1)) return MPC_ERR_ARG;
  // an overlapped step stages the gathered candidates in LDS
  if (wait_tag && (!gathered || n_gathered > kXchgLdsRanks)) return MPC_ERR_ARG;
  if (mode_ok(integrator) != MPC_OK || !is_cum(integrator) || !wide_ok(v_sc, beta_sc, n_cand))
    return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  if (!wall_clock_ok()) return MPC_ERR_UNSUPPORTED;
  EpisodeState* S = static_cast<EpisodeState*>(state);
  int e;
  const int pl2 = frexp(cfg->L, &e) == 0.5 ? 1 : 0;
  const int64_t grid = rollout_grid<kCplWide>(n_cand) + 1;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  constexpr int I = MPC_INTEG_RECT;
  auto launch = [&](auto pl2_tag) {
    constexpr bool P = decltype(pl2_tag)::value;
    k_episode_chain<I, kRotCum, kChainXchg, P><<<grid, kBlock, 0, st>>>(
        S, epoch, v_sc, beta_sc, n_cand, n_steps, static_cast<Rec*>(ws), gathered ? 1 : 0,
        reinterpret_cast<const Rec*>(local), 0, nullptr, nullptr, index_base, out_prev, gathered,
        n_gathered, *cfg, log, log_capacity, gathered ? wait_tag : 0u);
  };
  if (pl2)
    launch(std::true_type{});
  else
    launch(std::false_type{});
  return last_hip_status();
}

int mpc_stream_create_cu_reserved(int32_t reserved_per_xcd, mpc_stream_t* stream) {
  if (!stream || reserved_per_xcd < 0 || reserved_per_xcd > 8) return MPC_ERR_ARG;
  int dev = 0, ncu = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipGetDeviceProperties(&prop, dev) != hipSuccess)
    return MPC_ERR_HIP;
  // Logical CU i of a stream's CU mask sits on XCD i % 8: bits 0-7 are CU 0
  // of XCDs 0-7 (measured on an MI355X in SPX mode, tools/micro/cumask.hip),
  // so clearing the first 8 * r bits leaves r CUs of every XCD to other
  // streams.  That layout was measured on one part only: any other device
  // (another architecture, or a partition mode with fewer XCDs / CUs) is
  // refused rather than given a mask that reserves the wrong CUs.
  if (ncu != 256 || strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return MPC_ERR_UNSUPPORTED;
  uint32_t mask[16];
  const int words = (ncu + 31) / 32;
  if (words > 16) return MPC_ERR_UNSUPPORTED;
  for (int w = 0; w < words; ++w) mask[w] = 0xffffffffu;
  for (int b = 0; b < 8 * reserved_per_xcd; ++b) mask[b / 32] &= ~(1u << (b % 32));
  hipStream_t st = nullptr;
  if (hipExtStreamCreateWithCUMask(&st, static_cast<uint32_t>(words), mask) != hipSuccess)
    return MPC_ERR_HIP;
  *stream = reinterpret_cast<mpc_stream_t>(st);
  return MPC_OK;
}

int mpc_stream_create_cu_share(int32_t part, int32_t parts, mpc_stream_t* stream) {
  if (!stream || parts < 1 || parts > 32 || part < 0 || part >= parts) return MPC_ERR_ARG;
  int dev = 0, ncu = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipGetDeviceProperties(&prop, dev) != hipSuccess)
    return MPC_ERR_HIP;
  // the layout of mpc_stream_create_cu_reserved: logical CU b is CU b / 8 of
  // XCD b % 8, so CU j of every XCD goes to part j % parts
  if (ncu != 256 || strncmp(prop.gcnArchName, "gfx950", 6) != 0) return MPC_ERR_UNSUPPORTED;
  uint32_t mask[8] = {};
  for (int b = 0; b < ncu; ++b)
    if ((b / 8) % parts == part) mask[b / 32] |= 1u << (b % 32);
  hipStream_t st = nullptr;
  if (hipExtStreamCreateWithCUMask(&st, 8u, mask) != hipSuccess) return MPC_ERR_HIP;
  *stream = reinterpret_cast<mpc_stream_t>(st);
  return MPC_OK;
}

int mpc_stream_destroy(mpc_stream_t stream) {
  if (!stream) return MPC_ERR_ARG;
  return hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)) == hipSuccess ? MPC_OK
                                                                               : MPC_ERR_HIP;
}

int mpc_episode_exchange_mark(void* state, uint32_t tag, mpc_stream_t stream) {
  if (!state || tag == 0) return MPC_ERR_ARG;
  k_exchange_mark<<<1, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      static_cast<EpisodeState*>(state), tag);
  return last_hip_status();
}

int mpc_episode_exchange_flush(const mpc_episode_config_t* cfg, void* state, int32_t integrator,
                               const mpc_candidate_t* gathered, int32_t n_gathered,
                               mpc_result_t* out, mpc_episode_log_t* log, int32_t log_capacity,
                               mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK || !state || !gathered || n_gathered < 1 || !out ||
      log_capacity < 0)
    return MPC_ERR_ARG;
  if (mode_ok(integrator) != MPC_OK || !is_cum(integrator)) return MPC_ERR_UNSUPPORTED;
  k_episode_advance_cand<MPC_INTEG_RECT, kRotCum>
      <<<1, kFinBlock, 0, reinterpret_cast<hipStream_t>(stream)>>>(
          *cfg, static_cast<EpisodeState*>(state), gathered, n_gathered, out, log, log_capacity);
  return last_hip_status();
}

// ------------------------ peer-to-peer exchange ------------------------------
size_t mpc_mailbox_bytes(int32_t world) {
  return world < 1 || world > kMailMaxRanks ? 0 : mailbox_bytes(world);
}

int mpc_mailbox_alloc(int32_t world, int32_t uncached, void** mailbox) {
  const size_t n = mpc_mailbox_bytes(world);
  if (!n || !mailbox) return MPC_ERR_ARG;
  *mailbox = nullptr;
  void* p = nullptr;
  if ((uncached ? hipExtMallocWithFlags(&p, n, hipDeviceMallocUncached) : hipMalloc(&p, n)) !=
      hipSuccess)
    return MPC_ERR_HIP;
  // zeroed before the caller can hand it out: no peer ever sees a stale tag
  if (hipMemset(p, 0, n) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    return MPC_ERR_HIP;
  }
  *mailbox = p;
  return MPC_OK;
}

int mpc_mailbox_free(void* mailbox) {
  if (!mailbox) return MPC_ERR_ARG;
  return hipFree(mailbox) == hipSuccess ? MPC_OK : MPC_ERR_HIP;
}

int mpc_ipc_handle(void* dev_ptr, void* handle) {
  static_assert(sizeof(hipIpcMemHandle_t) == MPC_IPC_HANDLE_BYTES, "IPC handle size");
  if (!dev_ptr || !handle) return MPC_ERR_ARG;
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, dev_ptr) != hipSuccess) return MPC_ERR_HIP;
  memcpy(handle, &h, sizeof(h));
  return MPC_OK;
}

int mpc_ipc_open(const void* handle, void** dev_ptr) {
  if (!handle || !dev_ptr) return MPC_ERR_ARG;
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  *dev_ptr = nullptr;
  return hipIpcOpenMemHandle(dev_ptr, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess
             ? MPC_OK
             : MPC_ERR_HIP;
}

int mpc_ipc_close(void* dev_ptr) {
  if (!dev_ptr) return MPC_ERR_ARG;
  return hipIpcCloseMemHandle(dev_ptr) == hipSuccess ? MPC_OK : MPC_ERR_HIP;
}

int mpc_peer_enable(int32_t peer_device) {
  int dev = 0, n = 0, can = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceCount(&n) != hipSuccess) return MPC_ERR_HIP;
  if (peer_device < 0 || peer_device >= n) return MPC_ERR_ARG;
  if (peer_device == dev) return MPC_OK;
  if (hipDeviceCanAccessPeer(&can, dev, peer_device) != hipSuccess || !can)
    return MPC_ERR_UNSUPPORTED;
  const hipError_t e = hipDeviceEnablePeerAccess(peer_device, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
  return e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled ? MPC_OK : MPC_ERR_HIP;
}

int mpc_mailbox_set_peers(void* mailbox, int32_t rank, int32_t world, const void* const* peers) {
  if (!mailbox || !peers || world < 1 || world > kMailMaxRanks || rank < 0 || rank >= world)
    return MPC_ERR_ARG;
  MailHdr h = {};   // (ping words zeroed too: mpc_mailbox_ping before any peer pings)
  for (int r = 0; r < world; ++r) {
    if (!peers[r]) return MPC_ERR_ARG;
    h.peers[r] = reinterpret_cast<uint64_t>(peers[r]);
  }
  if (peers[rank] != mailbox) return MPC_ERR_ARG;   // own row: the local mapping
  h.rank = rank;
  h.world = world;
  return hipMemcpy(mailbox, &h, sizeof(h), hipMemcpyHostToDevice) == hipSuccess ? MPC_OK
                                                                                : MPC_ERR_HIP;
}

int mpc_mailbox_ping(void* mailbox, uint32_t tag, int32_t* ok, mpc_stream_t stream) {
  if (!mailbox || !ok || tag == 0) return MPC_ERR_ARG;
  if (!wall_clock_ok()) return MPC_ERR_UNSUPPORTED;
  k_mailbox_ping<<<1, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(mailbox, tag, ok);
  return last_hip_status();
}

int mpc_mailbox_clear(void* mailbox, int32_t world, mpc_stream_t stream) {
  if (!mailbox || world < 1 || world > kMailMaxRanks) return MPC_ERR_ARG;
  return hipMemsetAsync(static_cast<char*>(mailbox) + kMailHdrBytes, 0,
                        mailbox_bytes(world) - kMailHdrBytes,
                        reinterpret_cast<hipStream_t>(stream)) == hipSuccess
             ? MPC_OK
             : MPC_ERR_HIP;
}

int mpc_episode_p2p_step(const mpc_episode_config_t* cfg, void* state, uint32_t epoch,
                         uint32_t prev_epoch, const double* v_sc, const double* beta_sc,
                         int64_t n_cand, int32_t n_steps, int64_t index_base, int32_t integrator,
                         void* ws, const void* ws_prev, size_t ws_bytes, const double* v_prev,
                         const double* beta_prev, void* mailbox, int32_t world,
                         mpc_result_t* out_prev, mpc_episode_log_t* log, int32_t log_capacity,
                         mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK ||
      check_episode_arrays(state, v_sc, beta_sc, n_cand, n_steps) != MPC_OK || index_base < 0 ||
      log_capacity < 0 || epoch == 0 || !mailbox || world < 1 || world > kMailMaxRanks)
    return MPC_ERR_ARG;
  if (prev_epoch) {
    // consecutive steps use the two mailbox slots alternately (epoch & 1)
    if (((epoch ^ prev_epoch) & 1u) == 0 || !out_prev || !ws_prev || !v_prev || !beta_prev)
      return MPC_ERR_ARG;
  }
  if (mode_ok(integrator, true, true) != MPC_OK || !is_cum(integrator) ||
      !chain_ctl_ok(v_sc, beta_sc, n_cand, integrator) ||
      (prev_epoch && !chain_ctl_ok(v_prev, beta_prev, n_cand, integrator)))
    return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  if (!wall_clock_ok()) return MPC_ERR_UNSUPPORTED;
  EpisodeState* S = static_cast<EpisodeState*>(state);
  int e;
  const int pl2 = frexp(cfg->L, &e) == 0.5 ? 1 : 0;
  // block 0 + one block per tile; the previous step's records are as many
  const int64_t tiles = rollout_grid<kCplWide>(n_cand);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  constexpr int I = MPC_INTEG_RECT;
  // (the exchange form's argument slots: gathered = this rank's mailbox,
  // n_gathered = world, wait_tag = the previous step's epoch)
  auto launch = [&](auto pl2_tag, auto tiled_tag) {
    constexpr bool P = decltype(pl2_tag)::value;
    constexpr bool T = decltype(tiled_tag)::value;
    k_episode_chain<I, kRotCum, kChainP2P, P, T><<<tiles + 1, kBlock, 0, st>>>(
        S, epoch, v_sc, beta_sc, n_cand, n_steps, static_cast<Rec*>(ws), prev_epoch ? 1 : 0,
        static_cast<const Rec*>(ws_prev), static_cast<int>(tiles), v_prev, beta_prev,
        index_base, out_prev, static_cast<const mpc_candidate_t*>(mailbox), world, *cfg, log,
        log_capacity, prev_epoch);
  };
  const bool tl = is_tiled(integrator);
  if (pl2)
    tl ? launch(std::true_type{}, std::true_type{}) : launch(std::true_type{}, std::false_type{});
  else
    tl ? launch(std::false_type{}, std::true_type{}) : launch(std::false_type{}, std::false_type{});
  return last_hip_status();
}

int mpc_episode_p2p_flush(const mpc_episode_config_t* cfg, void* state, uint32_t last_epoch,
                          const double* v_last, const double* beta_last, int64_t n_cand,
                          int32_t n_steps, int64_t index_base, int32_t integrator,
                          const void* ws_last, size_t ws_bytes, void* mailbox, int32_t world,
                          mpc_result_t* out, mpc_episode_log_t* log, int32_t log_capacity,
                          mpc_stream_t stream) {
  if (check_episode_cfg(cfg) != MPC_OK ||
      check_episode_arrays(state, v_last, beta_last, n_cand, n_steps) != MPC_OK ||
      index_base < 0 || !mailbox || last_epoch == 0 || world < 1 || world > kMailMaxRanks ||
      !out || log_capacity < 0 || !ws_last)
    return MPC_ERR_ARG;
  if (mode_ok(integrator, true, true) != MPC_OK || !is_cum(integrator) ||
      !chain_ctl_ok(v_last, beta_last, n_cand, integrator))
    return MPC_ERR_UNSUPPORTED;
  if (ws_bytes < mpc_workspace_bytes(n_cand, n_steps)) return MPC_ERR_WORKSPACE;
  if (!wall_clock_ok()) return MPC_ERR_UNSUPPORTED;
  auto launch = [&](auto tiled_tag) {
    constexpr bool T = decltype(tiled_tag)::value;
    k_episode_p2p_flush<MPC_INTEG_RECT, kRotCum, T>
        <<<1, kBlock, 0, reinterpret_cast<hipStream_t>(stream)>>>(
            *cfg, static_cast<EpisodeState*>(state), mailbox, last_epoch, world,
            static_cast<const Rec*>(ws_last), static_cast<int>(rollout_grid<kCplWide>(n_cand)),
            v_last, beta_last, n_cand, n_steps, index_base, out, log, log_capacity);
  };
  if (is_tiled(integrator))
    launch(std::true_type{});
  else
    launch(std::false_type{});
  return last_hip_status();
}

// ----------------------------- RCCL exchange --------------------------------
int mpc_comm_unique_id(void* id) {
  const rccl::Api& r = rccl::api();
  if (!id) return MPC_ERR_ARG;
  if (!r.ok) return MPC_ERR_UNSUPPORTED;
  rccl::UniqueId u;
  if (r.get_unique_id(&u) != rccl::kSuccess) return MPC_ERR_HIP;
  memcpy(id, &u, sizeof(u));
  return MPC_OK;
}

int mpc_comm_init_rank(const void* id, int32_t n_ranks, int32_t rank, mpc_comm_t* comm) {
  const rccl::Api& r = rccl::api();
  if (!id || !comm || n_ranks < 1 || rank < 0 || rank >= n_ranks) return MPC_ERR_ARG;
  if (!r.ok) return MPC_ERR_UNSUPPORTED;
  rccl::UniqueId u;
  memcpy(&u, id, sizeof(u));
  rccl::Comm c = nullptr;
  if (r.comm_init_rank(&c, n_ranks, u, rank) != rccl::kSuccess) return MPC_ERR_HIP;
  *comm = reinterpret_cast<mpc_comm_t>(c);
  return MPC_OK;
}

int mpc_comm_init_all(int32_t n_devices, const int32_t* devices, mpc_comm_t* comms) {
  const rccl::Api& r = rccl::api();
  if (n_devices < 1 || !comms) return MPC_ERR_ARG;
  if (!r.ok) return MPC_ERR_UNSUPPORTED;
  rccl::Comm* c = reinterpret_cast<rccl::Comm*>(comms);
  return r.comm_init_all(c, n_devices, devices) == rccl::kSuccess ? MPC_OK : MPC_ERR_HIP;
}

int mpc_comm_destroy(mpc_comm_t comm) {
  const rccl::Api& r = rccl::api();
  if (!comm) return MPC_ERR_ARG;
  if (!r.ok) return MPC_ERR_UNSUPPORTED;
  return r.comm_destroy(reinterpret_cast<rccl::Comm>(comm)) == rccl::kSuccess ? MPC_OK
                                                                              : MPC_ERR_HIP;
}

int mpc_exchange_allgather(mpc_comm_t comm, const mpc_candidate_t* local,
                           mpc_candidate_t* gathered, mpc_stream_t stream) {
  const rccl::Api& r = rccl::api();
  if (!comm || !local || !gathered) return MPC_ERR_ARG;
  if (!r.ok) return MPC_ERR_UNSUPPORTED;
  return r.all_gather(local, gathered, sizeof(mpc_candidate_t), rccl::kUint8,
                      reinterpret_cast<rccl::Comm>(comm),
                      reinterpret_cast<hipStream_t>(stream)) == rccl::kSuccess
             ? MPC_OK
             : MPC_ERR_HIP;
}

int mpc_exchange_allgather_group(int32_t n, const mpc_comm_t* comms,
                                 const mpc_candidate_t* const* local,
                                 mpc_candidate_t* const* gathered, const mpc_stream_t* streams) {
  const rccl::Api& r = rccl::api();
  if (n < 1 || !comms || !local || !gathered || !streams) return MPC_ERR_ARG;
  if (!r.ok) return MPC_ERR_UNSUPPORTED;
  if (r.group_start() != rccl::kSuccess) return MPC_ERR_HIP;
  int st = MPC_OK;
  for (int i = 0; i < n; ++i)
    if (r.all_gather(local[i], gathered[i], sizeof(mpc_candidate_t), rccl::kUint8,
                     reinterpret_cast<rccl::Comm>(comms[i]),
                     reinterpret_cast<hipStream_t>(streams[i])) != rccl::kSuccess)
      st = MPC_ERR_HIP;
  if (r.group_end() != rccl::kSuccess) st = MPC_ERR_HIP;
  return st;
}

// One word device -> coherent pinned host memory by a one-lane kernel (a
// vector store over the fabric), not by an async memory copy: a 4-B
// hipMemcpyAsync to pageable memory on a CU-masked stream (the overlapped
// exchange's launch stream) left its completion callback undelivered at
// process exit under rocprofv3's memory-copy tracing (profiles/r06/overlap_exit/).
__global__ void k_read_word(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst) {
  if (threadIdx.x == 0) *dst = *src;
}

int mpc_episode_chain_error(const void* state, int32_t* error, mpc_stream_t stream) {
  if (!state || !error) return MPC_ERR_ARG;
  static std::mutex mu;
  static uint32_t* host = nullptr;   // process lifetime
  std::lock_guard<std::mutex> lock(mu);
  if (!host && hipHostMalloc(reinterpret_cast<void**>(&host), 256, hipHostMallocCoherent) !=
                   hipSuccess) {
    host = nullptr;
    return MPC_ERR_HIP;
  }
  *reinterpret_cast<volatile uint32_t*>(host) = ~0u;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  k_read_word<<<1, 64, 0, st>>>(&static_cast<const EpisodeState*>(state)->chain_error, host);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
    return MPC_ERR_HIP;
  *error = static_cast<int32_t>(*reinterpret_cast<volatile uint32_t*>(host));
  return MPC_OK;
}

int mpc_episode_expand(const mpc_episode_config_t* cfg, void* state, double* v_sc,
                       double* beta_sc, int64_t n_cand, int32_t n_steps, int64_t index_base,
                       int32_t integrator, void* ws, size_t ws_bytes, mpc_result_t* out,
                       mpc_stream_t stream) {
  if (!out) return MPC_ERR_ARG;
  const int a =
      mpc_episode_sample(cfg, state, v_sc, beta_sc, n_cand, n_steps, index_base, stream);
  if (a != MPC_OK) return a;
  return mpc_episode_rollout(state, v_sc, beta_sc, n_cand, n_steps, index_base, integrator, ws,
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

// ----------------------------- batched episodes ----------------------------
size_t mpc_episodes_state_bytes(int32_t n_robots) {
  if (n_robots < 1) return 0;
  return episodes_cfg_offset(n_robots) + static_cast<size_t>(n_robots) * sizeof(mpc_episode_config_t);
}

int mpc_episodes_reset(const mpc_episode_config_t* cfgs, int32_t n_robots, void* state,
                       mpc_stream_t stream) {
  if (!cfgs || !state || n_robots < 1 || n_robots > 65535) return MPC_ERR_ARG;
  for (int32_t r = 0; r < n_robots; ++r)
    if (check_episode_cfg(&cfgs[r]) != MPC_OK) return MPC_ERR_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  char* s = static_cast<char*>(state);
  mpc_episode_config_t* dcfg = reinterpret_cast<mpc_episode_config_t*>(s + episodes_cfg_offset(n_robots));
  // (pageable host source: the copy has read it when the call returns)
  if (hipMemcpyAsync(dcfg, cfgs, static_cast<size_t>(n_robots) * sizeof(mpc_episode_config_t),
                     hipMemcpyHostToDevice, st) != hipSuccess)
    return MPC_ERR_HIP;
  k_episodes_reset<<<static_cast<unsigned>(cdiv(n_robots, 256)), 256, 0, st>>>(
      dcfg, n_robots, reinterpret_cast<RobotState*>(s));
  return last_hip_status();
}

int mpc_episodes_run(void* state, int32_t n_robots, int32_t n_steps, int32_t integrator,
                     int32_t max_calls, mpc_episode_log_t* log, int32_t log_capacity,
                     mpc_episodes_progress_t* progress, mpc_stream_t stream) {
  if (!state || n_robots < 1 || n_robots > 65535 || n_steps < 1 || n_steps > MPC_MAX_STEPS ||
      max_calls < 0 || log_capacity < 0 || (log && log_capacity < 1))
    return MPC_ERR_ARG;
  if (mode_ok(integrator) != MPC_OK) return MPC_ERR_UNSUPPORTED;
  if (max_calls == 0) return MPC_OK;
  char* s = static_cast<char*>(state);
  const mpc_episode_config_t* dcfg =
      reinterpret_cast<const mpc_episode_config_t*>(s + episodes_cfg_offset(n_robots));
#ifndef MPC_EP_VARIANT
#define MPC_EP_VARIANT 2
#endif
  // 0: one 256-thread block per robot, a lane's two candidates in turn;
  // 1: one wave per robot, its candidates two at a time (while the winner's
  //    trajectory fits one value per lane: emit_winner's store);
  // 2: one 256-thread block per robot, a lane's two candidates interleaved
  const int variant = (MPC_EP_VARIANT == 1 && 3 * n_steps > 64) ? 2 : MPC_EP_VARIANT;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  RobotState* robots = reinterpret_cast<RobotState*>(s);
  const int cap = log ? log_capacity : 0;
  dispatch_mode(integrator, [&](auto integ, auto rot) {
    constexpr int I = decltype(integ)::value;
    constexpr int R = decltype(rot)::value;
    if (variant == 1)
      k_episodes_run<I, R, 64, true><<<n_robots, 64, 0, st>>>(dcfg, robots, n_steps, max_calls,
                                                               log, cap, progress);
    else if (variant == 2)
      k_episodes_run<I, R, kBlock, true><<<n_robots, kBlock, 0, st>>>(
          dcfg, robots, n_steps, max_calls, log, cap, progress);
    else
      k_episodes_run<I, R, kBlock, false><<<n_robots, kBlock, 0, st>>>(
          dcfg, robots, n_steps, max_calls, log, cap, progress);
  });
  return last_hip_status();
}

// ----------------------------- full tree -----------------------------------
static size_t ft_align(size_t n) { return (n + 255) & ~static_cast<size_t>(255); }
static constexpr int64_t kFtMaxBlocks = 2048;
static constexpr int64_t kFtMinShare = 32;   // work units per wave at least (small trees)

// The current device's CU count (cached per device).
static int64_t device_cus() {
  static int64_t cache[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (cache[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
      cus = 256;
    cache[dev] = cus;
  }
  return cache[dev];
}

size_t mpc_fulltree_workspace_bytes(int32_t n_v, int32_t n_beta) {
  if (n_v < 1 || n_beta < 1) return 0;
  const size_t s1 = static_cast<size_t>(n_v) * static_cast<size_t>(n_beta);
  return ft_align(s1 * sizeof(FtCtl)) + 256 + kFtMaxBlocks * sizeof(Rec);
}

int mpc_fulltree_argmin(const mpc_fulltree_problem_t* p, const double* v_grid, int32_t n_v,
                        const double* beta_grid, int32_t n_beta, double incumbent,
                        int32_t integrator, int32_t shard, int32_t n_shards, void* ws,
                        size_t ws_bytes, mpc_fulltree_result_t* out, mpc_stream_t stream) {
  if (!p || !v_grid || !beta_grid || !out || n_v < 1 || n_beta < 1) return MPC_ERR_ARG;
  if (n_shards < 1 || shard < 0 || shard >= n_shards) return MPC_ERR_ARG;
  const int64_t s1 = static_cast<int64_t>(n_v) * n_beta;
  if (s1 > 2000000) return MPC_ERR_ARG;  // S1^3 must fit int64 leaf indices
  if (mode_ok(integrator, false) != MPC_OK) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_fulltree_workspace_bytes(n_v, n_beta)) return MPC_ERR_WORKSPACE;
  mpc_problem_t q;
  q.x = p->x;
  q.y = p->y;
  q.phi = p->phi;
  q.x_t = p->x_t;
  q.y_t = p->y_t;
  q.x_0 = p->x_0;
  q.y_0 = p->y_0;
  q.L = p->L;
  q.t_a = p->t_a;
  q.t_b = p->t_b;
  const Consts K = host_consts(q);
  char* w = static_cast<char*>(ws);
  FtCtl* ctl = reinterpret_cast<FtCtl*>(w);
  uint32_t* no_rot = reinterpret_cast<uint32_t*>(w + ft_align(s1 * sizeof(FtCtl)));
  Rec* part = reinterpret_cast<Rec*>(w + ft_align(s1 * sizeof(FtCtl)) + 256);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(no_rot, 0, sizeof(uint32_t), st) != hipSuccess) return MPC_ERR_HIP;
  // the shard's contiguous range of work units (ft_units), shared out evenly
  // over a grid of kFtWaves blocks per CU (one wave per SIMD each: every SIMD
  // holds the same number of equal shares), fewer for a small tree
  const int64_t n_units = ft_units(s1);
  const int64_t base = n_units / n_shards, rem = n_units % n_shards;
  const int64_t u_lo = shard * base + std::min<int64_t>(shard, rem);
  const int64_t u_hi = u_lo + base + (shard < rem ? 1 : 0);
  const int64_t grid = std::max<int64_t>(
      1, std::min({cdiv(u_hi - u_lo, kWaves * kFtMinShare), device_cus() * kFtWaves,
                   kFtMaxBlocks}));
  dispatch_mode2(integrator, [&](auto integ, auto rot) {
    constexpr int I = decltype(integ)::value;
    constexpr bool R = decltype(rot)::value;
    k_ft_controls<I><<<cdiv(s1, kBlock), kBlock, 0, st>>>(K, v_grid, beta_grid, n_beta, s1, ctl,
                                                          no_rot);
    k_ft_leaves<I, R><<<grid, kBlock, 0, st>>>(K, p->atan_target, ctl, no_rot, s1, u_lo, u_hi,
                                                part);
    k_ft_finalize<I, R><<<1, kFinBlock, 0, st>>>(part, static_cast<int>(grid), K, ctl, no_rot,
                                                 s1, incumbent, out);
  });
  return last_hip_status();
}

static int64_t ft_blocks_per_robot(int64_t s1, int32_t n) {
  // about 4096 blocks in total, at least one per robot
  const int64_t want = std::max<int64_t>(1, 4096 / std::max<int32_t>(n, 1));
  return std::max<int64_t>(1, std::min(cdiv(ft_units(s1), kWaves * kFtMinShare), want));
}

size_t mpc_fulltree_batched_workspace_bytes(int32_t n_problems, int32_t n_v, int32_t n_beta) {
  if (n_problems < 1 || n_v < 1 || n_beta < 1) return 0;
  const int64_t s1 = static_cast<int64_t>(n_v) * n_beta;
  return ft_align(s1 * sizeof(FtCtl)) + 256 + ft_align(n_problems * sizeof(FtRobot)) +
         static_cast<size_t>(n_problems) * ft_blocks_per_robot(s1, n_problems) * sizeof(Rec);
}

int mpc_fulltree_argmin_batched(const mpc_fulltree_problem_t* problems,
                                const double* incumbents, int32_t n_problems, double L,
                                double t_a, double t_b, const double* v_grid, int32_t n_v,
                                const double* beta_grid, int32_t n_beta, int32_t integrator,
                                void* ws, size_t ws_bytes, mpc_fulltree_result_t* out,
                                mpc_stream_t stream) {
  if (!problems || !out || !v_grid || !beta_grid || n_problems < 1 || n_v < 1 || n_beta < 1 ||
      n_problems > 65535)
    return MPC_ERR_ARG;
  const int64_t s1 = static_cast<int64_t>(n_v) * n_beta;
  if (s1 > 2000000) return MPC_ERR_ARG;
  if (mode_ok(integrator, false) != MPC_OK) return MPC_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < mpc_fulltree_batched_workspace_bytes(n_problems, n_v, n_beta))
    return MPC_ERR_WORKSPACE;
  mpc_problem_t q = {};
  q.x_t = 1.0;   // window-only constants for the shared control table
  q.y_t = 1.0;
  q.L = L;
  q.t_a = t_a;
  q.t_b = t_b;
  const Consts Kw = host_consts(q);
  char* w = static_cast<char*>(ws);
  FtCtl* ctl = reinterpret_cast<FtCtl*>(w);
  uint32_t* no_rot = reinterpret_cast<uint32_t*>(w + ft_align(s1 * sizeof(FtCtl)));
  FtRobot* robots = reinterpret_cast<FtRobot*>(w + ft_align(s1 * sizeof(FtCtl)) + 256);
  Rec* part = reinterpret_cast<Rec*>(w + ft_align(s1 * sizeof(FtCtl)) + 256 +
                                     ft_align(n_problems * sizeof(FtRobot)));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(no_rot, 0, sizeof(uint32_t), st) != hipSuccess) return MPC_ERR_HIP;
  const int64_t bx = ft_blocks_per_robot(s1, n_problems);
  k_ft_robots<<<cdiv(n_problems, 256), 256, 0, st>>>(problems, n_problems, L, t_a, t_b, robots);
  dispatch_mode2(integrator, [&](auto integ, auto rot) {
    constexpr int I = decltype(integ)::value;
    constexpr bool R = decltype(rot)::value;
    k_ft_controls<I><<<cdiv(s1, kBlock), kBlock, 0, st>>>(Kw, v_grid, beta_grid, n_beta, s1,
                                                          ctl, no_rot);
    k_ft_leaves_batched<I, R><<<dim3(static_cast<unsigned>(bx), n_problems), kBlock, 0, st>>>(
        robots, ctl, no_rot, s1, part);
    k_ft_finalize_batched<I, R><<<n_problems, kBlock, 0, st>>>(
        part, static_cast<int>(bx), robots, ctl, no_rot, s1, incumbents, out);
  });
  return last_hip_status();
}

// ----------------------------- full-tree episodes ----------------------------
// The state: FtEpisode[R], the lockstep form's scratch (ftl_bytes), then the
// R configurations (mpc_fulltree_episodes_reset copies them in).
size_t mpc_fulltree_episodes_state_bytes(int32_t n_robots) {
  if (n_robots < 1) return 0;
  return ftl_bytes(n_robots) +
         static_cast<size_t>(n_robots) * sizeof(mpc_fulltree_episode_config_t);
}

int mpc_fulltree_episodes_reset(const mpc_fulltree_episode_config_t* cfgs, int32_t n_robots,
                                void* state, mpc_stream_t stream) {
  if (!cfgs || !state || n_robots < 1 || n_robots > 65535) return MPC_ERR_ARG;
  for (int32_t r = 0; r < n_robots; ++r)
    if (cfgs[r].max_calls < 0) return MPC_ERR_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  char* s = static_cast<char*>(state);
  auto* dcfg = reinterpret_cast<mpc_fulltree_episode_config_t*>(s + ftl_bytes(n_robots));
  // (pageable host source: the copy has read it when the call returns)
  if (hipMemcpyAsync(dcfg, cfgs, static_cast<size_t>(n_robots) * sizeof(*cfgs),
                     hipMemcpyHostToDevice, st) != hipSuccess)
    return MPC_ERR_HIP;
  k_ft_episodes_reset<<<static_cast<unsigned>(cdiv(n_robots, 256)), 256, 0, st>>>(
      dcfg, n_robots, reinterpret_cast<FtEpisode*>(s));
  return last_hip_status();
}

int mpc_fulltree_episodes_run(void* state, int32_t n_robots, const double* v_grid, int32_t n_v,
                              const double* beta_grid, int32_t n_beta, double L, double delta_t,
                              double eps, int32_t integrator, int32_t max_calls,
                              mpc_episode_log_t* log, int32_t log_capacity,
                              mpc_episodes_progress_t* progress, mpc_stream_t stream) {
  if (!state || !v_grid || !beta_grid || n_robots < 1 || n_robots > 65535 || n_v < 1 ||
      n_beta < 1 || max_calls < 0 || log_capacity < 0 || (log && log_capacity < 1) ||
      !(L > 0.0) || !(delta_t > 0.0))
    return MPC_ERR_ARG;
  if (static_cast<int64_t>(n_v) * n_beta > kFtEpMaxS1) return MPC_ERR_UNSUPPORTED;
  if (mode_ok(integrator, false) != MPC_OK) return MPC_ERR_UNSUPPORTED;
  if (max_calls == 0) return MPC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  FtEpisode* E = reinterpret_cast<FtEpisode*>(state);
  const int cap = log ? log_capacity : 0;
#ifndef MPC_FT_LOCKSTEP
#define MPC_FT_LOCKSTEP 1
#endif
  if (!MPC_FT_LOCKSTEP) {   // one block per robot, every call in one launch
    dispatch_mode2(integrator, [&](auto integ, auto rot) {
      constexpr int I = decltype(integ)::value;
      constexpr bool R = decltype(rot)::value;
      k_ft_episodes_run<I, R><<<n_robots, kBlock, 0, st>>>(
          E, v_grid, n_v, beta_grid, n_beta, L, delta_t, eps, max_calls, log, cap, progress);
    });
    return last_hip_status();
  }
  // load-balanced lockstep (mpc_ftepisodes.h): three launches per call over
  // the robots still running, the leaves of each spread over `grid` blocks
  char* s = static_cast<char*>(state);
  auto* ls = reinterpret_cast<FtLockstep*>(s + ftl_ls_offset(n_robots));
  auto* ctl = reinterpret_cast<FtCtl*>(s + ftl_ctl_offset(n_robots));
  auto* live = reinterpret_cast<int32_t*>(s + ftl_live_offset(n_robots));
  auto* robots = reinterpret_cast<FtRobot*>(s + ftl_robots_offset(n_robots));
  auto* part = reinterpret_cast<Rec*>(s + ftl_part_offset(n_robots));
  const int64_t s1 = static_cast<int64_t>(n_v) * n_beta;
  const int grid = static_cast<int>(std::min<int64_t>(kFtlMaxGrid, device_cus() * kFtWaves));
  dispatch_mode2(integrator, [&](auto integ, auto rot) {
    constexpr int I = decltype(integ)::value;
    constexpr bool R = decltype(rot)::value;
    for (int call = 0; call < max_calls; ++call) {
      k_ftl_prepare<I><<<1, kFtlPrepBlock, 0, st>>>(E, n_robots, v_grid, n_v, beta_grid, n_beta,
                                                     L, delta_t, eps, grid, ls, ctl, live,
                                                     robots);
      k_ftl_leaves<I, R><<<grid, kBlock, 0, st>>>(ls, ctl, live, robots, s1, part);
      k_ftl_update<I, R><<<n_robots, kBlock, 0, st>>>(E, ls, ctl, live, robots, part, s1,
                                                      delta_t, log, cap);
    }
  });
  if (progress)
    k_ftl_progress<<<static_cast<unsigned>(cdiv(n_robots, 256)), 256, 0, st>>>(E, n_robots,
                                                                               progress);
  return last_hip_status();
}

}  // extern "C"
