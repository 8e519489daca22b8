// Host build of the kernel's own per-candidate arithmetic (mpc_device.h:
// step, cost, mpc_trig.h) for tests/test_replica.py.  The GPU must reproduce
// these states and costs bit for bit: same source, same IEEE operations, fma
// and rint are exact on both sides.  Test infrastructure only.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <unordered_map>

#include "../diplomjourney_amd/csrc/mpc_device.h"

// The device's reciprocal estimates (v_rcp_f64 is not an IEEE operation):
// a GPU test fetches them for every denominator the rollout will form
// (replica_tan_q -> mpc_rcp_estimate) and installs them here; without a table
// the host build uses 1.0 / q.
static std::unordered_map<uint64_t, double> g_rcp;
static int64_t g_rcp_misses = 0;

static double rcp_from_table(double q) {
  uint64_t k;
  memcpy(&k, &q, 8);
  const auto it = g_rcp.find(k);
  if (it == g_rcp.end()) {
    ++g_rcp_misses;
    return 1.0 / q;
  }
  return it->second;
}

extern "C" void replica_set_rcp_table(const double* q, const double* r, int64_t n) {
  g_rcp.clear();
  g_rcp_misses = 0;
  if (n <= 0) {
    mpc::trig::g_host_rcp_estimate = nullptr;
    return;
  }
  g_rcp.reserve(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) {
    uint64_t k;
    memcpy(&k, &q[i], 8);
    g_rcp[k] = r[i];
  }
  mpc::trig::g_host_rcp_estimate = rcp_from_table;
}

extern "C" int64_t replica_rcp_misses(void) { return g_rcp_misses; }

// The denominators tan_small forms for these steering angles.
extern "C" void replica_tan_q(const double* beta, int64_t n, double* q) {
  for (int64_t i = 0; i < n; ++i) q[i] = mpc::trig::tan_small_q(beta[i] * beta[i]);
}

extern "C" int replica_rollout(const mpc_problem_t* p, const double* v, const double* b,
                               int64_t n_cand, int32_t n_steps, int32_t integ, double* states,
                               double* costs) {
  mpc::Consts K;
  memset(&K, 0, sizeof(K));
  K.x = p->x; K.y = p->y; K.phi = p->phi;
  K.x_t = p->x_t; K.y_t = p->y_t; K.x_0 = p->x_0; K.y_0 = p->y_0;
  K.A = p->y_t - p->y_0; K.B = p->x_t - p->x_0;
  K.C1 = p->x_t * p->y_0; K.C2 = p->y_t * p->x_0;
  double (*volatile pw)(double, double) = pow;
  K.inv_den = 1.0 / sqrt(pw(K.A, 2.0) + pw(K.B, 2.0));
  K.L = p->L;
  int e;
  K.L_pow2 = frexp(p->L, &e) == 0.5;
  K.inv_L = K.L_pow2 ? 1.0 / p->L : 0.0;
  K.h = p->t_b - p->t_a;
  K.hlgth = 0.5 * (p->t_b - p->t_a);
  double (*volatile sn)(double) = sin;
  double (*volatile cs)(double) = cos;
  K.s0 = sn(p->phi);
  K.c0 = cs(p->phi);
  const bool rot = (integ & MPC_HEADING_ROTATE) != 0;
  const bool cum = (integ & MPC_HEADING_CUMULATIVE) != 0;
  const int ig = integ & 0xff;
  double traj[3 * MPC_MAX_STEPS];
  for (int64_t c = 0; c < n_cand; ++c) {
    double cst;
    if (ig == MPC_INTEG_RECT && cum)
      cst = mpc::rollout_candidate<MPC_INTEG_RECT, mpc::kRotCum>(K, v, b, n_cand, c, n_steps, traj);
    else if (ig == MPC_INTEG_RECT)
      cst = rot ? mpc::rollout_candidate<MPC_INTEG_RECT, 1>(K, v, b, n_cand, c, n_steps, traj)
                : mpc::rollout_candidate<MPC_INTEG_RECT, 0>(K, v, b, n_cand, c, n_steps, traj);
    else
      cst = rot ? mpc::rollout_candidate<MPC_INTEG_QK21, 1>(K, v, b, n_cand, c, n_steps, traj)
                : mpc::rollout_candidate<MPC_INTEG_QK21, 0>(K, v, b, n_cand, c, n_steps, traj);
    if (states)
      for (int s = 0; s < n_steps; ++s)
        for (int k = 0; k < 3; ++k) states[(s * 3 + k) * n_cand + c] = traj[3 * s + k];
    if (costs) costs[c] = cst;
  }
  return 0;
}
