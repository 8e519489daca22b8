// Host build of the kernel's own per-candidate arithmetic (mpc_device.h:
// step, cost, mpc_trig.h) for tests/test_replica.py.  The GPU must reproduce
// these states and costs bit for bit: same source, same IEEE operations, fma
// and rint are exact on both sides.  Test infrastructure only.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../diplomjourney_amd/csrc/mpc_device.h"

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
  K.den = sqrt(pw(K.A, 2.0) + pw(K.B, 2.0));
  K.L = p->L;
  int e;
  K.L_pow2 = frexp(p->L, &e) == 0.5;
  K.inv_L = K.L_pow2 ? 1.0 / p->L : 0.0;
  K.h = p->t_b - p->t_a;
  K.hlgth = 0.5 * (p->t_b - p->t_a);
  for (int64_t c = 0; c < n_cand; ++c) {
    double x = K.x, y = K.y, ph = K.phi;
    for (int s = 0; s < n_steps; ++s) {
      if (integ == MPC_INTEG_RECT)
        mpc::step<MPC_INTEG_RECT>(x, y, ph, v[s * n_cand + c], b[s * n_cand + c], K);
      else
        mpc::step<MPC_INTEG_QK21>(x, y, ph, v[s * n_cand + c], b[s * n_cand + c], K);
      if (states) {
        states[(s * 3 + 0) * n_cand + c] = x;
        states[(s * 3 + 1) * n_cand + c] = y;
        states[(s * 3 + 2) * n_cand + c] = ph;
      }
    }
    if (costs) costs[c] = mpc::cost(x, y, K);
  }
  return 0;
}
