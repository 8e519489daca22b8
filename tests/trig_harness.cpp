// Host build of diplomjourney_amd/csrc/mpc_trig.h for tests/test_trig.py.
#include <stdint.h>
#include "../diplomjourney_amd/csrc/mpc_trig.h"

extern "C" void trig_eval(const double* x, int64_t n, double* t, double* s, double* c) {
  for (int64_t i = 0; i < n; ++i) {
    t[i] = mpc::trig::tan_fast(x[i]);
    mpc::trig::sincos_fast(x[i], &s[i], &c[i]);
  }
}

extern "C" void trig_tan_small(const double* x, int64_t n, double* t) {
  for (int64_t i = 0; i < n; ++i) t[i] = mpc::trig::tan_small(x[i]);
}
