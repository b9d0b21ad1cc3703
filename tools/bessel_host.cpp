// Host build of rh_bessel.h for the CPU check against scipy (tests/test_bessel.py):
// D_n(x) = 0.5 (H1_{n-1}(x) - H1_{n+1}(x)), n = 0..11, exactly as k_qtf_hankel writes it.
#include "../raft-teststuff_amd/csrc/rh_bessel.h"

extern "C" void rh_hankel_deriv_host(int n, const double* x, double* out /* [n][12][2] */) {
  for (int i = 0; i < n; ++i) {
    double J[13], Y[13];
    rh::bessel_jy12(x[i], J, Y);
    double* o = out + (long)i * 24;
    o[0] = -J[1];
    o[1] = -Y[1];
    for (int k = 1; k < 12; ++k) {
      o[2 * k] = 0.5 * (J[k - 1] - J[k + 1]);
      o[2 * k + 1] = 0.5 * (Y[k - 1] - Y[k + 1]);
    }
  }
}
