// rh_bessel.h -- Bessel functions J_n, Y_n (n = 0..12, real x > 0) for the Kim & Yue Hankel
// table (raft/raft_member.py:1104-1107 evaluates scipy.special.hankel1 there).  Host + device:
// the same code is compiled for gfx950 (rh_qtf.hip) and for the CPU check of the restatement
// against scipy (tests/test_bessel.py builds tools/bessel_host.cpp with g++).
//   J : power series for x < 2; otherwise Miller's downward recurrence from N = 2 x + 40,
//       normalised by J0 + 2 (J2 + J4 + ...) = 1, rescaled against overflow (A&S 9.1.46, 9.12);
//   Y0: (pi/2) Y0 = (ln(x/2) + gamma) J0 - 2 sum_k (-1)^k J_2k / k              (A&S 9.1.88)
//   Y1 = -Y0': (pi/2) Y1 = (ln(x/2) + gamma) J1 - J0 / x + sum_k (-1)^k (J_2k-1 - J_2k+1) / k;
//   Y_n: forward recurrence Y_{n+1} = (2n/x) Y_n - Y_{n-1} (stable for Y).
// The J_k of the series / recurrence feed the Y0, Y1 sums: no library Bessel call is used.
#pragma once
#include <math.h>

#if defined(__HIPCC__)
#define RH_HD __host__ __device__
#else
#define RH_HD
#endif

namespace rh {

// Every J / Y index below is a compile-time constant (the loops that store are unrolled):
// a lane-dependent index into a register array would need divergent register indexing.
RH_HD inline void bessel_jy12(double x, double* J, double* Y) {
  const double kEulerGamma = 0.57721566490153286061;
  const double kPi = 3.14159265358979323846;
  double s0 = 0.0, s1 = 0.0, norm = 1.0;
  if (x < 2.0) {
    // series; the sums need J_k up to k = 31 (x < 2: J_31 < 1e-40)
    const double q = -0.25 * x * x;
    double lead = 1.0;                 // (x/2)^k / k!
    double jprev2 = 0.0;               // J_{k-2}
    double jprev1 = 0.0;               // J_{k-1}
    auto series = [&](int k) {
      double term = lead, jk = lead;
      for (int m = 1; m <= 18; ++m) {
        term *= q / (double)(m * (m + k));
        jk += term;
      }
      if (k >= 2 && (k & 1) == 0) s0 += (((k / 2) & 1) ? -1.0 : 1.0) * jk / (k / 2);
      if (k >= 3 && (k & 1) == 1) {    // (J_{2kk-1} - J_{2kk+1}) with 2kk + 1 = k
        const int kk = (k - 1) / 2;
        s1 += ((kk & 1) ? -1.0 : 1.0) * (jprev2 - jk) / kk;
      }
      jprev2 = jprev1;
      jprev1 = jk;
      lead *= 0.5 * x / (double)(k + 1);
      return jk;
    };
#pragma unroll
    for (int k = 0; k <= 12; ++k) J[k] = series(k);
#pragma unroll 1
    for (int k = 13; k < 32; ++k) (void)series(k);
  } else {
    int N = 2 * (int)x + 40;
    N += N & 1;                        // even start
    double bjp = 0.0, bj = 1.0;        // J_{k+1}, J_k (unnormalised)
    double Jt[13];                     // J_0..J_12 once the sweep reaches them
    norm = 0.0;
    auto step = [&](int k) {           // bj <- J_{k-1}; accumulate the sums for m = k - 1
      const double bjm = (2.0 * k / x) * bj - bjp;
      const double jm2 = bjp;          // J_{m+2}
      bjp = bj;
      bj = bjm;
      const int m = k - 1;
      if (m > 0 && (m & 1) == 0) {
        norm += 2.0 * bj;
        s0 += (((m / 2) & 1) ? -1.0 : 1.0) * bj / (m / 2);
      }
      if (m & 1) {                     // m = 2 kk - 1: (-1)^kk (J_m - J_{m+2}) / kk
        const int kk = (m + 1) / 2;
        s1 += ((kk & 1) ? -1.0 : 1.0) * (bj - jm2) / kk;
      }
    };
    auto rescale = [&](double r) {
      bj *= r;
      bjp *= r;
      norm *= r;
      s0 *= r;
      s1 *= r;
    };
#pragma unroll 1
    for (int k = N; k >= 14; --k) {    // no stores above order 12
      step(k);
      if (fabs(bj) > 1e250) rescale(1e-250);
    }
#pragma unroll
    for (int k = 13; k >= 1; --k) {    // orders 12 .. 0: static indices
      step(k);
      Jt[k - 1] = bj;
      if (fabs(bj) > 1e250) {
        rescale(1e-250);
#pragma unroll
        for (int n = k - 1; n <= 12; ++n) Jt[n] *= 1e-250;
      }
    }
    norm += bj;                        // + J0
#pragma unroll
    for (int n = 0; n <= 12; ++n) J[n] = Jt[n];
  }
  const double inv = 1.0 / norm;
#pragma unroll
  for (int n = 0; n <= 12; ++n) J[n] *= inv;
  s0 *= inv;
  s1 *= inv;
  const double lg = log(0.5 * x) + kEulerGamma;
  Y[0] = (2.0 / kPi) * (lg * J[0] - 2.0 * s0);
  Y[1] = (2.0 / kPi) * (lg * J[1] - J[0] / x + s1);
#pragma unroll
  for (int n = 1; n < 12; ++n) Y[n + 1] = (2.0 * n / x) * Y[n] - Y[n - 1];
}

}  // namespace rh
