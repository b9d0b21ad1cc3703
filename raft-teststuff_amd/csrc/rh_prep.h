// rh_prep.h -- native per-design host preparation: members, statics, added mass and the
// device-table layout, for many designs at once on host threads (rh_prep_designs).
//
// The same arithmetic as the Python mirror (restated from the reference, file:line per step):
//   member discretisation and pose   raft/member.py      <- raft/raft_member.py:23-304
//   member inertia / hydrostatics     raft/statics.py     <- raft/raft_member.py:307-874
//   RNA inertia, FOWT totals          raft/statics.py     <- raft/raft_fowt.py:291-565, raft_rotor.py:376-458
//   added mass, inertial excitation   raft/member.py      <- raft/raft_member.py:877-1050
//   node / member tables, M, B, C     raft/prep.py        (device layout, raft/raft_model.py:911-913)
// The Python path is the parity reference for this code (tests/test_native_prep.py compares
// every table and matrix); it is what a design sweep (C5) spends its host time on, so it runs
// here in C++ without per-design interpreter work.  Host code only (no device calls).
//
// Spec format: one float64 record per design (raft/native_prep.py design_spec writes it):
//   header [kHdr]: magic, nmemb, nrot, rho, g, r6[6], flags of the given statics
//                  (M_struc, B_struc, C_struc, C_hydro, C_moor), then the given 6x6 blocks
//   per member   : type, circ, potMod, MCF, nacelle, nst, ncap, nhead, has_t, gamma, dlsMax,
//                  rho_shell, rA[3], rB[3], headings[nhead] (deg, heading_adjust included),
//                  stations[nst], d[nst] or sl[nst][2], t[nst] (has_t), l_fill[nst-1],
//                  rho_fill[nst-1], Cd_q, Cd_p1, Cd_p2, Cd_End, Ca_q, Ca_p1, Ca_p2, Ca_End [nst each],
//                  cap_stations[ncap], cap_t[ncap], cap_d_in[ncap]
//   per rotor    : mRNA, IxRNA, IrRNA, xCG_RNA, overhang, shaft_tilt (rad), shaft_toe (rad),
//                  yaw_mode, r_rel[3] (rRNA or the default), has_hHub, hHub
#pragma once
#include <algorithm>
#include <atomic>
#include <cmath>
#include <string>
#include <thread>
#include <vector>

#include "rh_bessel.h"   // J_n, Y_n of real x: the MacCamy-Fuchs Hankel functions (host side here)

#pragma clang fp contract(off)   // NumPy rounds every product and sum separately

namespace rhp {

constexpr double kPi = 3.141592653589793;
constexpr int kMagic = 7301;
constexpr int kHdr = 16;

struct V3 {
  double x[3];
  double& operator[](int i) { return x[i]; }
  double operator[](int i) const { return x[i]; }
};
struct M3 {
  double a[3][3];
};
struct M6 {
  double a[6][6];
};

inline V3 v3(double a, double b, double c) { return V3{{a, b, c}}; }
inline V3 add(const V3& a, const V3& b) { return v3(a[0] + b[0], a[1] + b[1], a[2] + b[2]); }
inline V3 sub(const V3& a, const V3& b) { return v3(a[0] - b[0], a[1] - b[1], a[2] - b[2]); }
inline V3 scl(const V3& a, double s) { return v3(a[0] * s, a[1] * s, a[2] * s); }
inline V3 cross(const V3& a, const V3& b) {   // np.cross
  return v3(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
}
inline double dot(const V3& a, const V3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline M3 mm(const M3& A, const M3& B) {
  M3 C;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C.a[i][j] = A.a[i][0] * B.a[0][j] + A.a[i][1] * B.a[1][j] + A.a[i][2] * B.a[2][j];
  return C;
}
inline V3 mv(const M3& A, const V3& x) {
  V3 y;
  for (int i = 0; i < 3; ++i) y[i] = A.a[i][0] * x[0] + A.a[i][1] * x[1] + A.a[i][2] * x[2];
  return y;
}
inline M3 tr(const M3& A) {
  M3 B;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) B.a[i][j] = A.a[j][i];
  return B;
}
inline M3 outer(const V3& a, const V3& b) {
  M3 C;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C.a[i][j] = a[i] * b[j];
  return C;
}
inline M3 zero3() { return M3{}; }
inline M6 zero6() { return M6{}; }

// raft/helpers.py:357-384 (hydro_math.rotation_matrix)
inline M3 rotation_matrix(double x3, double x2, double x1) {
  const double s1 = std::sin(x1), c1 = std::cos(x1), s2 = std::sin(x2), c2 = std::cos(x2), s3 = std::sin(x3),
               c3 = std::cos(x3);
  return M3{{{c1 * c2, c1 * s2 * s3 - c3 * s1, s1 * s3 + c1 * c3 * s2},
             {c2 * s1, c1 * c3 + s1 * s2 * s3, c3 * s1 * s2 - c1 * s3},
             {-s2, c2 * s3, c2 * c3}}};
}
inline M3 alternator(const V3& r) {   // getH (raft/helpers.py:346-355)
  return M3{{{0, r[2], -r[1]}, {-r[2], 0, r[0]}, {r[1], -r[0], 0}}};
}
// raft/helpers.py:455-478
inline M6 translate_3to6(const M3& Min, const V3& r) {
  const M3 H = alternator(r);
  const M3 MH = mm(Min, H), HMH = mm(mm(H, Min), tr(H));
  M6 o = zero6();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      o.a[i][j] = Min.a[i][j];
      o.a[i][3 + j] = MH.a[i][j];
      o.a[3 + j][i] = MH.a[i][j];
      o.a[3 + i][3 + j] = HMH.a[i][j];
    }
  return o;
}
inline M3 blk(const M6& M, int r0, int c0) {
  M3 B;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) B.a[i][j] = M.a[r0 + i][c0 + j];
  return B;
}
// raft/helpers.py:481-503
inline M6 translate_6to6(const M6& Min, const V3& r) {
  const M3 H = alternator(r), Ht = tr(H);
  const M3 A = blk(Min, 0, 0), Bm = blk(Min, 0, 3), Cm = blk(Min, 3, 0), D = blk(Min, 3, 3);
  const M3 AH = mm(A, H), HAHt = mm(mm(H, A), Ht), CH = mm(Cm, H), HtB = mm(Ht, Bm);
  M6 o = zero6();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      o.a[i][j] = A.a[i][j];
      o.a[i][3 + j] = AH.a[i][j] + Bm.a[i][j];
      o.a[3 + i][3 + j] = ((HAHt.a[i][j] + CH.a[i][j]) + HtB.a[i][j]) + D.a[i][j];
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) o.a[3 + j][i] = o.a[i][3 + j];
  return o;
}
inline void acc6(M6& A, const M6& B) {
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) A.a[i][j] += B.a[i][j];
}

// np.interp(x, xp, fp) with the default end values (fp[0] / fp[-1])
inline double np_interp(double x, const double* xp, const double* fp, int n) {
  if (x <= xp[0]) return fp[0];
  if (x >= xp[n - 1]) return fp[n - 1];
  int lo = 0, hi = n - 1;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (xp[mid] <= x) lo = mid; else hi = mid;
  }
  if (xp[lo] == x) return fp[lo];
  const double slope = (fp[lo + 1] - fp[lo]) / (xp[lo + 1] - xp[lo]);
  return slope * (x - xp[lo]) + fp[lo];
}

// ------------------------------------------------------------------------------- member
struct Member {
  int type = 2, circ = 1, potMod = 0, mcf = 0, nacelle = 0, has_t = 0;
  double gamma = 0, dlsMax = 5, rho_shell = 8500, l = 0;
  V3 rA0{}, rB0{};
  std::vector<double> st, d, sl0, sl1, t, l_fill, rho_fill, cdq, cdp1, cdp2, cdend, caq, cap1, cap2, caend, cap_st,
      cap_t, cap_d;
  // discretisation
  int ns = 0;
  std::vector<double> ls, dls, ds0, ds1, drs0, drs1;
  // pose
  M3 R{};
  V3 q{}, p1{}, p2{}, rA{}, rB{};
  std::vector<V3> r;
  M3 qMat{}, p1Mat{}, p2Mat{};
  // hydro constants
  std::vector<double> a_i;
  std::vector<M3> Imat;
  std::vector<double> imat_mcf;   // MacCamy-Fuchs members: [ns][9][nw] complex (re, im), else empty
  M6 M_struc{};
  std::vector<double> mfill, pfill;

  double coef(const std::vector<double>& f, int il) const { return np_interp(ls[il], st.data(), f.data(), (int)st.size()); }

  // raft/member.py _discretise (raft/raft_member.py:169-220)
  void discretise() {
    const int n = (int)st.size();
    auto D0 = [&](int i) { return circ ? d[i] : sl0[i]; };
    auto D1 = [&](int i) { return circ ? d[i] : sl1[i]; };
    ls = {0.0};
    dls = {0.0};
    ds0 = {0.5 * D0(0)};
    ds1 = {0.5 * D1(0)};
    drs0 = {0.5 * D0(0)};
    drs1 = {0.5 * D1(0)};
    for (int i = 1; i < n; ++i) {
      const double lstrip = st[i] - st[i - 1];
      if (lstrip > 0.0) {
        const int nsi = (int)std::ceil(lstrip / dlsMax);
        const double dlstrip = lstrip / nsi;
        const double m0 = 0.5 * (D0(i) - D0(i - 1)) / lstrip, m1 = 0.5 * (D1(i) - D1(i - 1)) / lstrip;
        for (int j = 0; j < nsi; ++j) {
          ls.push_back(st[i - 1] + dlstrip * (0.5 + j));
          dls.push_back(dlstrip);
          ds0.push_back(D0(i - 1) + dlstrip * 2 * m0 * (0.5 + j));
          ds1.push_back(D1(i - 1) + dlstrip * 2 * m1 * (0.5 + j));
          drs0.push_back(dlstrip * m0);
          drs1.push_back(dlstrip * m1);
        }
      } else if (lstrip == 0.0) {
        ls.push_back(st[i - 1]);
        dls.push_back(0.0);
        ds0.push_back(0.5 * (D0(i - 1) + D0(i)));
        ds1.push_back(0.5 * (D1(i - 1) + D1(i)));
        drs0.push_back(0.5 * (D0(i) - D0(i - 1)));
        drs1.push_back(0.5 * (D1(i) - D1(i - 1)));
      }
    }
    ls.push_back(st[n - 1]);
    dls.push_back(0.0);
    ds0.push_back(0.5 * D0(n - 1));
    ds1.push_back(0.5 * D1(n - 1));
    drs0.push_back(-0.5 * D0(n - 1));
    drs1.push_back(-0.5 * D1(n - 1));
    ns = (int)ls.size();
    r.assign(ns, V3{});
    a_i.assign(ns, 0.0);
    Imat.assign(ns, zero3());
  }

  // raft/member.py setPosition (raft/raft_member.py:245-304)
  void set_position(const double* r6) {
    const V3 rAB = sub(rB0, rA0);
    const double nrm = std::sqrt(dot(rAB, rAB));
    const V3 qq = v3(rAB[0] / nrm, rAB[1] / nrm, rAB[2] / nrm);
    const double beta = std::atan2(qq[1], qq[0]);
    const double phi = std::atan2(std::sqrt(qq[0] * qq[0] + qq[1] * qq[1]), qq[2]);
    const double s1 = std::sin(beta), c1 = std::cos(beta), s2 = std::sin(phi), c2 = std::cos(phi);
    const double g = gamma * (kPi / 180.0);
    const double s3 = std::sin(g), c3 = std::cos(g);
    const M3 R0{{{c1 * c2 * c3 - s1 * s3, -c3 * s1 - c1 * c2 * s3, c1 * s2},
                 {c1 * s3 + c2 * c3 * s1, c1 * c3 - c2 * s1 * s3, s1 * s2},
                 {-c3 * s2, s2 * s3, c2}}};
    const V3 pp1 = v3(R0.a[0][0], R0.a[1][0], R0.a[2][0]);
    const V3 pp2 = cross(qq, pp1);
    const M3 Rp = rotation_matrix(r6[3], r6[4], r6[5]);
    R = mm(Rp, R0);
    q = mv(Rp, qq);
    p1 = mv(Rp, pp1);
    p2 = mv(Rp, pp2);
    const V3 t6 = v3(r6[0], r6[1], r6[2]);
    rA = add(t6, mv(Rp, rA0));
    rB = add(t6, mv(Rp, rB0));
    const V3 rABd = sub(rB, rA);
    for (int i = 0; i < ns; ++i) r[i] = add(rA, scl(rABd, ls[i] / l));
    qMat = outer(q, q);
    p1Mat = outer(p1, p1);
    p2Mat = outer(p2, p2);
  }

  double side_volume(int il) const {
    double v = circ ? 0.25 * kPi * (ds0[il] * ds0[il]) * dls[il] : ds0[il] * ds1[il] * dls[il];
    if (r[il][2] + 0.5 * dls[il] > 0) v = v * (0.5 * dls[il] - r[il][2]) / dls[il];
    return v;
  }
  void end_volume_area(int il, double& v, double& a) const {
    if (circ) {
      const double ds = ds0[il], drs = drs0[il];
      v = kPi / 12.0 * std::fabs(std::pow(ds + drs, 3.0) - std::pow(ds - drs, 3.0));
      a = kPi * ds * drs;
    } else {
      const double mp = ((ds0[il] + drs0[il]) + (ds1[il] + drs1[il])) / 2;
      const double mn = ((ds0[il] - drs0[il]) + (ds1[il] - drs1[il])) / 2;
      v = kPi / 12.0 * (std::pow(mp, 3.0) - std::pow(mn, 3.0));
      a = (ds0[il] + drs0[il]) * (ds1[il] + drs1[il]) - (ds0[il] - drs0[il]) * (ds1[il] - drs1[il]);
    }
  }

  // raft/member.py getCmSides (raft/raft_member.py:1053-1088): the side inertia coefficients
  // at wave number k, MacCamy-Fuchs Cm = 4i / (pi (kR)^2 H1'(kR)) with
  // H1'(x) = (H_0(x) - H_2(x)) / 2 (H = H^(1) = J + iY), blended from the plain 1 + Ca at
  // k = 0 to Cm at k = pi / (5 R) by a cosine ramp
  void cm_sides(int il, double k, double* c1, double* c2) const {   // c1, c2: (re, im)
    const double Cm_p1_0 = 1. + coef(cap1, il), Cm_p2_0 = 1. + coef(cap2, il);
    const double R = ds0[il] / 2;
    const double x = k * R;
    double Cr = 0.0, Ci = 0.0;
    if (x > 0) {
      double J[13], Y[13];
      rh::bessel_jy12(x, J, Y);
      const double hr = 0.5 * (J[0] - J[2]), hi = 0.5 * (Y[0] - Y[2]);   // H1'(x)
      const double s = kPi * (x * x);
      const double dr = s * hr, di = s * hi;                             // pi (kR)^2 H1'
      // 4i / (dr + i di) in the form of NumPy's complex scalar division (Smith's, by a reciprocal)
      if (std::fabs(dr) >= std::fabs(di)) {
        const double rat = di / dr, scl = 1.0 / (dr + di * rat);
        Cr = (0.0 + 4.0 * rat) * scl;
        Ci = (4.0 - 0.0 * rat) * scl;
      } else {
        const double rat = dr / di, scl = 1.0 / (di + dr * rat);
        Cr = (0.0 * rat + 4.0) * scl;
        Ci = (4.0 * rat - 0.0) * scl;
      }
    }
    const double Tr = kPi / 5 / R;
    double ramp = k < Tr ? 0.5 * (1 - std::cos(kPi * (k - 0) / Tr)) : 1.0;
    if (k <= 0) ramp = 0.0;
    c1[0] = Cr * ramp + Cm_p1_0 * (1 - ramp);
    c1[1] = Ci * ramp;
    c2[0] = Cr * ramp + Cm_p2_0 * (1 - ramp);
    c2[1] = Ci * ramp;
  }

  // raft/member.py calcHydroConstants (raft/raft_member.py:877-1050); a MacCamy-Fuchs member's
  // inertial excitation matrix per wave number k[nw] goes to imat_mcf (its Imat stays zero, as
  // in the Python path), every other member's Imat is frequency independent
  M6 hydro_constants(const V3& r_ref, double rho, const double* kw, int nw) {
    M6 A = zero6();
    if (mcf) imat_mcf.assign((size_t)ns * 9 * nw * 2, 0.0);
    for (int il = 0; il < ns; ++il) {
      if (!(r[il][2] < 0) || potMod) continue;
      const double v_side = side_volume(il);
      const double Ca_p1 = coef(cap1, il), Ca_p2 = coef(cap2, il), Ca_End = coef(caend, il);
      double v_end, a_end;
      end_volume_area(il, v_end, a_end);
      const double c1 = 1. + Ca_p1, c2 = 1. + Ca_p2;
      const double rvs = rho * v_side, rve = rho * v_end * Ca_End;
      M3 I, Am;
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          I.a[i][j] = rvs * (c1 * p1Mat.a[i][j] + c2 * p2Mat.a[i][j]) + rve * qMat.a[i][j];
          Am.a[i][j] = rvs * (Ca_p1 * p1Mat.a[i][j] + Ca_p2 * p2Mat.a[i][j]) + rve * qMat.a[i][j];
        }
      if (mcf) {
        // rho v_side (c1 p1Mat + c2 p2Mat) + I_end with complex c1, c2 (NumPy's order)
        double* Im = imat_mcf.data() + (size_t)il * 9 * nw * 2;
        for (int ik = 0; ik < nw; ++ik) {
          double m1[2], m2[2];
          cm_sides(il, kw[ik], m1, m2);
          for (int e = 0; e < 9; ++e) {
            const int i = e / 3, j = e % 3;
            const double tr = m1[0] * p1Mat.a[i][j] + m2[0] * p2Mat.a[i][j];
            const double ti = m1[1] * p1Mat.a[i][j] + m2[1] * p2Mat.a[i][j];
            Im[((size_t)e * nw + ik) * 2] = rvs * tr + rve * qMat.a[i][j];
            Im[((size_t)e * nw + ik) * 2 + 1] = rvs * ti;
          }
        }
      } else {
        Imat[il] = I;
      }
      a_i[il] = a_end;
      acc6(A, translate_3to6(Am, sub(r[il], r_ref)));
    }
    return A;
  }
};

// ---------------------------------------------------------------------------- statics
// raft/statics.py frustum_vcv (raft/helpers.py:36-63); rect: pairs of side lengths
inline void frustum_vcv(bool circ, double dA0, double dA1, double dB0, double dB1, double H, double& V, double& hc) {
  const double sA = circ ? dA0 : dA0 + dA1, sB = circ ? dB0 : dB0 + dB1;
  if (sA == 0 && sB == 0) {
    V = hc = 0.0;
    return;
  }
  double a1, a2, am;
  if (circ) {
    a1 = 0.25 * kPi * (dA0 * dA0);
    a2 = 0.25 * kPi * (dB0 * dB0);
    am = 0.25 * kPi * dA0 * dB0;
  } else {
    a1 = dA0 * dA1;
    a2 = dB0 * dB1;
    am = std::sqrt(a1 * a2);
  }
  V = (a1 + a2 + am) * H / 3;
  hc = ((a1 + 2 * am + 3 * a2) / (a1 + am + a2)) * H / 4;
}

inline void frustum_moi(double dA, double dB, double H, double p, double& Ir, double& Ia) {
  if (H == 0) {
    Ir = Ia = 0.0;
    return;
  }
  const double r1 = dA / 2, r2 = dB / 2;
  if (dA == dB) {
    Ir = (1.0 / 12) * (p * H * kPi * (r1 * r1)) * (3 * (r1 * r1) + 4 * (H * H));
    Ia = 0.5 * p * kPi * H * std::pow(r1, 4.0);
    return;
  }
  const double q5 = (std::pow(r2, 5.0) - std::pow(r1, 5.0)) / (r2 - r1);
  Ir = (1.0 / 20) * p * kPi * H * q5 + (1.0 / 30) * p * kPi * std::pow(H, 3.0) * (r1 * r1 + 3 * r1 * r2 + 6 * (r2 * r2));
  Ia = (1.0 / 10) * p * kPi * H * q5;
}

inline void rect_frustum_moi(double La, double Wa, double Lb, double Wb, double H, double p, double& Ixx, double& Iyy,
                             double& Izz) {
  if (H == 0) {
    Ixx = Iyy = Izz = 0.0;
    return;
  }
  if (La == Lb && Wa == Wb) {
    const double M = p * La * Wa * H;
    Ixx = (1.0 / 12) * M * (Wa * Wa + 4 * (H * H));
    Iyy = (1.0 / 12) * M * (La * La + 4 * (H * H));
    Izz = (1.0 / 12) * M * (La * La + Wa * Wa);
    return;
  }
  double x2, y2, z2;
  const double H3 = std::pow(H, 3.0);
  if (La != Lb && Wa != Wb) {
    const double dL = Lb - La, dW = Wb - Wa;
    x2 = (1.0 / 12) * p *
         (std::pow(dL, 3.0) * H * (Wb / 5 + Wa / 20) + (dL * dL) * La * H * (3 * Wb / 4 + Wa / 4) +
          dL * (La * La) * H * (Wb + Wa / 2) + std::pow(La, 3.0) * H * (Wb / 2 + Wa / 2));
    y2 = (1.0 / 12) * p *
         (std::pow(dW, 3.0) * H * (Lb / 5 + La / 20) + (dW * dW) * Wa * H * (3 * Lb / 4 + La / 4) +
          dW * (Wa * Wa) * H * (Lb + La / 2) + std::pow(Wa, 3.0) * H * (Lb / 2 + La / 2));
    z2 = p * (Wb * Lb / 5 + Wa * Lb / 20 + La * Wb / 20 + Wa * La * (1.0 / 30)) * H3;
  } else if (La == Lb) {
    const double L = La;
    x2 = (1.0 / 24) * p * std::pow(L, 3.0) * H * (Wb + Wa);
    y2 = (1.0 / 48) * p * L * H * (std::pow(Wb, 3.0) + Wa * (Wb * Wb) + (Wa * Wa) * Wb + std::pow(Wa, 3.0));
    z2 = (1.0 / 12) * p * L * H3 * (3 * Wb + Wa);
  } else {
    const double W = Wa;
    x2 = (1.0 / 48) * p * W * H * (std::pow(Lb, 3.0) + La * (Lb * Lb) + (La * La) * Lb + std::pow(La, 3.0));
    y2 = (1.0 / 24) * p * std::pow(W, 3.0) * H * (Lb + La);
    z2 = (1.0 / 12) * p * W * H3 * (3 * Lb + La);
  }
  Ixx = y2 + z2;
  Iyy = x2 + z2;
  Izz = x2 + y2;
}

// raft/statics.py _place (raft/raft_member.py:538-547)
inline void place(M6& Mloc, double mass, double Ix, double Iy, double Iz, const M3& R, const V3& center, bool integer) {
  M6 Mm = zero6();
  Mm.a[0][0] = Mm.a[1][1] = Mm.a[2][2] = mass;
  const M3 T = tr(R);
  M3 Id = zero3();
  Id.a[0][0] = Ix;
  Id.a[1][1] = Iy;
  Id.a[2][2] = Iz;
  const M3 Irot = mm(tr(T), mm(Id, T));
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Mm.a[3 + i][3 + j] = integer ? std::trunc(Irot.a[i][j]) : Irot.a[i][j];
  acc6(Mloc, translate_6to6(Mm, center));
}

// raft/statics.py member_inertia (raft/raft_member.py:307-707); returns mass, sets center
inline bool member_inertia(Member& m, const V3& rPRP, double& mass_out, V3& center_out, std::string& err) {
  m.M_struc = zero6();
  V3 mass_center{};
  double Ixx = 0, Iyy = 0, Izz = 0;
  const int n = (int)m.st.size();
  m.mfill.clear();
  m.pfill.clear();
  for (int i = 1; i < n; ++i) {
    const double l = m.st[i] - m.st[i - 1];
    double mass, m_fill, rho_fill;
    V3 center{};
    if (l == 0.0) {
      mass = m_fill = rho_fill = 0.0;
    } else {
      const double rho_shell = m.rho_shell, l_fill = m.l_fill[i - 1];
      rho_fill = m.rho_fill[i - 1];
      double dA0, dA1, dB0, dB1;
      if (m.circ) {
        dA0 = dA1 = m.d[i - 1];
        dB0 = dB1 = m.d[i];
      } else {
        dA0 = m.sl0[i - 1];
        dA1 = m.sl1[i - 1];
        dB0 = m.sl0[i];
        dB1 = m.sl1[i];
      }
      const double dAi0 = dA0 - 2 * m.t[i - 1], dAi1 = dA1 - 2 * m.t[i - 1];
      const double dBi0 = dB0 - 2 * m.t[i], dBi1 = dB1 - 2 * m.t[i];
      double V_o, hco, V_i, hci;
      frustum_vcv(m.circ, dA0, dA1, dB0, dB1, l, V_o, hco);
      frustum_vcv(m.circ, dAi0, dAi1, dBi0, dBi1, l, V_i, hci);
      const double v_shell = V_o - V_i;
      const double m_shell = v_shell * rho_shell;
      const double hc_shell = (hco * V_o - hci * V_i) / (V_o - V_i);
      const double dBf0 = (dBi0 - dAi0) * (l_fill / l) + dAi0, dBf1 = (dBi1 - dAi1) * (l_fill / l) + dAi1;
      double v_fill, hc_fill;
      frustum_vcv(m.circ, dAi0, dAi1, dBf0, dBf1, l_fill, v_fill, hc_fill);
      m_fill = v_fill * rho_fill;
      mass = m_shell + m_fill;
      const double hc = (hc_fill * m_fill + hc_shell * m_shell) / mass;
      if (m.circ) {
        double Ir_o, Ia_o, Ir_i, Ia_i, Ir_f, Ia_f;
        frustum_moi(dA0, dB0, l, rho_shell, Ir_o, Ia_o);
        frustum_moi(dAi0, dBi0, l, rho_shell, Ir_i, Ia_i);
        frustum_moi(dAi0, dBf0, l_fill, rho_fill, Ir_f, Ia_f);
        const double I_rad = (Ir_o - Ir_i) + Ir_f - mass * (hc * hc);
        Ixx = Iyy = I_rad;
        Izz = (Ia_o - Ia_i) + Ia_f;
      } else {
        double xo, yo, zo, xi, yi, zi, xf, yf, zf;
        rect_frustum_moi(dA0, dA1, dB0, dB1, l, rho_shell, xo, yo, zo);
        rect_frustum_moi(dAi0, dAi1, dBi0, dBi1, l, rho_shell, xi, yi, zi);
        rect_frustum_moi(dAi0, dAi1, dBf0, dBf1, l_fill, rho_fill, xf, yf, zf);
        Ixx = (xo - xi) + xf - mass * (hc * hc);
        Iyy = (yo - yi) + yf - mass * (hc * hc);
        Izz = (zo - zi) + zf;
      }
      center = sub(add(m.rA, scl(m.q, m.st[i - 1] + hc)), rPRP);
      (void)m_shell;
      m.mfill.push_back(m_fill);
      m.pfill.push_back(rho_fill);
      mass_center = add(mass_center, scl(center, mass));
      place(m.M_struc, mass, Ixx, Iyy, Izz, m.R, center, false);
      continue;
    }
    m.mfill.push_back(m_fill);
    m.pfill.push_back(rho_fill);
    mass_center = add(mass_center, scl(center, mass));
    place(m.M_struc, mass, Ixx, Iyy, Izz, m.R, center, true);
  }
  // end caps and bulkheads (raft/raft_member.py:553-700)
  const int nc = (int)m.cap_st.size();
  if (nc > 0 && !m.circ) {
    err = "RectangularFrustumMOI() missing 2 required positional arguments: 'H' and 'p'";
    return false;
  }
  std::vector<double> dd(nc > 0 ? n : 0);
  for (int i = 0; i < (int)dd.size(); ++i) dd[i] = m.d[i] - 2 * m.t[i];
  auto interp = [&](double x) { return np_interp(x, m.st.data(), dd.data(), n); };
  for (int i = 0; i < nc; ++i) {
    const double L = m.cap_st[i], h = m.cap_t[i], rho_cap = m.rho_shell, hole = m.cap_d[i];
    double dA, dB, dAi, dBi;
    if (L == m.st[0]) {
      dA = dd[0];
      dB = interp(L + h);
      dAi = hole;
      dBi = dB * (dAi / dA);
    } else if (L == m.st[n - 1]) {
      dA = interp(L - h);
      dB = dd[n - 1];
      dBi = hole;
      dAi = dA * (dBi / dB);
    } else if ((m.st[0] < L && L < m.st[0] + h) || (m.st[n - 1] - h < L && L < m.st[n - 1])) {
      err = "This setup cannot be handled by getIneria yet";
      return false;
    } else if (i < nc - 1 && L == m.cap_st[i + 1]) {
      dA = interp(L - h);
      dB = dd[i];
      dBi = hole;
      dAi = dA * (dBi / dB);
    } else if (i > 0 && L == m.cap_st[i - 1]) {
      dA = dd[i];
      dB = interp(L + h);
      dAi = hole;
      dBi = dB * (dAi / dA);
    } else {
      const double dM = interp(L);
      dA = interp(L - h / 2);
      dB = interp(L + h / 2);
      dAi = dA * (hole / dM);
      dBi = dB * (hole / dM);
    }
    double V_o, hco, V_i, hci;
    frustum_vcv(true, dA, dA, dB, dB, h, V_o, hco);
    frustum_vcv(true, dAi, dAi, dBi, dBi, h, V_i, hci);
    const double m_cap = (V_o - V_i) * rho_cap;
    const double hc_cap = (hco * V_o - hci * V_i) / (V_o - V_i);
    double Ir_o, Ia_o, Ir_i, Ia_i;
    frustum_moi(dA, dB, h, rho_cap, Ir_o, Ia_o);
    frustum_moi(dAi, dBi, h, rho_cap, Ir_i, Ia_i);
    Ixx = Iyy = (Ir_o - Ir_i) - m_cap * (hc_cap * hc_cap);
    Izz = Ia_o - Ia_i;
    const V3 pos = sub(add(m.rA, scl(m.q, L)), rPRP);
    V3 cc;
    if (L == m.st[0]) cc = add(pos, scl(m.q, hc_cap));
    else if (L == m.st[n - 1]) cc = sub(pos, scl(m.q, h - hc_cap));
    else cc = sub(pos, scl(m.q, (h / 2) - hc_cap));
    mass_center = add(mass_center, scl(cc, m_cap));
    place(m.M_struc, m_cap, Ixx, Iyy, Izz, m.R, cc, false);
  }
  mass_out = m.M_struc.a[0][0];
  center_out = scl(mass_center, 1.0);
  for (int k = 0; k < 3; ++k) center_out[k] = mass_center[k] / mass_out;
  return true;
}

inline double lin(double x, double xA, double xB, double yA, double yB) { return yA + (x - xA) * (yB - yA) / (xB - xA); }

// raft/statics.py member_hydrostatics (raft/raft_member.py:712-874): this member's C_hydro
inline M6 member_hydrostatics(const Member& m, const V3& rPRP, double rho, double g) {
  M6 Cmat = zero6();
  const V3 rHS = v3(rPRP[0], rPRP[1], 0.0);
  const int n = (int)m.st.size();
  for (int i = 1; i < n; ++i) {
    const V3 rA = sub(add(m.rA, scl(m.q, m.st[i - 1])), rHS);
    const V3 rB = sub(add(m.rA, scl(m.q, m.st[i])), rHS);
    if (rA[2] * rB[2] <= 0) {
      const double phi = std::atan2(std::sqrt(m.q[0] * m.q[0] + m.q[1] * m.q[1]), m.q[2]);
      const double cphi = std::cos(phi);
      const double xWP = lin(0, rA[2], rB[2], rA[0], rB[0]);
      const double yWP = lin(0, rA[2], rB[2], rA[1], rB[1]);
      double AWP, IxWP, IyWP;
      if (m.circ) {
        const double dWP = lin(0, rA[2], rB[2], m.d[i], m.d[i - 1]);
        AWP = (kPi / 4) * (dWP * dWP);
        IxWP = IyWP = (kPi / 64) * std::pow(dWP, 4.0);
      } else {
        const double s0 = lin(0, rA[2], rB[2], m.sl0[i], m.sl0[i - 1]);
        const double s1 = lin(0, rA[2], rB[2], m.sl1[i], m.sl1[i - 1]);
        AWP = s0 * s1;
        M3 Il = zero3();
        Il.a[0][0] = (1.0 / 12) * s0 * std::pow(s1, 3.0);
        Il.a[1][1] = (1.0 / 12) * std::pow(s0, 3.0) * s1;
        const M3 T = tr(m.R);
        const M3 Irot = mm(mm(tr(T), Il), T);
        IxWP = Irot.a[0][0];
        IyWP = Irot.a[1][1];
      }
      const double LWP = std::fabs(rA[2] / cphi);
      double V_i, hc;
      if (m.circ) {
        const double dWP = lin(0, rA[2], rB[2], m.d[i], m.d[i - 1]);
        frustum_vcv(true, m.d[i - 1], m.d[i - 1], dWP, dWP, LWP, V_i, hc);
      } else {
        const double s0 = lin(0, rA[2], rB[2], m.sl0[i], m.sl0[i - 1]);
        const double s1 = lin(0, rA[2], rB[2], m.sl1[i], m.sl1[i - 1]);
        frustum_vcv(false, m.sl0[i - 1], m.sl1[i - 1], s0, s1, LWP, V_i, hc);
      }
      const V3 rc = add(rA, scl(m.q, hc));
      const double rg = rho * g;
      Cmat.a[2][2] += rg * AWP / cphi;
      Cmat.a[2][3] += rg * (-AWP * yWP);
      Cmat.a[2][4] += rg * (AWP * xWP);
      Cmat.a[3][2] += rg * (-AWP * yWP);
      Cmat.a[3][3] += rg * (IxWP + AWP * (yWP * yWP));
      Cmat.a[3][4] += rg * (AWP * xWP * yWP);
      Cmat.a[4][2] += rg * (AWP * xWP);
      Cmat.a[4][3] += rg * (AWP * xWP * yWP);
      Cmat.a[4][4] += rg * (IyWP + AWP * (xWP * xWP));
      Cmat.a[3][3] += rg * V_i * rc[2];
      Cmat.a[4][4] += rg * V_i * rc[2];
    } else if (rA[2] <= 0 && rB[2] <= 0) {
      const double lseg = m.st[i] - m.st[i - 1];
      double V_i, hc;
      if (m.circ) frustum_vcv(true, m.d[i - 1], m.d[i - 1], m.d[i], m.d[i], lseg, V_i, hc);
      else frustum_vcv(false, m.sl0[i - 1], m.sl1[i - 1], m.sl0[i], m.sl1[i], lseg, V_i, hc);
      const V3 rc = add(rA, scl(m.q, hc));
      Cmat.a[3][3] += rho * g * V_i * rc[2];
      Cmat.a[4][4] += rho * g * V_i * rc[2];
    }
  }
  return Cmat;
}

struct Rotor {
  double mRNA, IxRNA, IrRNA, xCG, overhang, tilt, toe;
  int yaw_mode;
  V3 r_rel;
};

// ------------------------------------------------------------------------------ design
struct Result {
  int ok = 0;
  std::string err;
  int nn = 0, nm = 0;
  std::vector<double> packed;   // w, k, node [NF][max(nn,1)], memb [MF][max(nm,1)], M, B, C
  std::vector<int> mstart;
  double statics[5 * 36] = {};  // M_struc, B_struc, C_struc, C_hydro, A_hydro_morison
  std::vector<double> imat;     // [nn][9][nw] complex (re, im) when a node is MacCamy-Fuchs, else empty
};

struct Reader {
  const double* p;
  const double* end;
  bool bad = false;
  double get() {
    if (p >= end) {
      bad = true;
      return 0.0;
    }
    return *p++;
  }
  // an element count: an integer in [0, what is left of the record] (a malformed record would
  // otherwise size vectors from arbitrary doubles)
  int count() {
    const double v = get();
    if (!(v >= 0.0) || v > (double)(end - p) || v != (double)(long long)v) {
      bad = true;
      return 0;
    }
    return (int)v;
  }
  void vec(std::vector<double>& v, int n) {
    v.resize(n > 0 ? n : 0);
    for (int i = 0; i < n; ++i) v[i] = get();
  }
};

// One design: parse the spec, build the members (heading copies), statics, added mass and
// the packed device tables.
inline void prep_one(const double* spec, long long len, int nw, const double* w, const double* k, Result& out) {
  Reader rd{spec, spec + len};
  if ((int)rd.get() != kMagic) {
    out.err = "rh_prep_designs: bad spec record (magic)";
    return;
  }
  const int nmemb = rd.count(), nrot = rd.count();
  if (rd.bad) {
    out.err = "rh_prep_designs: bad spec record (member / rotor counts)";
    return;
  }
  const double rho = rd.get(), g = rd.get();
  double r6[6];
  for (double& x : r6) x = rd.get();
  int given[5];
  for (int& x : given) x = (int)rd.get();
  M6 gm[5];
  for (int b = 0; b < 5; ++b) {
    gm[b] = zero6();
    if (given[b])
      for (int e = 0; e < 36; ++e) gm[b].a[e / 6][e % 6] = rd.get();
  }
  std::vector<Member> mems;
  mems.reserve((size_t)nmemb * 4);   // (a Member is some thirty vectors: growing the array moves them all)
  for (int im = 0; im < nmemb; ++im) {
    Member b;
    b.type = (int)rd.get();
    b.circ = (int)rd.get();
    b.potMod = (int)rd.get();
    b.mcf = (int)rd.get();
    b.nacelle = (int)rd.get();
    const int nst = rd.count(), ncap = rd.count(), nhead = rd.count();
    if (rd.bad) {
      out.err = "rh_prep_designs: bad spec record (station / cap / heading counts)";
      return;
    }
    b.has_t = (int)rd.get();
    const double gamma0 = rd.get();
    b.dlsMax = rd.get();
    b.rho_shell = rd.get();
    V3 rA0, rB0;
    for (int i = 0; i < 3; ++i) rA0[i] = rd.get();
    for (int i = 0; i < 3; ++i) rB0[i] = rd.get();
    std::vector<double> heads, st;
    rd.vec(heads, nhead);
    rd.vec(st, nst);
    if (b.circ) rd.vec(b.d, nst);
    else {
      b.sl0.resize(nst);
      b.sl1.resize(nst);
      for (int i = 0; i < nst; ++i) {
        b.sl0[i] = rd.get();
        b.sl1[i] = rd.get();
      }
    }
    if (b.has_t) rd.vec(b.t, nst);
    std::vector<double> lfill;
    rd.vec(lfill, nst - 1);
    rd.vec(b.rho_fill, nst - 1);
    rd.vec(b.cdq, nst);
    rd.vec(b.cdp1, nst);
    rd.vec(b.cdp2, nst);
    rd.vec(b.cdend, nst);
    rd.vec(b.caq, nst);
    rd.vec(b.cap1, nst);
    rd.vec(b.cap2, nst);
    rd.vec(b.caend, nst);
    std::vector<double> capst;
    rd.vec(capst, ncap);
    rd.vec(b.cap_t, ncap);
    rd.vec(b.cap_d, ncap);
    if (rd.bad) break;
    if (b.mcf && !b.circ) b.mcf = 0;   // (raft/member.py: MCF applies to circular members only)
    if (nst < 2) {
      out.err = "At least two stations entries must be provided";
      return;
    }
    // raft/member.py __init__ (raft/raft_member.py:23-96), once per heading copy
    if ((rA0[2] == 0 || rB0[2] == 0) && b.type != 3) {
      out.err = "RAFT Members cannot start or end on the waterplane";
      return;
    }
    if (rB0[2] < rA0[2]) std::swap(rA0, rB0);
    const V3 rAB = sub(rB0, rA0);
    b.l = std::sqrt(dot(rAB, rAB));
    const double span = st[nst - 1] - st[0];
    b.st.resize(nst);
    for (int i = 0; i < nst; ++i) b.st[i] = (st[i] - st[0]) / span * b.l;
    b.l_fill.resize(nst - 1);
    for (int i = 0; i < nst - 1; ++i) b.l_fill[i] = lfill[i] / span * b.l;
    b.cap_st.resize(ncap);
    for (int i = 0; i < ncap; ++i) b.cap_st[i] = (capst[i] - st[0]) / span * b.l;
    for (int ih = 0; ih < nhead; ++ih) {
      Member c = b;
      const double hd = heads[ih];
      c.gamma = gamma0;
      c.rA0 = rA0;
      c.rB0 = rB0;
      if (hd != 0.0) {
        const double cs = std::cos(hd * (kPi / 180.0)), sn = std::sin(hd * (kPi / 180.0));
        const M3 rot{{{cs, -sn, 0}, {sn, cs, 0}, {0, 0, 1}}};
        c.rA0 = mv(rot, rA0);
        c.rB0 = mv(rot, rB0);
        if (rAB[0] == 0.0 && rAB[1] == 0) c.gamma += hd;
      }
      if (c.circ) c.gamma = 0;
      c.discretise();
      mems.push_back(std::move(c));
    }
  }
  std::vector<Rotor> rots(nrot);
  for (auto& ro : rots) {
    ro.mRNA = rd.get();
    ro.IxRNA = rd.get();
    ro.IrRNA = rd.get();
    ro.xCG = rd.get();
    ro.overhang = rd.get();
    ro.tilt = rd.get();
    ro.toe = rd.get();
    ro.yaw_mode = (int)rd.get();
    for (int i = 0; i < 3; ++i) ro.r_rel[i] = rd.get();
    const int has_hub = (int)rd.get();
    const double hHub = rd.get();
    if (has_hub) {   // raft/statics.py RNA.__init__: q = rotation_matrix(0, tilt, toe) x
      const V3 qh = mv(rotation_matrix(0, ro.tilt, ro.toe), v3(1.0, 0.0, 0.0));
      ro.r_rel[2] = hHub - qh[2] * ro.overhang;
    }
  }
  if (rd.bad || rd.p != rd.end) {
    out.err = "rh_prep_designs: spec record length does not match its content";
    return;
  }
  const V3 rP = v3(r6[0], r6[1], r6[2]);
  for (auto& m : mems) m.set_position(r6);

  // statics (raft/statics.py fowt_statics): computed unless a full set is given
  M6 M_struc = zero6(), C_struc = zero6(), C_hydro = zero6();
  const bool full = given[0] && given[2] && given[3];
  bool need_t = !full;
  for (auto& m : mems)
    if (!m.nacelle && !m.has_t && need_t) {
      out.err = "Key 't' not found in input file...";
      return;
    }
  if (!full) {
    V3 m_center_sum{};
    for (auto& m : mems) {
      if (m.nacelle) continue;
      double mass;
      V3 center;
      if (!member_inertia(m, rP, mass, center, out.err)) return;
      acc6(M_struc, m.M_struc);
      m_center_sum = add(m_center_sum, scl(center, mass));
      acc6(C_hydro, member_hydrostatics(m, rP, rho, g));
    }
    for (auto& m : mems)
      if (m.nacelle) acc6(C_hydro, member_hydrostatics(m, rP, rho, g));
    const M3 Rp = rotation_matrix(r6[3], r6[4], r6[5]);
    for (auto& ro : rots) {   // raft/statics.py RNA.setPosition (raft/raft_rotor.py:376-458)
      double yaw;
      const double heading = r6[5];
      switch (ro.yaw_mode) {
        case 0: yaw = 0.0 - heading + 0.0; break;
        case 1: yaw = 0.0 - heading; break;
        case 2: yaw = 0.0; break;
        case 3: yaw = 0.0 - heading; break;
        default: out.err = "Unsupported yaw_mode value. Must be 0, 1, or 2."; return;
      }
      const M3 Rq_rel = rotation_matrix(0, ro.tilt, ro.toe + yaw);
      const M3 Rq = mm(Rq_rel, Rp);
      const V3 qv = mv(Rp, mv(Rq_rel, v3(1.0, 0.0, 0.0)));
      const V3 r_rrp = mv(Rp, ro.r_rel);
      const V3 r_cg = add(r_rrp, scl(qv, ro.xCG));
      // rotateMatrix6 of diag(m, m, m, Ix, Ir, Ir): R M R^T per 3x3 block
      M3 Md = zero3(), Id = zero3();
      Md.a[0][0] = Md.a[1][1] = Md.a[2][2] = ro.mRNA;
      Id.a[0][0] = ro.IxRNA;
      Id.a[1][1] = Id.a[2][2] = ro.IrRNA;
      const M3 A = mm(mm(Rq, Md), tr(Rq)), D = mm(mm(Rq, Id), tr(Rq)), Z = mm(mm(Rq, zero3()), tr(Rq));
      M6 Mm = zero6();
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          Mm.a[i][j] = A.a[i][j];
          Mm.a[i][3 + j] = Z.a[i][j];
          Mm.a[3 + j][i] = Z.a[i][j];
          Mm.a[3 + i][3 + j] = D.a[i][j];
        }
      acc6(M_struc, translate_6to6(Mm, r_cg));
      m_center_sum = add(m_center_sum, scl(r_cg, ro.mRNA));
    }
    const double m_all = M_struc.a[0][0];
    const double zcg = m_center_sum[2] / m_all;
    C_struc.a[3][3] = C_struc.a[4][4] = -m_all * g * zcg;
  }
  if (given[0]) M_struc = gm[0];
  const M6 B_struc = given[1] ? gm[1] : zero6();
  if (given[2]) C_struc = gm[2];
  if (given[3]) C_hydro = gm[3];
  const M6 C_moor = given[4] ? gm[4] : zero6();

  // added mass and inertial excitation (raft/fowt.py calcHydroConstants)
  M6 A_hydro = zero6();
  for (auto& m : mems) acc6(A_hydro, m.hydro_constants(rP, rho, k, nw));

  // tables (raft/prep.py node_table / linear_matrices / host_tables)
  constexpr int NF = RH_NF_COUNT, MF = RH_MF_COUNT;
  std::vector<double> cols;               // node rows of NF fields, back to back
  std::vector<std::vector<double>> mcols;
  std::vector<const double*> mcf_blocks;   // per node: its [9][nw] complex block, or NULL
  out.mstart = {0};
  for (auto& m : mems) {
    int nsub = 0;
    for (int il = 0; il < m.ns; ++il) nsub += m.r[il][2] < 0;
    if (nsub) {
      const V3 rA = sub(m.rA, rP);
      const V3 cq = cross(rA, m.q), c1 = cross(rA, m.p1), c2 = cross(rA, m.p2);
      mcols.push_back({m.q[0], m.q[1], m.q[2], cq[0], cq[1], cq[2], m.p1[0], m.p1[1], m.p1[2], c1[0], c1[1], c1[2],
                       m.p2[0], m.p2[1], m.p2[2], c2[0], c2[1], c2[2], dot(m.q, m.q), dot(m.p1, m.p1),
                       dot(m.p2, m.p2)});
      out.mstart.push_back(out.mstart.back() + nsub);
    }
    for (int il = 0; il < m.ns; ++il) {
      if (!(m.r[il][2] < 0)) continue;
      const double dls = m.dls[il];
      double aq, ap1, ap2, aend;
      if (m.circ) {
        aq = kPi * m.ds0[il] * dls;
        ap1 = ap2 = m.ds0[il] * dls;
        aend = std::fabs(kPi * m.ds0[il] * m.drs0[il]);
      } else {
        aq = 2 * (m.ds0[il] + m.ds0[il]) * dls;
        ap1 = m.ds0[il] * dls;
        ap2 = m.ds1[il] * dls;
        aend = std::fabs((m.ds0[il] + m.drs0[il]) * (m.ds1[il] + m.drs1[il]) -
                         (m.ds0[il] - m.drs0[il]) * (m.ds1[il] - m.drs1[il]));
      }
      const V3& r = m.r[il];
      const V3 rr = sub(r, rP);
      const double c[] = {r[0], r[1], r[2], rr[0], rr[1], rr[2], m.q[0], m.q[1], m.q[2], m.p1[0], m.p1[1],
                          m.p1[2], m.p2[0], m.p2[1], m.p2[2], aq, ap1, ap2, aend, m.coef(m.cdq, il),
                          m.coef(m.cdp1, il), m.coef(m.cdp2, il), m.coef(m.cdend, il), m.circ ? 1.0 : 0.0,
                          m.a_i[il], m.mcf ? 1.0 : 0.0};
      static_assert(sizeof(c) / sizeof(double) + 10 == NF, "node table fields");
      mcf_blocks.push_back(m.mcf ? m.imat_mcf.data() + (size_t)il * 9 * nw * 2 : nullptr);
      cols.insert(cols.end(), c, c + sizeof(c) / sizeof(double));
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) cols.push_back(m.Imat[il].a[i][j]);
      cols.push_back(m.ls[il]);
    }
  }
  const int nn = (int)(cols.size() / NF), nm = (int)mcols.size();
  const int nnc = nn ? nn : 1, nmc = nm ? nm : 1;
  out.nn = nn;
  out.nm = nm;
  bool any_mcf = false;
  for (const double* blk : mcf_blocks) any_mcf |= blk != nullptr;
  if (any_mcf) {   // (raft/prep.py node_table: zeros for the other nodes)
    out.imat.assign((size_t)nn * 9 * nw * 2, 0.0);
    for (int n = 0; n < nn; ++n)
      if (mcf_blocks[n]) std::copy(mcf_blocks[n], mcf_blocks[n] + (size_t)9 * nw * 2, out.imat.data() + (size_t)n * 9 * nw * 2);
  }
  out.packed.assign((size_t)2 * nw + (size_t)NF * nnc + (size_t)MF * nmc + 3 * 36, 0.0);
  double* P = out.packed.data();
  std::copy(w, w + nw, P);
  std::copy(k, k + nw, P + nw);
  double* T = P + 2 * nw;
  for (int n = 0; n < nn; ++n)
    for (int f = 0; f < NF; ++f) T[(size_t)f * nnc + n] = cols[(size_t)n * NF + f];
  double* Mt = T + (size_t)NF * nnc;
  for (int j = 0; j < nm; ++j)
    for (int f = 0; f < MF; ++f) Mt[(size_t)f * nmc + j] = mcols[j][f];
  double* MBC = Mt + (size_t)MF * nmc;
  for (int e = 0; e < 36; ++e) {
    const int i = e / 6, j = e % 6;
    MBC[e] = M_struc.a[i][j] + A_hydro.a[i][j];                               // M_lin (raft/raft_model.py:911)
    MBC[36 + e] = B_struc.a[i][j] + 0.0;                                       // B_lin: B_struc + B_gyro (zero)
    MBC[72 + e] = (C_struc.a[i][j] + C_moor.a[i][j]) + C_hydro.a[i][j];        // C_lin (:913)
    out.statics[e] = M_struc.a[i][j];
    out.statics[36 + e] = B_struc.a[i][j];
    out.statics[72 + e] = C_struc.a[i][j];
    out.statics[108 + e] = C_hydro.a[i][j];
    out.statics[144 + e] = A_hydro.a[i][j];
  }
  out.ok = 1;
}

}  // namespace rhp

struct rh_prep {
  std::vector<rhp::Result> res;
  std::vector<long long> off;     // per design: offset of its packed tables in `all`
  std::vector<long long> moff;    // ... of its member ranges in `mst`
  std::vector<double> all;
  std::vector<int> mst;
};
